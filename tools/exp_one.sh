#!/bin/bash
# Times the headline bench with experiment libraries: tools/exp_one.sh NAME...
# (tools/exp/lib_NAME.so; "base" = the product library).  GPU box only.
# ARGS: extra bench.py arguments (e.g. "--config 2"), TAG: log-name prefix.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/exp
for n in "$@"; do
  lib=$PWD/tools/exp/lib_$n.so; [ $n = base ] && lib=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
  NP_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 2 $ARGS > gpurun_out/exp/$TAG$n.log 2>&1
  rc=$?; [ $rc -eq 0 ] || [ $rc -eq 3 ] || { tail -3 gpurun_out/exp/$TAG$n.log; exit $rc; }  # 3: round trip differs (phase-removal builds)
  python3 -c "
import json; d=json.loads(open('gpurun_out/exp/$TAG$n.log').read().strip().split('\n')[-1]); print('$TAG$n', d['value'], d['roundtrip_ok'], {k:v['ms'] for k,v in d['kernels'].items()})"
done
