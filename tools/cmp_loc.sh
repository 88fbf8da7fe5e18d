#!/bin/bash
# GPU tests + headline A/B against tools/exp/lib_head.so with kernel-trace stats of both (GPU box).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/loc; export TMPDIR=/tmp
bash tools/gpu_check_quick.sh || exit 1
for n in head base; do
  lib=$PWD/tools/exp/lib_$n.so; [ $n = base ] && lib=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
  NP_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/loc/$n --output-format csv -- python3 bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/loc/$n.log 2>&1 || exit 1
  f=$(ls gpurun_out/loc/$n/*/*_kernel_stats.csv | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'np::' in r['Name']: print('$n', r['Name'].split('<')[0].split('::')[-1], r['Name'].split('<')[1].split('>')[0], round(float(r['AverageNs'])/1e3,1))"
done
