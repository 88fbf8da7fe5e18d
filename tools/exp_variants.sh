#!/bin/bash
# Experiment builds of the library with phases of the fast kernels disabled
# (NP_EXP bits, fast_common.hpp), for timing phases apart.  CPU side: builds
# tools/exp/lib_<bits>.so.  GPU side (--run): times encode / reconstruct of each.
set -e
cd "$(dirname "$0")/.."
if [ "$1" != "--run" ]; then
  for b in ${BITS:-1 2 3 4 6 8 16 32 56 57 64}; do
    make -s -j8 -C reed-solomon-novelpoly_amd OUT=$PWD/tools/exp/lib_$b.so OBJDIR=$PWD/tools/exp/build_$b EXTRA=-DNP_EXP=$b 2>&1 | grep -i error || true
  done
  exit 0
fi
for b in ${RUNBITS:-0 1 2 3 4 6 8 16 32 56 57}; do
  lib=$PWD/tools/exp/lib_$b.so
  [ $b = 0 ] && lib=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
  NP_LIB_PATH=$lib timeout -k 10 120 python bench.py --no-cpu --steps 5 --warmup 2 > gpurun_out/exp_$b.log 2>&1 || true
  python3 -c "
import json,sys
d=json.loads(open('gpurun_out/exp_$b.log').read().strip().split('\n')[-1])
print('NP_EXP=$b', {k:v['ms'] for k,v in d['kernels'].items()})" || tail -3 gpurun_out/exp_$b.log
done
