#!/bin/bash
# Round-4 probe 10: k = 2048 (6,144-12,288 validators) on the big kernels
# (default) against the size-1024 sub-transform kernels (NP_HUGE=1).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp
for vc in 6144 7000 10000 12000; do
  for h in def 1; do
    if [ $h = 1 ]; then export NP_HUGE=1; else unset NP_HUGE; fi
    timeout -k 10 180 python bench.py --no-cpu --steps 10 --warmup 2 --n-wanted $vc --batch 512 --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/exp/p10_${vc}_$h.log 2>&1 || { tail -3 gpurun_out/exp/p10_${vc}_$h.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/exp/p10_${vc}_$h.log').read().strip().split('\n')[-1]); c=d['config']; print('p10 vc$vc huge=$h', c['n'], c['k'], d['value'], d['roundtrip_ok'], {k:v['ms'] for k,v in d['kernels'].items()})"
  done
done
