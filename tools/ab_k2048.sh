#!/bin/bash
# k = 2048 (6,144-12,288 validators): big kernels (default) vs the sub-transform
# path (NP_HUGE=2), 1 MiB x 512.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/k2048
for vc in 7000 8000 10000 12000; do for m in 0x 1; do
  env $( [ $m = 0x ] || echo NP_HUGE=$m ) timeout -k 10 200 python bench.py --no-cpu --steps 5 --warmup 2 --batch 512 --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/k2048/vc${vc}_$m.log 2>&1 || exit 1
  python3 -c "
import json; d=json.loads(open('gpurun_out/k2048/vc${vc}_$m.log').read().strip().split('\n')[-1])
c=d['config']; print('vc$vc NP_HUGE=$m', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:v['ms'] for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
done; done
