#!/bin/bash
# Throughput of shapes outside the BASELINE configs (DESIGN measurements, not
# the headline): 1 MiB payloads, batch 1024 (512 for n >= 4096), erasures =
# the validator count's recoverability threshold.  Validator counts: 300 (n512
# k64, n/k 8), 700 (n1024 k128, 8), 1200 (n2048 k256, 8), 2000 (n2048 k512,
# 4), 2500 (n4096 k512, 8), 5000 (n8192 k1024, 8), 1024 (config 3 shape,
# reference point).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/shapes
for vc in ${VCS:-1024 300 700 1200 2000 2500 5000}; do
  b=1024; [ $vc -gt 2048 ] && b=512
  timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 --n-wanted $vc --batch $b --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/shapes/vc$vc.log 2>&1 || { tail -5 gpurun_out/shapes/vc$vc.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/shapes/vc$vc.log').read().strip().split('\n')[-1])
c=d['config']; print('vc=$vc', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
done
