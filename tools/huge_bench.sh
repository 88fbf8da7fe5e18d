#!/bin/bash
# Throughput above 8,192 validators: 1 MiB payloads, batch 256,
# erasures = the recoverability threshold; k = 2048 on the big kernels and on
# the sub-transform path (NP_HUGE=1), k >= 4096 on the sub-transform path.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/huge
run() { tag=$1; shift
  timeout -k 10 300 env "$@" --out gpurun_out/huge/$tag.json > gpurun_out/huge/$tag.log 2>&1 || { tail -5 gpurun_out/huge/$tag.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/huge/$tag.log').read().strip().split('\n')[-1])
c=d['config']; print('$tag', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
}
B="python bench.py --no-cpu --steps 3 --warmup 1 --batch ${BATCH:-256}"
for vc in ${VCS:-10000 16384 20000 30000 40000 65536}; do
  run vc$vc NP_X=1 $B --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) || exit 1
done
[ -n "$NOAB" ] || run vc10000_huge NP_HUGE=1 $B --n-wanted 10000 --erase 3334
