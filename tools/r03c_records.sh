#!/bin/bash
# Round-3 closing records (GPU box): the three BASELINE bench lines (after
# profiles/r03*_pmc_summary.json were refreshed, so their roofline.traffic is
# this build's) and the resident-kernel shapes, written to
# gpurun_out/r03c/*.json.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03c
timeout -k 10 300 python bench.py --out gpurun_out/r03c/bench.json > gpurun_out/r03c/bench.log 2>&1 || exit 1
for c in 2 4; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu --out gpurun_out/r03c/cfg$c.json > gpurun_out/r03c/cfg$c.log 2>&1 || exit 1; done
run() { tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 --out gpurun_out/r03c/$tag.json "$@" > gpurun_out/r03c/$tag.log 2>&1 || { tail -5 gpurun_out/r03c/$tag.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03c/$tag.json'))
c=d['config']; print('$tag', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
}
run shapes_vc1600 --n-wanted 1600 --batch 1024 --erase 534 &&
run shapes_vc2000 --n-wanted 2000 --batch 1024 --erase 667 &&
run shapes_vc2500 --n-wanted 2500 --batch 512 --erase 834 &&
run shapes_vc3000 --n-wanted 3000 --batch 512 --erase 1000 &&
run shapes_vc5000 --n-wanted 5000 --batch 512 --erase 1667 &&
run refbench_vc2000_10MB --n-wanted 2000 --batch 100 --payload 10000000 --erase 667
