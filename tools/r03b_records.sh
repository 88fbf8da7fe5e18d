#!/bin/bash
# Round-3 records of the k = 512 resident kernels and the unaligned-row paths
# (DESIGN §4.9, §6): bench lines written to gpurun_out/r03b/*.json.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r03b
run() { tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 --out gpurun_out/r03b/$tag.json "$@" > gpurun_out/r03b/$tag.log 2>&1 || { tail -5 gpurun_out/r03b/$tag.log; exit 1; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r03b/$tag.json'))
c=d['config']; print('$tag', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
}
run shapes_vc1600 --n-wanted 1600 --batch 1024 --erase 534 &&
run shapes_vc2000 --n-wanted 2000 --batch 1024 --erase 667 &&
run shapes_vc2500 --n-wanted 2500 --batch 512 --erase 834 &&
run shapes_vc3000 --n-wanted 3000 --batch 512 --erase 1000 &&
run refbench_vc2000_10MB --n-wanted 2000 --batch 100 --payload 10000000 --erase 667 &&
run odd_c3_1000000 --payload 1000000 &&
run odd_c3_1000001 --payload 1000001 &&
run odd_vc100_1000003 --n-wanted 100 --batch 1024 --payload 1000003 --erase 34
