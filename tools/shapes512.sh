cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s512
run() { # tag env args
  tag=$1; shift
  timeout -k 10 300 env "$@" > gpurun_out/s512/$tag.log 2>&1 || { tail -5 gpurun_out/s512/$tag.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('gpurun_out/s512/$tag.log').read().strip().split('\n')[-1])
c=d['config']; print('$tag', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:(v['ms'], v['frac'], round(v['traffic']/v['algorithmic_bytes'],2) if v.get('traffic') else None) for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
}
B="python bench.py --no-cpu --steps 5 --warmup 2"
run vc2000 NP_X=1 $B --n-wanted 2000 --batch 1024 --erase 667 &&
run vc2000_big NP_RES=0 $B --n-wanted 2000 --batch 1024 --erase 667 &&
run vc1600 NP_X=1 $B --n-wanted 1600 --batch 1024 --erase 534 &&
run vc2500 NP_X=1 $B --n-wanted 2500 --batch 512 --erase 834 &&
run vc3000 NP_X=1 $B --n-wanted 3000 --batch 512 --erase 1000 &&
run vc3000_big NP_RES=0 $B --n-wanted 3000 --batch 512 --erase 1000 &&
run vc2000_10MB NP_X=1 $B --n-wanted 2000 --batch 100 --payload 10000000 --erase 667 &&
run vc2000_10MB_big NP_RES=0 $B --n-wanted 2000 --batch 100 --payload 10000000 --erase 667
