#!/bin/bash
# Round records on the GPU box: the BASELINE bench lines (configs 3, 2, 4, each
# with the reference CPU path timed beside it), config 1 on the CPU alone
# (oracle/_ref/cpu_bench_ref: the reference's cxx/RSErasureCode.c + crate
# glue, config 1 = n16 k8, 4 KiB payloads), and shapes outside the configs
# (validator counts 2 .. 12,000, the reference bench's 10 MB payloads) into
# gpurun_out/<TAG>/*.json.  Usage: tools/records.sh TAG [VCS="..."]
set -o pipefail
TAG=${1:-r04}
cd $GRAFT_REPO_ROOT
D=gpurun_out/$TAG
mkdir -p $D
timeout -k 10 300 python bench.py --out $D/bench.json > $D/bench.log 2>&1 || exit $?
for c in 2 4; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --cpu-seconds 8 --out $D/cfg$c.json > $D/cfg$c.log 2>&1 || exit $?; done
for f in bench cfg2 cfg4; do python3 -c "
import json; d=json.load(open('$D/$f.json')); print('$f', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, 'cpu', d.get('cpu_baseline', {}).get('value'))"; done
if [ -x oracle/_ref/cpu_bench_ref ]; then exe=oracle/_ref/cpu_bench_ref; else exe=oracle/cpu_bench_port; fi
timeout -k 10 120 $exe 16 8 4096 8 1 5 > $D/cfg1_cpu.json || exit $?
cat $D/cfg1_cpu.json
run() { tag=$1; shift
  timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 --out $D/$tag.json "$@" > $D/$tag.log 2>&1 || { tail -5 $D/$tag.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$D/$tag.json'))
c=d['config']; print('$tag', 'n', c['n'], 'k', c['k'], 'GiB/s', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, 'ok', d['roundtrip_ok'])"
}
for vc in ${VCS:-2 3 6 10 20 40 100 300 700 1200 1600 2000 2500 3000 5000 7000 10000 16384 20000 30000 40000 50000 65536}; do
  b=1024; [ $vc -gt 2048 ] && b=512
  run shapes_vc$vc --n-wanted $vc --batch $b --erase $(( (vc - 1) / 3 + 1 )) || exit 1
done
run refbench_vc2000_10MB --n-wanted 2000 --batch 100 --payload 10000000 --erase 667
