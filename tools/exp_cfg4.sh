#!/bin/bash
# Config-4 (or $CFG) timing of experiment builds (ab_libs/lib<TAG>.so; results may be
# wrong by design, so the bench's round-trip exit code is ignored).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/exp4
for r in 1 2; do for t in "$@"; do
NP_LIB_PATH=$PWD/ab_libs/lib$t.so timeout -k 10 120 python bench.py --config ${CFG:-4} --no-cpu --steps ${STEPS:-10} --warmup 2 > gpurun_out/exp4/$t$r.log 2>&1
[ $? -ge 124 ] && exit 1
python3 -c "
import json,sys
d=json.loads(open('gpurun_out/exp4/$t$r.log').read().strip().split('\n')[-1])
print('$t', $r, d['value'], {k:v['ms'] for k,v in d['kernels'].items()}, d['roundtrip_ok'])"
done; done
