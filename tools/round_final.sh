#!/bin/bash
# Round-end record on the GPU box: default 20-step bench (JSON line), config 2/4
# bench lines, then tools/profile_round.sh (kernel-trace stats + PMC passes).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 300 python bench.py > gpurun_out/final/bench.log 2>&1 || exit $?
tail -1 gpurun_out/final/bench.log
for c in 2 4; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/final/bench_cfg$c.log 2>&1 || exit $?; tail -1 gpurun_out/final/bench_cfg$c.log; done
bash tools/profile_round.sh ${1:-r01}
