#!/bin/bash
# Round record on the GPU box: the default bench line, config 2/4 bench lines,
# then tools/profile_round.sh for configs 3, 2 and 4.  Usage: round_final.sh TAG
set -o pipefail
TAG=${1:-r02}
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
timeout -k 10 300 python bench.py > gpurun_out/final/bench.log 2>&1 || exit $?
tail -1 gpurun_out/final/bench.log
for c in 2 4; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/final/bench_cfg$c.log 2>&1 || exit $?; tail -1 gpurun_out/final/bench_cfg$c.log; done
bash tools/profile_round.sh $TAG 3 && bash tools/profile_round.sh ${TAG}_cfg2 2 && bash tools/profile_round.sh ${TAG}_cfg4 4
