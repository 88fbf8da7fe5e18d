#!/bin/bash
# Round-4 probe 2: per-wave decode stamps, host-memory e2e (pinned and
# pageable), records.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/wave_stamps.py > gpurun_out/r04/wave_stamps.log 2>&1 || exit $?
cat gpurun_out/r04/wave_stamps.log
for c in 3 4; do timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $([ $c = 3 ] && echo 256 || echo 64) > gpurun_out/r04/e2e_cfg$c.json 2> gpurun_out/r04/e2e_cfg$c.err || { tail -5 gpurun_out/r04/e2e_cfg$c.err; exit 1; }; cat gpurun_out/r04/e2e_cfg$c.json; done
bash tools/records.sh r04a
