#!/bin/bash
# Config-4 phase-removal timings (tools/exp/lib_x*.so; wrong output by design)
# and the config-4 PMC / kernel-trace record of the product build.
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
ARGS="--config 4" TAG=c4_ bash tools/exp_one.sh base skip x1 x256 x512 x1024 x2 base skip || exit 1
bash tools/profile_round.sh r03c_cfg4 4
