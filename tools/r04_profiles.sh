#!/bin/bash
# Round-4 profiles: kernel-trace stats and PMC passes for configs 3, 2 and 4.
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/profile_round.sh r04 3 > gpurun_out/prof_r04.log 2>&1 || { tail -20 gpurun_out/prof_r04.log; exit 1; }
bash tools/profile_round.sh r04_cfg2 2 > gpurun_out/prof_r04_cfg2.log 2>&1 || { tail -20 gpurun_out/prof_r04_cfg2.log; exit 1; }
bash tools/profile_round.sh r04_cfg4 4 > gpurun_out/prof_r04_cfg4.log 2>&1 || { tail -20 gpurun_out/prof_r04_cfg4.log; exit 1; }
echo profiles done
