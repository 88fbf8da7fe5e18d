#!/bin/bash
# GPU tests, then the product against tools/exp/lib_head.so on configs 3, 4 and
# the small (100 validators) and k = 512 (2000 validators) shapes (GPU box).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
bash tools/exp_one.sh head base head base || exit 1
ARGS="--config 4" TAG=c4_ bash tools/exp_one.sh head base || exit 1
ARGS="--n-wanted 100 --erase 34" TAG=v100_ bash tools/exp_one.sh head base || exit 1
ARGS="--n-wanted 2000 --erase 667" TAG=v2000_ bash tools/exp_one.sh head base || exit 1
