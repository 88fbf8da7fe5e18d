#!/bin/bash
# GPU tests, then config 2 (k = 64) and 700 validators (k = 128) against tools/exp/lib_head.so (GPU box).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
ARGS="--config 2" TAG=c2_ bash tools/exp_one.sh head base head base || exit 1
ARGS="--n-wanted 700 --erase 234" TAG=v700_ bash tools/exp_one.sh head base || exit 1
ARGS="--n-wanted 300 --erase 100" TAG=v300_ bash tools/exp_one.sh head base || exit 1
