#!/bin/bash
# GPU tests, then the k = 512 / 1024 / 2048 shapes against tools/exp/lib_head.so (GPU box).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
ARGS="--config 4" TAG=c4_ bash tools/exp_one.sh head base head base || exit 1
ARGS="--n-wanted 2000 --erase 667 --batch 1024" TAG=v2000_ bash tools/exp_one.sh head base || exit 1
ARGS="--n-wanted 7000 --erase 2334 --batch 512" TAG=v7000_ bash tools/exp_one.sh head base || exit 1
