#!/bin/bash
# GPU suite on the in-tree build, then A/B of ab_libs/libB.so and libC.so on
# configs 3 and 2 and the 100-validator shape (fast / small decodes).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
CONFIG=3 ROUNDS=3 bash tools/ab_libs.sh ab_libs/libB.so ab_libs/libC.so || exit 1
CONFIG=2 ROUNDS=2 bash tools/ab_libs.sh ab_libs/libB.so ab_libs/libC.so || exit 1
BENCH_ARGS="--n-wanted 100 --batch 1024 --erase 34" ROUNDS=2 bash tools/ab_libs.sh ab_libs/libB.so ab_libs/libC.so
