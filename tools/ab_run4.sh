#!/bin/bash
# GPU suite on the in-tree build, then A/B of ab_libs/libB.so and libC.so on
# config 4 and the k = 512 / 1024 decode shapes (n/k = 4 and 8).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
CONFIG=4 ROUNDS=2 bash tools/ab_libs.sh ab_libs/libB.so ab_libs/libC.so || exit 1
for a in "2000 1024 667" "3000 512 1000" "5000 512 1667"; do set -- $a
  BENCH_ARGS="--n-wanted $1 --batch $2 --erase $3" ROUNDS=2 bash tools/ab_libs.sh ab_libs/libB.so ab_libs/libC.so || exit 1
done
