#!/bin/bash
# GPU suite on the in-tree build, then A/B of ab_libs/libB.so and libC.so on
# the sub-transform path (16,384, 30,000 and 65,536 validators, 1 MiB x 512).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
for vc in 16384 30000 65536; do
  BENCH_ARGS="--n-wanted $vc --batch 512 --erase $(( (vc - 1) / 3 + 1 ))" ROUNDS=2 bash tools/ab_libs.sh ab_libs/libB.so ab_libs/libC.so || exit 1
done
