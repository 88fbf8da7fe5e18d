#!/bin/bash
# Round-4 probe 6: GPU tests with the next-tile row prefetch (NP_REC_TILE_PREFETCH=1
# in the product), A/B against tpf0 at config 3 and at 1200 validators (8 segments).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu6.log 2>&1; rc=$?
tail -3 gpurun_out/r04/pytest_gpu6.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu6.log | head -20; exit $rc; fi
TAG=p6_ bash tools/exp_one.sh base tpf0 base tpf0 || exit $?
TAG=p6v1200_ ARGS="--n-wanted 1200 --batch 1024 --erase 400" bash tools/exp_one.sh base tpf0 base tpf0 || exit $?
