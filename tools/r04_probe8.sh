#!/bin/bash
# Round-4 probe 8: GPU tests with the encode's fused tower -> Cantor conversion
# (NP_ENC_CONV=1 in the product), A/B against conv0 at configs 3 and 2.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu8.log 2>&1; rc=$?
tail -3 gpurun_out/r04/pytest_gpu8.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu8.log | head -20; exit $rc; fi
TAG=p8_ bash tools/exp_one.sh base conv0 base conv0 || exit $?
TAG=p8c2_ ARGS="--config 2" bash tools/exp_one.sh base conv0 || exit $?
TAG=p8v700_ ARGS="--n-wanted 700 --batch 1024 --erase 234" bash tools/exp_one.sh base conv0 || exit $?
