#!/bin/bash
# Round-4 probe 5: GPU tests (product and the decode row-DMA variant), decode
# row-DMA A/B at configs 3 and 2, encode HIW-early A/B, pageable pin-in-place e2e.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu5.log 2>&1; rc=$?
tail -3 gpurun_out/r04/pytest_gpu5.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu5.log | head -20; exit $rc; fi
NP_LIB_PATH=$PWD/tools/exp/lib_rowdma.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu5_rowdma.log 2>&1; rc=$?
tail -3 gpurun_out/r04/pytest_gpu5_rowdma.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu5_rowdma.log | head -20; exit $rc; fi
TAG=p5_ bash tools/exp_one.sh base rowdma hiw base rowdma hiw || exit $?
TAG=p5c2_ ARGS="--config 2" bash tools/exp_one.sh base rowdma base rowdma || exit $?
for c in 3 4; do timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $([ $c = 3 ] && echo 256 || echo 64) > gpurun_out/r04/e2e5_cfg$c.json 2> gpurun_out/r04/e2e5_cfg$c.err || { tail -5 gpurun_out/r04/e2e5_cfg$c.err; exit 1; }; cat gpurun_out/r04/e2e5_cfg$c.json; done
