#!/bin/bash
# Round-4 probe 4: GPU tests, encode spread-store A/B, config-4 row-table DMA
# A/B, per-wave stamps, pageable e2e.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu4.log 2>&1; rc=$?
tail -3 gpurun_out/r04/pytest_gpu4.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu4.log | head -20; exit $rc; fi
TAG=p4_ bash tools/exp_one.sh base spread hiw hiwspread base spread hiw hiwspread || exit $?
TAG=p4c4_ ARGS="--config 4" bash tools/exp_one.sh base resdma0 base resdma0 || exit $?
NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/enc_stamps.py > gpurun_out/r04/enc_stamps2.log 2>&1 || { cat gpurun_out/r04/enc_stamps2.log; exit 1; }
tail -22 gpurun_out/r04/enc_stamps2.log
NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/res_stamps.py > gpurun_out/r04/res_stamps2.log 2>&1 || { cat gpurun_out/r04/res_stamps2.log; exit 1; }
tail -20 gpurun_out/r04/res_stamps2.log
for c in 3 4; do timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $([ $c = 3 ] && echo 256 || echo 64) > gpurun_out/r04/e2e4_cfg$c.json 2> gpurun_out/r04/e2e4_cfg$c.err || { tail -5 gpurun_out/r04/e2e4_cfg$c.err; exit 1; }; cat gpurun_out/r04/e2e4_cfg$c.json; done
