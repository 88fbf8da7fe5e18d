#!/bin/bash
# Round-4 probe on the GPU box: GPU tests, the headline bench, and the
# per-phase stamps of the config-3 decode (tools/exp/lib_st64.so, NP_EXP=64).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/r04/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r04/bench.log 2>&1 || exit $?
tail -1 gpurun_out/r04/bench.log | cut -c1-300
NP_LIB_PATH=$PWD/tools/exp/lib_st64.so timeout -k 10 120 python tools/phase_stamps.py > gpurun_out/r04/stamps.log 2>&1 || exit $?
cat gpurun_out/r04/stamps.log
[ -x tools/microbench/bfly_rates ] || make -s -C tools/microbench bfly_rates || exit $?
timeout -k 10 120 tools/microbench/bfly_rates > gpurun_out/r04/bfly_rates.txt 2>&1 || exit $?
cat gpurun_out/r04/bfly_rates.txt
