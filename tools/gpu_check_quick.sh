#!/bin/bash
# GPU tests + the headline bench against tools/exp/lib_head.so (GPU box).
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; exit $rc; }
bash tools/exp_one.sh head base head base ${EXTRA_LIBS}
