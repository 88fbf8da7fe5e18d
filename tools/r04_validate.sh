#!/bin/bash
# Round-4 validation of the final product on the GPU box: the whole GPU test
# suite, then the headline bench line (with its CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
D=gpurun_out/r04v
mkdir -p $D
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -25 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
timeout -k 10 300 python bench.py --out $D/bench.json > $D/bench.log 2>&1 || { tail -5 $D/bench.log; exit 1; }
tail -1 $D/bench.log | cut -c1-400
