#!/bin/bash
# GPU box: host-pipeline parity (pageable + pinned) and the e2e rates of configs 3 and 4.
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/e2e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_noncodeword.py tests/test_gpu_multi.py -m gpu -x -v --timeout 120 --timeout-method thread -k "host" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python tools/e2e_bench.py --config 3 > $OUT/cfg3.json 2> $OUT/cfg3.err || { tail $OUT/cfg3.err; exit 1; }
cat $OUT/cfg3.json
timeout -k 10 300 python tools/e2e_bench.py --config 4 --batch 64 > $OUT/cfg4.json 2> $OUT/cfg4.err || { tail $OUT/cfg4.err; exit 1; }
cat $OUT/cfg4.json
