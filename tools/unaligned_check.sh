#!/bin/bash
# Unaligned-access microbenchmark, then the GPU parity tests of the resident
# (k = 512 / 1024) kernels, then the 10 MB reference bench shape.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ua
timeout -k 10 120 tools/microbench/unaligned > gpurun_out/ua/unaligned.txt 2>&1; rc=$?; cat gpurun_out/ua/unaligned.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "512 or 1024 or 2000 or 2500 or 5000 or 4096 or noncodeword or fuzz" > gpurun_out/ua/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/ua/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu --steps 5 --warmup 2 --n-wanted 2000 --batch 100 --payload 10000000 --erase 667 > gpurun_out/ua/vc2000_10MB.log 2>&1 && tail -1 gpurun_out/ua/vc2000_10MB.log | python3 -c "
import json,sys; d=json.loads(sys.stdin.read()); print('10MB', d['value'], {k:(v['ms'], v['frac']) for k,v in d['kernels'].items()}, d['roundtrip_ok'])"
