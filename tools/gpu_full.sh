#!/bin/bash
# GPU tests, headline bench, config 2/4 benches and the PCIe end-to-end bench.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 3 > gpurun_out/bench.log 2>&1 || exit $?
for c in 2 4; do timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_cfg$c.log 2>&1 || exit $?; done
python3 - <<'PY'
import json
for f in ("bench", "bench_cfg2", "bench_cfg4"):
    d = json.loads(open(f"gpurun_out/{f}.log").read().strip().split("\n")[-1])
    print(f, d["value"], {k: (v["ms"], v["frac"]) for k, v in d["kernels"].items()})
PY
