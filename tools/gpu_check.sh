#!/bin/bash
# GPU tests (whole -m gpu suite, or the files given as arguments), then the
# default bench line and the config 2 / 4 bench lines.  Stops at the first
# failing step.  Outputs under gpurun_out/check/.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/check
mkdir -p $OUT
TESTS=${@:-tests}
timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py --cpu-seconds 3 > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log
for c in 2 4; do
  timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > $OUT/bench_cfg$c.log 2>&1 || { tail -20 $OUT/bench_cfg$c.log; exit 1; }
done
python3 - <<'PY'
import json
for f in ("bench", "bench_cfg2", "bench_cfg4"):
    d = json.loads(open(f"gpurun_out/check/{f}.log").read().strip().split("\n")[-1])
    print(f, d["value"], d["ms_per_step"], {k: (v["ms"], v["frac"]) for k, v in d["kernels"].items()})
PY
