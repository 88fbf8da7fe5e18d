#!/bin/bash
# GPU box: parity tests touching k = 1024, then config-4 bench lines with the
# resident kernels (NP_RES=1) and the scratch kernels (NP_RES=0).
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/res
mkdir -p $OUT
K=${1:-"1366 or 2048-1024 or 3000-1024 or digests or full_size"}
FILES=${FILES:-tests/test_gpu_parity.py}
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 120 --timeout-method thread -k "$K" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" $OUT/pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 2 --no-cpu > $OUT/bench_res.log 2>&1 || { tail -20 $OUT/bench_res.log; exit 1; }
NP_RES=0 timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 2 --no-cpu > $OUT/bench_big.log 2>&1 || { tail -20 $OUT/bench_big.log; exit 1; }
python3 - <<'PY'
import json
for f in ("bench_res", "bench_big"):
    d = json.loads(open(f"gpurun_out/res/{f}.log").read().strip().split("\n")[-1])
    print(f, d["value"], d["ms_per_step"], {k: (v["ms"], v["frac"]) for k, v in d["kernels"].items()})
PY
