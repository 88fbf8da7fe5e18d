#!/bin/bash
# A/B/... timing of library builds on the GPU box: the headline bench (or
# CONFIG=c) for each build in turn, ROUNDS (default 3) interleaved rounds of
# 20 timed steps, then per build the median value and kernel times.
# Usage: tools/ab_libs.sh LIB...   (paths relative to the repo root)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
R=${ROUNDS:-3}
i=0
for r in $(seq 1 $R); do
  j=0
  for lib in "$@"; do
    NP_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu ${BENCH_ARGS:---config ${CONFIG:-3}} --steps 20 --warmup 3 > gpurun_out/ab/L${j}_$r.log 2>&1 || { tail -5 gpurun_out/ab/L${j}_$r.log; exit 1; }
    j=$((j+1))
  done
done
python3 - "$R" "$@" <<'PY'
import json, statistics, sys
R = int(sys.argv[1]); libs = sys.argv[2:]
for j, lib in enumerate(libs):
    v = []
    for r in range(1, R + 1):
        d = json.loads(open(f"gpurun_out/ab/L{j}_{r}.log").read().strip().split("\n")[-1])
        v.append((d["value"], d["kernels"]["encode"]["ms"], d["kernels"]["reconstruct"]["ms"]))
    print(f"{lib:45s}", [x[0] for x in v], "median", statistics.median(x[0] for x in v),
          "enc", statistics.median(x[1] for x in v), "rec", statistics.median(x[2] for x in v))
PY
