#!/bin/bash
# A/B timing of two library builds on the GPU box: runs the headline bench
# alternately (A B A B A B), 20 timed steps each, and prints every value and
# the median per build.  Usage: tools/ab_bench.sh LIB_A LIB_B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab
for r in 1 2 3; do
  for t in A B; do
    lib=$1; [ $t = B ] && lib=$2
    NP_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/ab/$t$r.log 2>&1 || exit 1
  done
done
python3 - <<'PY'
import json, statistics
for t in "AB":
    v = []
    for r in (1, 2, 3):
        d = json.loads(open(f"gpurun_out/ab/{t}{r}.log").read().strip().split("\n")[-1])
        v.append((d["value"], d["kernels"]["encode"]["ms"], d["kernels"]["reconstruct"]["ms"]))
    print(t, [x[0] for x in v], "median", statistics.median(x[0] for x in v),
          "enc", statistics.median(x[1] for x in v), "rec", statistics.median(x[2] for x in v))
PY
