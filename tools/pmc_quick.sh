#!/bin/bash
# One PMC pass over a short bench run (GPU box): per-kernel counter means.
# Usage: pmc_quick.sh TAG COUNTER...
TAG=$1; shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/pq
timeout -s KILL 120 rocprofv3 --pmc "$@" -d gpurun_out/pq/$TAG --output-format csv -- python3 bench.py --no-cpu --steps 2 --warmup 1 ${BENCH_ARGS} > gpurun_out/pq/$TAG.log 2>&1 || exit 1
f=$(ls -t gpurun_out/pq/$TAG/*/*_counter_collection.csv | head -1)
python3 - "$f" <<'PY'
import csv, sys, collections
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "k_" not in n: continue
    agg[n[n.find("k_"):].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in agg.items():
    w = sum(c["SQ_WAVES"]) / len(c["SQ_WAVES"]) if "SQ_WAVES" in c else 1
    print(n, {k: round(sum(v) / len(v) / w, 1) for k, v in c.items() if k != "SQ_WAVES"}, "waves", w)
PY
