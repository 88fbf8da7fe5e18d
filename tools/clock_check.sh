#!/bin/bash
# Effective shader clock of the codec kernels (GRBM_GUI_ACTIVE / 8 / duration,
# MI355X_MICROARCH.md DVFS note) for the product build and an experiment build.
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/clk
for lib in "" ${EXP_LIBS}; do
  tag=${lib:-product}; tag=$(basename $tag .so)
  NP_LIB_PATH=${lib:+$PWD/$lib} timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/clk/$tag --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 > gpurun_out/clk/$tag.log 2>&1 || exit 1
  f=$(ls -t gpurun_out/clk/$tag/*/*_counter_collection.csv | head -1)
  python3 - "$f" "$tag" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    n = r["Kernel_Name"]
    if "k_" not in n: continue
    n = n[n.find("k_"):].split("(")[0]
    agg[n][r["Counter_Name"]].append(float(r["Counter_Value"]))
for n, c in agg.items():
    ga = sum(c["GRBM_GUI_ACTIVE"]) / len(c["GRBM_GUI_ACTIVE"])
    gc = sum(c["GRBM_COUNT"]) / len(c["GRBM_COUNT"])
    print(sys.argv[2], n, "GUI_ACTIVE", ga, "COUNT", gc, "active/count", round(ga / gc, 3))
PY
done
