#!/bin/bash
# Kernel-trace stats of one short bench run (GPU box): gpurun_out/qs/<tag>
TAG=${1:-q}
shift
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/qs
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/qs/$TAG --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 "$@" > gpurun_out/qs/$TAG.log 2>&1 || exit $?
f=$(ls -t gpurun_out/qs/$TAG/*/*_kernel_stats.csv | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"]
    n = n[n.find("k_"):][:60] if "k_" in n else n[:60]
    print(f'{float(r["AverageNs"])/1e3:10.1f} us  x{r["Calls"]:>3}  {n}')
PY
