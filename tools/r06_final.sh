#!/bin/bash
# Round-6 closing run on the GPU box: the GPU test suite, the records
# (tools/records.sh: BASELINE lines with CPU baselines, config-1 CPU record,
# shapes), the config-3 kernel trace and PMC passes (tools/profile_round.sh),
# and the PCIe-inclusive rates (tools/e2e_bench.py).  Usage:
#   bash tools/r06_final.sh [RECORDS_TAG [PROFILE_TAG [PART]]]   (defaults r06f, r06,
#   all; PART a = tests and records, b = profiles and PCIe rates)
set -o pipefail
cd $GRAFT_REPO_ROOT
RT=${1:-r06f}
PT=${2:-r06}
PART=${3:-ab}
D=gpurun_out/$RT
mkdir -p $D
if [[ $PART == *a* ]]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $D/pytest_gpu.log 2>&1 || { tail -25 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
bash tools/records.sh $RT > $D/records.log 2>&1 || { tail -20 $D/records.log; exit 1; }
cat $D/records.log
fi
[[ $PART == *b* ]] || { echo final part a done; exit 0; }
bash tools/profile_round.sh $PT 3 > gpurun_out/prof_$PT.log 2>&1 || { tail -20 gpurun_out/prof_$PT.log; exit 1; }
bash tools/profile_round.sh ${PT}_cfg4 4 > gpurun_out/prof_${PT}_cfg4.log 2>&1 || { tail -20 gpurun_out/prof_${PT}_cfg4.log; exit 1; }
bash tools/profile_round.sh ${PT}_cfg2 2 > gpurun_out/prof_${PT}_cfg2.log 2>&1 || { tail -20 gpurun_out/prof_${PT}_cfg2.log; exit 1; }
for c in 3 4; do
  timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $([ $c = 3 ] && echo 256 || echo 64) > $D/e2e_cfg$c.json 2> $D/e2e_cfg$c.err || { tail -5 $D/e2e_cfg$c.err; exit 1; }
  cat $D/e2e_cfg$c.json
done
echo final done
