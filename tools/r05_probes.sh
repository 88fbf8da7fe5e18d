#!/bin/bash
# Round-5 GPU probes: one function per gpurun call (bash tools/r05_probes.sh <name>).
# Every GPU step runs under its own timeout and the steps stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r05

suite() {  # the whole GPU suite, then smoke
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r05/pytest_gpu_$1.log 2>&1; rc=$?
  echo "suite: $(tail -1 gpurun_out/r05/pytest_gpu_$1.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r05/pytest_gpu_$1.log | head -20; exit $rc; }
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05/smoke_$1.log 2>&1 || exit $?
  tail -1 gpurun_out/r05/smoke_$1.log
}

bench() {  # headline bench line
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 3 > gpurun_out/r05/bench_$1.log 2>&1 || exit $?
  tail -1 gpurun_out/r05/bench_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], {k:(v['ms'],v['frac']) for k,v in d['kernels'].items()})"
}

e2e() {  # PCIe-inclusive host-pipeline rates, configs 3 and 4
  for c in 3 4; do
    b=256; [ $c -eq 4 ] && b=64
    timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $b > gpurun_out/r05/e2e_$1_cfg$c.json 2> gpurun_out/r05/e2e_$1_cfg$c.err || exit $?
    cat gpurun_out/r05/e2e_$1_cfg$c.json
  done
}

p1() {  # the host-pipeline fix: whole suite, smoke, bench, e2e
  suite p1 && bench p1 && e2e p1
}

"$@"
