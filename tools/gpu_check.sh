set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --cpu-seconds 3 > gpurun_out/bench.log 2>&1; rc=$?
cat gpurun_out/bench.log | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/e2e_bench.py > gpurun_out/e2e.log 2>&1; rc=$?
tail -2 gpurun_out/e2e.log
exit $rc
