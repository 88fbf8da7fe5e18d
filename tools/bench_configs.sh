set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for c in 2 4; do timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu > gpurun_out/bench_cfg$c.log 2>&1 || exit 1; tail -1 gpurun_out/bench_cfg$c.log | cut -c1-600; done
