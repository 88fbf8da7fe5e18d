cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/base
for c in 3 4 2; do timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 2 --no-cpu > gpurun_out/base/bench_cfg$c.log 2>&1 || exit $?; tail -1 gpurun_out/base/bench_cfg$c.log; done
