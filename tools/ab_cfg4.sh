#!/bin/bash
# A/B of two builds on config 4 (k = 1024 path) on the GPU box: the big-path
# parity tests on the in-tree build, then config-4 benches alternating
# ab_libs/libA.so and ab_libs/libB.so (built in this container with
# `make -C reed-solomon-novelpoly_amd OUT=$PWD/ab_libs/libX.so OBJDIR=/tmp/objX`).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ab4
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "big_path or reconstruct_shapes or full_size" > gpurun_out/ab4/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/ab4/pytest.log
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/ab4/pytest.log | head; exit $rc; }
for r in 1 2; do for t in A B; do
NP_LIB_PATH=$PWD/ab_libs/lib$t.so timeout -k 10 120 python bench.py --config 4 --no-cpu --steps 10 --warmup 2 > gpurun_out/ab4/$t$r.log 2>&1 || exit 1
done; done
python3 - <<'PY'
import json
for t in "AB":
    for r in (1,2):
        d=json.loads(open(f"gpurun_out/ab4/{t}{r}.log").read().strip().split("\n")[-1])
        print(t, r, d["value"], {k:v["ms"] for k,v in d["kernels"].items()}, d.get("roundtrip_ok"))
PY
