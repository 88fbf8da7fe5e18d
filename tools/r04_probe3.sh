#!/bin/bash
# Round-4 probe 3: per-wave encode stamps, host copy microbenchmark.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/enc_stamps.py > gpurun_out/r04/enc_stamps.log 2>&1 || { cat gpurun_out/r04/enc_stamps.log; exit 1; }
cat gpurun_out/r04/enc_stamps.log
timeout -k 10 120 tools/microbench/host_copy > gpurun_out/r04/host_copy.txt 2>&1 || exit $?
cat gpurun_out/r04/host_copy.txt
NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/res_stamps.py > gpurun_out/r04/res_stamps.log 2>&1 || { cat gpurun_out/r04/res_stamps.log; exit 1; }
cat gpurun_out/r04/res_stamps.log
timeout -k 10 300 python tools/e2e_bench.py --config 4 --batch 64 > gpurun_out/r04/e2e_cfg4_nt.json 2> gpurun_out/r04/e2e_cfg4_nt.err || { tail -5 gpurun_out/r04/e2e_cfg4_nt.err; exit 1; }
cat gpurun_out/r04/e2e_cfg4_nt.json
