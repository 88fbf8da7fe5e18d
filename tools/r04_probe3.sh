#!/bin/bash
# Round-4 probe 3: per-wave encode stamps, host copy microbenchmark.
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04
NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/enc_stamps.py > gpurun_out/r04/enc_stamps.log 2>&1 || { cat gpurun_out/r04/enc_stamps.log; exit 1; }
cat gpurun_out/r04/enc_stamps.log
timeout -k 10 120 tools/microbench/host_copy > gpurun_out/r04/host_copy.txt 2>&1 || exit $?
cat gpurun_out/r04/host_copy.txt
