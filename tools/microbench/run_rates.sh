#!/bin/bash
# GPU box: VALU issue rates and HBM copy calibration -> gpurun_out/mb/
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/mb
timeout -k 10 120 tools/microbench/valu_rates > gpurun_out/mb/valu_rates.txt 2>&1 &&
timeout -k 10 120 tools/microbench/calib_traffic > gpurun_out/mb/calib_traffic.txt 2>&1
rc=$?
cat gpurun_out/mb/*.txt
exit $rc
