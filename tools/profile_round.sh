#!/bin/bash
# GPU-box profiling for one round and one bench config: kernel-trace stats of
# the bench, separate PMC passes for FETCH_SIZE / WRITE_SIZE / SQ counters, and
# the calibration microbenchmark for the 8-byte-per-lane access width.
# Usage: tools/profile_round.sh TAG [CONFIG]   -> gpurun_out/prof_<TAG>/
# (then, here: python tools/pmc_summary.py TAG -> profiles/<TAG>_pmc_summary.json)
set -o pipefail
TAG=${1:-r02}
CFG=${2:-3}
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
# the calibration kernel of the FETCH/WRITE correction: build it here if the
# tree came without it (it is git-ignored)
[ -x tools/microbench/calib_traffic ] || make -s -C tools/microbench calib_traffic || exit $?
B="bench.py --no-cpu --config $CFG --steps 3 --warmup 1"
BS="bench.py --no-cpu --config $CFG --steps 10 --warmup 3"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/stats --output-format csv -- python3 $BS > $OUT/stats.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch --output-format csv -- python3 $B > $OUT/fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write --output-format csv -- python3 $B > $OUT/write.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_INSTS_LDS -d $OUT/sq --output-format csv -- python3 $B > $OUT/sq.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $OUT/sq2 --output-format csv -- python3 $B > $OUT/sq2.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/calib_fetch --output-format csv -- tools/microbench/calib_traffic > $OUT/calib_fetch.log 2>&1 &&
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/calib_write --output-format csv -- tools/microbench/calib_traffic > $OUT/calib_write.log 2>&1
rc=$?
ls $OUT
exit $rc
