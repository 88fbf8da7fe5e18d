#!/bin/bash
# Round-4 GPU probes (one gpurun call each: bash tools/r04_probes.sh NAME).
# Their A/B results are collected in profiles/r04_ab.txt; the libraries they
# compare are tools/build_variant.sh builds (tools/exp/lib_NAME.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r04 gpurun_out/exp

# Round-4 probe on the GPU box: GPU tests, the headline bench, and the
# per-phase stamps of the config-3 decode (tools/exp/lib_st64.so, NP_EXP=64).
p1() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest_gpu.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu.log | head -20; exit $rc; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu > gpurun_out/r04/bench.log 2>&1 || exit $?
  tail -1 gpurun_out/r04/bench.log | cut -c1-300
  NP_LIB_PATH=$PWD/tools/exp/lib_st64.so timeout -k 10 120 python tools/phase_stamps.py > gpurun_out/r04/stamps.log 2>&1 || exit $?
  cat gpurun_out/r04/stamps.log
  [ -x tools/microbench/bfly_rates ] || make -s -C tools/microbench bfly_rates || exit $?
  timeout -k 10 120 tools/microbench/bfly_rates > gpurun_out/r04/bfly_rates.txt 2>&1 || exit $?
  cat gpurun_out/r04/bfly_rates.txt
}

# Round-4 probe 2: per-wave decode stamps, host-memory e2e (pinned and
# pageable), records.
p2() {
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/wave_stamps.py > gpurun_out/r04/wave_stamps.log 2>&1 || exit $?
  cat gpurun_out/r04/wave_stamps.log
  for c in 3 4; do timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $([ $c = 3 ] && echo 256 || echo 64) > gpurun_out/r04/e2e_cfg$c.json 2> gpurun_out/r04/e2e_cfg$c.err || { tail -5 gpurun_out/r04/e2e_cfg$c.err; exit 1; }; cat gpurun_out/r04/e2e_cfg$c.json; done
  bash tools/records.sh r04a
}

# Round-4 probe 3: per-wave encode stamps, host copy microbenchmark.
p3() {
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/enc_stamps.py > gpurun_out/r04/enc_stamps.log 2>&1 || { cat gpurun_out/r04/enc_stamps.log; exit 1; }
  cat gpurun_out/r04/enc_stamps.log
  timeout -k 10 120 tools/microbench/host_copy > gpurun_out/r04/host_copy.txt 2>&1 || exit $?
  cat gpurun_out/r04/host_copy.txt
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/res_stamps.py > gpurun_out/r04/res_stamps.log 2>&1 || { cat gpurun_out/r04/res_stamps.log; exit 1; }
  cat gpurun_out/r04/res_stamps.log
  timeout -k 10 300 python tools/e2e_bench.py --config 4 --batch 64 > gpurun_out/r04/e2e_cfg4_nt.json 2> gpurun_out/r04/e2e_cfg4_nt.err || { tail -5 gpurun_out/r04/e2e_cfg4_nt.err; exit 1; }
  cat gpurun_out/r04/e2e_cfg4_nt.json
}

# Round-4 probe 4: GPU tests, encode spread-store A/B, config-4 row-table DMA
# A/B, per-wave stamps, pageable e2e.
p4() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu4.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest_gpu4.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu4.log | head -20; exit $rc; fi
  TAG=p4_ bash tools/exp_one.sh base spread hiw hiwspread base spread hiw hiwspread || exit $?
  TAG=p4c4_ ARGS="--config 4" bash tools/exp_one.sh base resdma0 base resdma0 || exit $?
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/enc_stamps.py > gpurun_out/r04/enc_stamps2.log 2>&1 || { cat gpurun_out/r04/enc_stamps2.log; exit 1; }
  tail -22 gpurun_out/r04/enc_stamps2.log
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/res_stamps.py > gpurun_out/r04/res_stamps2.log 2>&1 || { cat gpurun_out/r04/res_stamps2.log; exit 1; }
  tail -20 gpurun_out/r04/res_stamps2.log
  for c in 3 4; do timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $([ $c = 3 ] && echo 256 || echo 64) > gpurun_out/r04/e2e4_cfg$c.json 2> gpurun_out/r04/e2e4_cfg$c.err || { tail -5 gpurun_out/r04/e2e4_cfg$c.err; exit 1; }; cat gpurun_out/r04/e2e4_cfg$c.json; done
}

# Round-4 probe 5: GPU tests (product and the decode row-DMA variant), decode
# row-DMA A/B at configs 3 and 2, encode HIW-early A/B, pageable pin-in-place e2e.
p5() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu5.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest_gpu5.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu5.log | head -20; exit $rc; fi
  NP_LIB_PATH=$PWD/tools/exp/lib_rowdma.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu5_rowdma.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest_gpu5_rowdma.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu5_rowdma.log | head -20; exit $rc; fi
  TAG=p5_ bash tools/exp_one.sh base rowdma hiw base rowdma hiw || exit $?
  TAG=p5c2_ ARGS="--config 2" bash tools/exp_one.sh base rowdma base rowdma || exit $?
  for c in 3 4; do timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $([ $c = 3 ] && echo 256 || echo 64) > gpurun_out/r04/e2e5_cfg$c.json 2> gpurun_out/r04/e2e5_cfg$c.err || { tail -5 gpurun_out/r04/e2e5_cfg$c.err; exit 1; }; cat gpurun_out/r04/e2e5_cfg$c.json; done
}

# Round-4 probe 6: GPU tests with the next-tile row prefetch (NP_REC_TILE_PREFETCH=1
# in the product), A/B against tpf0 at config 3 and at 1200 validators (8 segments).
p6() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu6.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest_gpu6.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu6.log | head -20; exit $rc; fi
  TAG=p6_ bash tools/exp_one.sh base tpf0 base tpf0 || exit $?
  TAG=p6v1200_ ARGS="--n-wanted 1200 --batch 1024 --erase 400" bash tools/exp_one.sh base tpf0 base tpf0 || exit $?
}

# Round-4 probe 8: GPU tests with the encode's fused tower -> Cantor conversion
# (NP_ENC_CONV=1 in the product), A/B against conv0 at configs 3 and 2.
p8() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu8.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest_gpu8.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu8.log | head -20; exit $rc; fi
  TAG=p8_ bash tools/exp_one.sh base conv0 base conv0 || exit $?
  TAG=p8c2_ ARGS="--config 2" bash tools/exp_one.sh base conv0 || exit $?
  TAG=p8v700_ ARGS="--n-wanted 700 --batch 1024 --erase 234" bash tools/exp_one.sh base conv0 || exit $?
}

# Round-4 probe 9: the generic kernels' rate at 2-21 validators (k = 1, 2, 4;
# smallmin8 = NP_SMALL_MINK=8) against the small kernels of the product.
p9() {
  for vc in 2 3 6 10 20; do
    TAG=p9v${vc}_ ARGS="--n-wanted $vc --batch 1024 --erase $(( (vc - 1) / 3 + 1 ))" bash tools/exp_one.sh base smallmin8 || exit $?
  done
}

# Round-4 probe 10: k = 2048 (6,144-12,288 validators) on the big kernels
# (default) against the size-1024 sub-transform kernels (NP_HUGE=1).
p10() {
  for vc in 6144 7000 10000 12000; do
    for h in def 1; do
      if [ $h = 1 ]; then export NP_HUGE=1; else unset NP_HUGE; fi
      timeout -k 10 180 python bench.py --no-cpu --steps 10 --warmup 2 --n-wanted $vc --batch 512 --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/exp/p10_${vc}_$h.log 2>&1 || { tail -3 gpurun_out/exp/p10_${vc}_$h.log; exit 1; }
      python3 -c "
import json; d=json.loads(open('gpurun_out/exp/p10_${vc}_$h.log').read().strip().split('\n')[-1]); c=d['config']; print('p10 vc$vc huge=$h', c['n'], c['k'], d['value'], d['roundtrip_ok'], {k:v['ms'] for k,v in d['kernels'].items()})"
    done
  done
}

# Round-4 profiles: kernel-trace stats and PMC passes for configs 3, 2 and 4.
profiles() {
  bash tools/profile_round.sh r04 3 > gpurun_out/prof_r04.log 2>&1 || { tail -20 gpurun_out/prof_r04.log; exit 1; }
  bash tools/profile_round.sh r04_cfg2 2 > gpurun_out/prof_r04_cfg2.log 2>&1 || { tail -20 gpurun_out/prof_r04_cfg2.log; exit 1; }
  bash tools/profile_round.sh r04_cfg4 4 > gpurun_out/prof_r04_cfg4.log 2>&1 || { tail -20 gpurun_out/prof_r04_cfg4.log; exit 1; }
  echo profiles done
}

# Round-4 probe 11: GPU tests with the multi-tile k = 64 / 128 decodes
# (NP_REC_MT_SMALL=1 in the product), A/B against mt0 at config 2 and 300 /
# 700 validators.
p11() {
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu11.log 2>&1; rc=$?
  tail -3 gpurun_out/r04/pytest_gpu11.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu11.log | head -20; exit $rc; fi
  TAG=p11c2_ ARGS="--config 2" bash tools/exp_one.sh base mt0 base mt0 || exit $?
  TAG=p11v300_ ARGS="--n-wanted 300 --batch 1024 --erase 100" bash tools/exp_one.sh base mt0 || exit $?
  TAG=p11v700_ ARGS="--n-wanted 700 --batch 1024 --erase 234" bash tools/exp_one.sh base mt0 || exit $?
  TAG=p11v190_ ARGS="--n-wanted 190 --batch 1024 --erase 64" bash tools/exp_one.sh base mt0 || exit $?
}

# Round-4 probe 13: the encode's next-tile payload DMA without the barrier
# (nobar: NP_ENC_DMA_NOBAR=1), spread over the last cq pass (spread:
# NP_ENC_DMA_SPREAD=1; spreadnb: both; parity first for the two riskier ones),
# the merge rows loaded during the forward high pass (merge2: NP_MERGE_EARLY=2),
# and the decode's tiles per workgroup (NP_REC_TPW 4 / 16 against the
# launcher's 8) at config 3; cross-lane move rates (permlane_rates).
p13() {
  for v in nobar spreadnb; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu13_$v.log 2>&1; rc=$?
    tail -2 gpurun_out/r04/pytest_gpu13_$v.log
    if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu13_$v.log | head -20; exit $rc; fi
  done
  TAG=p13_ bash tools/exp_one.sh base nobar spread spreadnb merge2 base nobar spread spreadnb merge2 || exit $?
  for t in 4 16 8; do
    NP_REC_TPW=$t timeout -k 10 120 python bench.py --no-cpu --steps 10 --warmup 2 > gpurun_out/exp/p13_tpw$t.log 2>&1 || { tail -3 gpurun_out/exp/p13_tpw$t.log; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/exp/p13_tpw$t.log').read().strip().split('\\n')[-1]); print('p13_tpw$t', d['value'], {k:v['ms'] for k,v in d['kernels'].items()})"
  done
  [ -x tools/microbench/permlane_rates ] || make -s -C tools/microbench permlane_rates || exit 1
  timeout -k 10 120 tools/microbench/permlane_rates > gpurun_out/r04/permlane_rates.txt 2>&1 || exit 1
  cat gpurun_out/r04/permlane_rates.txt
}

# Round-4 probe 14: per-wave phase stamps of the final config-3 encode and
# decode (NP_EXP=192 build st192).
p14() {
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/wave_stamps.py > gpurun_out/r04/wave_stamps_final.log 2>&1 || { tail -5 gpurun_out/r04/wave_stamps_final.log; exit 1; }
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/enc_stamps.py > gpurun_out/r04/enc_stamps_final.log 2>&1 || { tail -5 gpurun_out/r04/enc_stamps_final.log; exit 1; }
  head -32 gpurun_out/r04/wave_stamps_final.log
  head -24 gpurun_out/r04/enc_stamps_final.log
}

# Round-4 probe 15: the next tile's payload by 16-byte LDS-DMA pieces
# (x4: NP_ENC_DMA_X4=1; parity first) against the product at config 3.
p15() {
  NP_LIB_PATH=$PWD/tools/exp/lib_x4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu15_x4.log 2>&1; rc=$?
  tail -2 gpurun_out/r04/pytest_gpu15_x4.log
  if [ $rc -ne 0 ]; then grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu15_x4.log | head -20; exit $rc; fi
  TAG=p15_ bash tools/exp_one.sh base x4 base x4 base x4 || exit $?
}

# Round-4 probe 17: the product with scalar-base DMA addresses (parity
# suite), against the 64-bit per-lane addresses ('sad0') and the next tile's
# DMA from 4 or 8 waves only after a barrier ('w4', 'w8'), at config 3; then
# the product's encode stamps
p17() {
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu17.log 2>&1; rc=$?
  echo "product: $(tail -1 gpurun_out/r04/pytest_gpu17.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu17.log | head -20; exit $rc; }
  for v in w4 w8; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "encode or roundtrip" > gpurun_out/r04/pytest_gpu17_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu17_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu17_$v.log | head -20; exit $rc; }
  done
  TAG=p17_ bash tools/exp_one.sh base sad0 w4 w8 base sad0 w4 w8 || exit $?
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 120 python tools/enc_stamps.py > gpurun_out/r04/enc_stamps_x4.txt 2>&1 || exit $?
  tail -22 gpurun_out/r04/enc_stamps_x4.txt
}

# Round-4 probe 18: progress-based issue priority in the transform passes
# (NP_PRIO_PROGRESS=1 'prio'; with the 4-wave DMA 'priow4'), parity first,
# against the product and 'w4' at config 3, then 'prio' at config 4
p18() {
  for v in prio priow4; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu18_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu18_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu18_$v.log | head -20; exit $rc; }
  done
  TAG=p18_ bash tools/exp_one.sh base w4 prio priow4 base w4 prio priow4 || exit $?
  ARGS="--config 4" TAG=p18c4_ bash tools/exp_one.sh base prio || exit $?
}

# Round-4 probe 19: the product with progress priority in the encode and the
# decode's per-tile lane id (parity suite); A/B at config 3 against the encode
# without priority ('prio0'), the decode's spilled thread id ('tidspill'),
# priority in the decode's segment cq ('pd1') or high ('pd2') levels, and the
# 4-wave DMA ('w4'); config 4 and 1200 validators against 'prio0'
p19() {
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu19.log 2>&1; rc=$?
  echo "product: $(tail -1 gpurun_out/r04/pytest_gpu19.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu19.log | head -20; exit $rc; }
  for v in pd1 pd2 w4; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu19_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu19_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu19_$v.log | head -20; exit $rc; }
  done
  TAG=p19_ bash tools/exp_one.sh base prio0 tidspill pd1 pd2 w4 base prio0 tidspill pd1 pd2 w4 || exit $?
  ARGS="--config 4" TAG=p19c4_ bash tools/exp_one.sh base prio0 base prio0 || exit $?
  TAG=p19v300_ ARGS="--n-wanted 300 --batch 1024 --erase 100" bash tools/exp_one.sh base prio0 || exit $?
}

# Round-4 probe 20: probe 19 with the product's parity suite run with
# serialized kernels first (probe 19's run faulted in
# test_host_pipeline_all_systematic[12289-4097-73728-3-pageable], a huge-path
# case whose kernels did not change: a fault now names its kernel), then
# probe 19's A/B
p20() {
  AMD_SERIALIZE_KERNEL=3 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r04/pytest_gpu20.log 2>&1; rc=$?
  echo "product (serialized): $(tail -1 gpurun_out/r04/pytest_gpu20.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|error|assert" gpurun_out/r04/pytest_gpu20.log | head -30; exit $rc; }
  for v in pd1 pd2 w4; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not pipeline" > gpurun_out/r04/pytest_gpu20_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu20_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu20_$v.log | head -20; exit $rc; }
  done
  TAG=p20_ bash tools/exp_one.sh base prio0 tidspill pd1 pd2 w4 base prio0 tidspill pd1 pd2 w4 || exit $?
  ARGS="--config 4" TAG=p20c4_ bash tools/exp_one.sh base prio0 base prio0 || exit $?
  TAG=p20v300_ ARGS="--n-wanted 300 --batch 1024 --erase 100" bash tools/exp_one.sh base prio0 || exit $?
}

# Round-4 probe 21: one priority schedule per barrier-free span of the
# decode's segment sweep (NP_PRIO_DEC=8 'span'), parity first, against the
# product and 'pd1' at config 3
p21() {
  NP_LIB_PATH=$PWD/tools/exp/lib_span.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not pipeline" > gpurun_out/r04/pytest_gpu21_span.log 2>&1; rc=$?
  echo "span: $(tail -1 gpurun_out/r04/pytest_gpu21_span.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu21_span.log | head -20; exit $rc; }
  TAG=p21_ bash tools/exp_one.sh base span pd1 base span pd1 base span pd1 || exit $?
}

# Round-4 probe 22: the product with the decode's span priority (parity
# suite); A/B at config 3 against the span schedule over the forward
# transform as well ('sf'), the encode's span schedule ('espan') and no decode
# priority ('dec0'); config 2 and 300 validators against 'dec0'
p22() {
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r04/pytest_gpu22.log 2>&1; rc=$?
  echo "product: $(tail -1 gpurun_out/r04/pytest_gpu22.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu22.log | head -20; exit $rc; }
  for v in sf espan; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not pipeline" > gpurun_out/r04/pytest_gpu22_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu22_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu22_$v.log | head -20; exit $rc; }
  done
  TAG=p22_ bash tools/exp_one.sh base sf espan dec0 base sf espan dec0 || exit $?
  ARGS="--config 2" TAG=p22c2_ bash tools/exp_one.sh base dec0 base dec0 || exit $?
  TAG=p22v300_ ARGS="--n-wanted 300 --batch 1024 --erase 100" bash tools/exp_one.sh base dec0 || exit $?
}

# Round-4 probe 23: progress-based priority in the resident kernels' encode
# ('res1') and decode ('res2') at config 4 and 2000 validators, and in the
# huge kernels ('huge3') at 10000 validators; parity first
p23() {
  for v in res1 res2 huge3; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not pipeline" > gpurun_out/r04/pytest_gpu23_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu23_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu23_$v.log | head -20; exit $rc; }
  done
  ARGS="--config 4" TAG=p23c4_ bash tools/exp_one.sh base res1 res2 base res1 res2 || exit $?
  TAG=p23v2000_ ARGS="--n-wanted 2000 --batch 1024 --erase 667" bash tools/exp_one.sh base res1 res2 || exit $?
  TAG=p23v10000_ ARGS="--n-wanted 10000 --batch 512 --erase 3334" bash tools/exp_one.sh base huge3 base huge3 || exit $?
  TAG=p23c3_ bash tools/exp_one.sh base base || exit $?
}

# Round-4 probe 24: the resident decode's span schedule ('rspan',
# NP_PRIO_RES=7) at config 4 and 2000 validators; the fast decode's
# premultiply at priority 3 or 1 instead of 2 ('pm3', 'pm1') at config 3
p24() {
  for v in rspan pm3 pm1; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not pipeline" > gpurun_out/r04/pytest_gpu24_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu24_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu24_$v.log | head -20; exit $rc; }
  done
  ARGS="--config 4" TAG=p24c4_ bash tools/exp_one.sh base rspan base rspan || exit $?
  TAG=p24v2000_ ARGS="--n-wanted 2000 --batch 1024 --erase 667" bash tools/exp_one.sh base rspan || exit $?
  TAG=p24_ bash tools/exp_one.sh base pm3 pm1 base pm3 pm1 || exit $?
}

# Round-4 probe 25: progress-based priority in the big kernels (k = 2048:
# 7000 validators; 'big3' = encode and decode), parity first
p25() {
  NP_LIB_PATH=$PWD/tools/exp/lib_big3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not pipeline" > gpurun_out/r04/pytest_gpu25_big3.log 2>&1; rc=$?
  echo "big3: $(tail -1 gpurun_out/r04/pytest_gpu25_big3.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu25_big3.log | head -20; exit $rc; }
  TAG=p25v7000_ ARGS="--n-wanted 7000 --batch 512 --erase 2334" bash tools/exp_one.sh base big3 base big3 || exit $?
}

# Round-4 probe 26: the fast decode's high levels at 3, 3, 2, 2 inside the span
# ('hi4'; with the premultiply at 1: 'hi4pm1') at config 3, parity first
p26() {
  for v in hi4 hi4pm1; do
    NP_LIB_PATH=$PWD/tools/exp/lib_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "not pipeline" > gpurun_out/r04/pytest_gpu26_$v.log 2>&1; rc=$?
    echo "$v: $(tail -1 gpurun_out/r04/pytest_gpu26_$v.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04/pytest_gpu26_$v.log | head -20; exit $rc; }
  done
  TAG=p26_ bash tools/exp_one.sh base hi4 hi4pm1 base hi4 hi4pm1 base hi4 hi4pm1 || exit $?
}

"$@"
