#!/bin/bash
# GPU probes: one function per gpurun call (bash tools/probes.sh <name> ...; records under gpurun_out/$R, R = NP_ROUND or r06).
# Every GPU step runs under its own timeout and the steps stop at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=${NP_ROUND:-r06}
mkdir -p gpurun_out/$R

suite() {  # the whole GPU suite, then smoke
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$R/pytest_gpu_$1.log 2>&1; rc=$?
  echo "suite: $(tail -1 gpurun_out/$R/pytest_gpu_$1.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$R/pytest_gpu_$1.log | head -20; exit $rc; }
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$R/smoke_$1.log 2>&1 || exit $?
  tail -1 gpurun_out/$R/smoke_$1.log
}

bench() {  # headline bench line
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --cpu-seconds 3 > gpurun_out/$R/bench_$1.log 2>&1 || exit $?
  tail -1 gpurun_out/$R/bench_$1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], {k:(v['ms'],v['frac']) for k,v in d['kernels'].items()})"
}

e2e() {  # PCIe-inclusive host-pipeline rates, configs 3 and 4
  for c in 3 4; do
    b=256; [ $c -eq 4 ] && b=64
    timeout -k 10 300 python tools/e2e_bench.py --config $c --batch $b > gpurun_out/$R/e2e_$1_cfg$c.json 2> gpurun_out/$R/e2e_$1_cfg$c.err || exit $?
    cat gpurun_out/$R/e2e_$1_cfg$c.json
  done
}

cfgs() {  # configs 2 and 4 bench lines
  for c in 2 4; do
    timeout -k 10 300 python bench.py --config $c --steps 5 --warmup 2 --no-cpu > gpurun_out/$R/bench_$1_cfg$c.log 2>&1 || exit $?
    tail -1 gpurun_out/$R/bench_$1_cfg$c.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg$c', d['value'], {k:(v['ms'],v['frac']) for k,v in d['kernels'].items()})"
  done
}

p2() {  # experiment switches pruned (code objects unchanged but for dead code): suite, benches
  suite p2 && bench p2 && bench p2b && cfgs p2
}

ab() {  # A/B of libraries on one box: ab TAG CONFIG LIB... (product = "prod"); two passes each
  tag=$1; cfg=$2; shift 2
  for pass in 1 2; do
    for lib in "$@"; do
      path=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
      [ "$lib" != prod ] && path=$PWD/tools/exp/lib_$lib.so
      NP_LIB_PATH=$path timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu > gpurun_out/$R/ab_${tag}_${lib}_$pass.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/ab_${tag}_${lib}_$pass.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$tag cfg$cfg $lib pass$pass', d['value'], {k:v['ms'] for k,v in d['kernels'].items()})"
    done
  done
}

p3() {  # pruned library against round 4's at configs 2, 3, 4
  ab p3 2 prod r04 && ab p3 3 prod r04 && ab p3 4 prod r04
}

micro() {  # bit-slicing microbenchmark
  timeout -k 10 180 ./tools/microbench/bitslice > gpurun_out/$R/bitslice.txt 2>&1 || exit $?
  cat gpurun_out/$R/bitslice.txt
}

hugeprof() {  # kernel-trace stats of the sub-transform path at 20,000 / 40,000 / 65,536 validators
  export TMPDIR=/tmp
  for vc in ${VCS:-65536 40000 20000}; do
    out=$PWD/gpurun_out/$R/prof_huge_$vc
    mkdir -p $out
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 --batch 512 --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) > $out/bench.log 2>&1 || exit $?
    tail -1 $out/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vc$vc', d['value'], {k:v['ms'] for k,v in d['kernels'].items()})"
    f=$(find $out -name "*kernel_stats.csv" | head -1)
    python3 -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:14]:
    print('  %-70s calls %5s avg %9.1f us total %8.2f ms' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))"
  done
}

# slices(): the NP_HUGE_SLICE_MB sweep of probe p4 (profiles/r05/huge/slice_sweep.txt);
# the knob was removed after it, so the function is gone too.

p4() {  # sub-transform path: kernel profile (the slice sweep ran here too, with a knob since removed)
  hugeprof
}

p6() {  # paired sub-transform decode: huge tests, then 65,536 / 50,000 validators with and without pairing
  p5
}

p5() {  # paired sub-transform encode: huge tests, then 65,536 / 50,000 validators with and without pairing
  timeout -k 10 600 python -u -m pytest tests/test_gpu_huge.py tests/test_gpu_noncodeword.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/pytest_huge_p5.log 2>&1; rc=$?
  echo "huge tests: $(tail -1 gpurun_out/$R/pytest_huge_p5.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$R/pytest_huge_p5.log | head -20; exit $rc; }
  for vc in 65536 50000; do
    for pr in 1 0; do
      NP_HUGE_PAIR=$pr timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --batch 512 --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/$R/pair_${vc}_$pr.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/pair_${vc}_$pr.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vc$vc pair=$pr', d['value'], {k:v['ms'] for k,v in d['kernels'].items()}, d.get('roundtrip_ok'))"
    done
  done
}

p7() {  # empty-segment skip (n = 8k fast reconstruct): parity tests, then 300 / 700 / 1200 validators benches
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_noncodeword.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/pytest_p7.log 2>&1; rc=$?
  echo "tests: $(tail -1 gpurun_out/$R/pytest_p7.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$R/pytest_p7.log | head -20; exit $rc; }
  for vc in ${VCS:-300 700 1200 5000}; do
    for lib in ${LIBS:-prod base}; do
      path=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
      [ $lib != prod ] && path=$PWD/tools/exp/lib_$lib.so
      NP_LIB_PATH=$path timeout -k 10 300 python bench.py --no-cpu --steps 10 --warmup 3 --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/$R/seg_${vc}_$lib.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/seg_${vc}_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vc$vc $lib', d['value'], d['config'].get('batch'), {k:v['ms'] for k,v in d['kernels'].items()})"
    done
  done
}

p8() {  # empty sub-segment skip, k >= 512 (kernels_big.hip)
  VCS="2500 3000 5000 10000 2000" p7
}

p9() {  # empty-segment skip in the resident decodes (k = 512 / 1024, n = 8k)
  VCS="2500 3000 5000" LIBS="prod k1024 base" p7
}

p10() {  # empty 1024-row blocks in the sub-transform decode: huge tests, then 20,000 .. 65,536 validators
  timeout -k 10 600 python -u -m pytest tests/test_gpu_huge.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/pytest_huge_p10.log 2>&1; rc=$?
  echo "huge tests: $(tail -1 gpurun_out/$R/pytest_huge_p10.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$R/pytest_huge_p10.log | head -20; exit $rc; }
  for vc in 20000 40000 50000 65536; do
    for lib in prod base; do
      path=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
      [ $lib != prod ] && path=$PWD/tools/exp/lib_$lib.so
      NP_LIB_PATH=$path timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --batch 512 --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/$R/blk_${vc}_$lib.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/blk_${vc}_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vc$vc $lib', d['value'], {k:v['ms'] for k,v in d['kernels'].items()}, d.get('roundtrip_ok'))"
    done
  done
}

p11() {  # register-resident error locator: locator + parity + huge tests, then huge benches against HEAD's library
  if [ -z "$BENCH_ONLY" ]; then
    timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_huge.py tests/test_gpu_noncodeword.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/pytest_p11.log 2>&1; rc=$?
    echo "tests: $(tail -1 gpurun_out/$R/pytest_p11.log)"
    [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$R/pytest_p11.log | head -20; exit $rc; }
  fi
  for vc in 65536 40000 20000; do
    for lib in prod base; do
      path=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
      [ $lib != prod ] && path=$PWD/tools/exp/lib_$lib.so
      NP_LIB_PATH=$path timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --batch 512 --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/$R/loc_${vc}_$lib.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/loc_${vc}_$lib.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vc$vc $lib', d['value'], {k:v['ms'] for k,v in d['kernels'].items()}, d.get('roundtrip_ok'))"
    done
  done
  export TMPDIR=/tmp
  out=$PWD/gpurun_out/$R/prof_loc_65536
  mkdir -p $out
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out --output-format csv -- python3 bench.py --no-cpu --steps 3 --warmup 1 --batch 512 --n-wanted 65536 --erase 21846 > $out/bench.log 2>&1 || exit $?
  f=$(find $out -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print('  %-60s calls %5s avg %9.1f us total %8.2f ms' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))"
}

p12() {  # the register-resident locator: whole GPU suite and smoke, then p11's benches and profile
  suite p12 && BENCH_ONLY=1 p11
}

p13() {  # pinning in place opt-in (pin cases in a child process): whole suite, smoke, e2e
  suite p13 && e2e p13
}

hugeab() {  # huge tests, then VCS benches prod vs base (tools/exp/lib_base.so), two passes
  timeout -k 10 600 python -u -m pytest tests/test_gpu_huge.py tests/test_gpu_noncodeword.py ${TESTS_EXTRA} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$R/pytest_huge_$1.log 2>&1; rc=$?
  echo "huge tests: $(tail -1 gpurun_out/$R/pytest_huge_$1.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/$R/pytest_huge_$1.log | head -20; exit $rc; }
  for pass in 1 2; do
  for vc in ${VCS:-65536 50000 40000}; do
    for lib in prod base; do
      path=$PWD/reed-solomon-novelpoly_amd/lib/libnovelpoly_hip.so
      [ $lib != prod ] && path=$PWD/tools/exp/lib_$lib.so
      NP_LIB_PATH=$path timeout -k 10 300 python bench.py --no-cpu --steps 3 --warmup 1 --batch 512 --n-wanted $vc --erase $(( (vc - 1) / 3 + 1 )) > gpurun_out/$R/$1_${vc}_${lib}_$pass.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/$1_${vc}_${lib}_$pass.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('vc$vc $lib p$pass', d['value'], {k:v['ms'] for k,v in d['kernels'].items()}, d.get('roundtrip_ok'))"
    done
  done
  done
}

stamps() {  # HEAD wave-stamp table of the config-3 decode (NP_EXP=192 build; tools/wave_stamps.py)
  NP_LIB_PATH=$PWD/tools/exp/lib_192.so timeout -k 10 300 python tools/wave_stamps.py > gpurun_out/$R/decode_wave_stamps.txt 2>&1 || exit $?
  cat gpurun_out/$R/decode_wave_stamps.txt
}

p1() {  # the host-pipeline fix: whole suite, smoke, bench, e2e
  suite p1 && bench p1 && e2e p1
}


tpw() {  # tiles per workgroup of the config-3 encode / decode (NP_ENC_TPW, NP_REC_TPW), two passes
  for pass in 1 2; do
    for v in default 4 8 16 32; do
      if [ $v = default ]; then env=""; else env="NP_ENC_TPW=$v NP_REC_TPW=$v"; fi
      env $env timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/$R/tpw_${v}_$pass.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/tpw_${v}_$pass.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('tpw $v pass $pass', d['value'], {k:v['ms'] for k,v in d['kernels'].items()})"
    done
  done
}

res256() {  # the k = 256 decode on the resident kernels (NP_REC_RES256) against the fast one: parity, A/B, kernel trace
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "res256" --timeout 120 --timeout-method thread \
    > gpurun_out/$R/pytest_res256_$1.log 2>&1 || { tail -30 gpurun_out/$R/pytest_res256_$1.log; exit 1; }
  tail -1 gpurun_out/$R/pytest_res256_$1.log
  for pass in 1 2; do
    for v in 0 1; do
      NP_REC_RES256=$v timeout -k 10 200 python bench.py --no-cpu --steps 10 --warmup 3 > gpurun_out/$R/res256_${v}_$pass.log 2>&1 || exit $?
      tail -1 gpurun_out/$R/res256_${v}_$pass.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('res256=$v pass $pass', d['value'], {k:v['ms'] for k,v in d['kernels'].items()})"
    done
  done
  export NP_REC_RES256=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/prof_res256_$1 -o run -- python bench.py --no-cpu --steps 10 --warmup 3 \
    > gpurun_out/$R/prof_res256_$1.log 2>&1 || exit $?
  f=$(find gpurun_out/$R/prof_res256_$1 -name '*kernel_stats.csv' | head -1); head -8 "$f" | cut -c1-160
}

res256prof() {  # wave stamps of the k = 256 resident decode (NP_EXP=192 build), then its PMC passes (tools/profile_round.sh)
  CFG=3 BATCH=1024 NP_REC_RES256=1 NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 300 python tools/res_stamps.py \
    > gpurun_out/$R/res256_wave_stamps.txt 2>&1 || { tail -20 gpurun_out/$R/res256_wave_stamps.txt; exit 1; }
  cat gpurun_out/$R/res256_wave_stamps.txt
  NP_REC_RES256=1 timeout -k 10 900 bash tools/profile_round.sh r06_res256 3 > gpurun_out/$R/prof_res256.log 2>&1 || { tail -20 gpurun_out/$R/prof_res256.log; exit 1; }
  f=$(find gpurun_out/prof_r06_res256/stats -name '*kernel_stats.csv' | head -1); head -6 "$f" | cut -c1-160
}

stampsab() {  # wave stamps of both config-3 decodes on one box: fast (tools/wave_stamps.py) and k = 256 resident (tools/res_stamps.py)
  NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 300 python tools/wave_stamps.py > gpurun_out/$R/decode_wave_stamps.txt 2>&1 || exit $?
  CFG=3 BATCH=1024 NP_REC_RES256=1 NP_LIB_PATH=$PWD/tools/exp/lib_st192.so timeout -k 10 300 python tools/res_stamps.py \
    > gpurun_out/$R/res256_wave_stamps.txt 2>&1 || exit $?
  head -8 gpurun_out/$R/decode_wave_stamps.txt; head -8 gpurun_out/$R/res256_wave_stamps.txt
}

prefixnt() {  # thread count of k_prefix_locator (NP_PREFIX_NT, a knob of the build this ran on, removed since): parity files, then kernel traces of the config-3 bench per count
  timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_noncodeword.py -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/$R/pytest_prefixnt_$1.log 2>&1 || { tail -30 gpurun_out/$R/pytest_prefixnt_$1.log; exit 1; }
  tail -1 gpurun_out/$R/pytest_prefixnt_$1.log
  export TMPDIR=/tmp
  for pass in 1 2; do
    for v in 256 512 1024; do
      NP_PREFIX_NT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/prof_pnt_${v}_$pass --output-format csv -- python3 bench.py --no-cpu --steps 10 --warmup 3 \
        > gpurun_out/$R/pnt_${v}_$pass.log 2>&1 || exit $?
      f=$(find gpurun_out/$R/prof_pnt_${v}_$pass -name '*kernel_stats.csv' | head -1)
      echo "nt $v pass $pass: $(grep prefix_locator "$f" | awk -F'",' '{print $2}' | cut -d, -f3) ns; bench $(tail -1 gpurun_out/$R/pnt_${v}_$pass.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['kernels']['reconstruct']['ms'])")"
    done
  done
}

pntall() {  # k_prefix_locator thread count per n (experiment library tools/exp/lib_pnt.so built with an NP_PREFIX_NT knob, not in the product): kernel-trace averages
  export TMPDIR=/tmp
  for shape in "cfg2:--config 2" "vc300:--n-wanted 300 --batch 1024 --erase 100" "cfg3:--config 3" "cfg4:--config 4"; do
    name=${shape%%:*}; args=${shape#*:}
    for v in 64 128 256 512; do
      NP_PREFIX_NT=$v NP_LIB_PATH=$PWD/tools/exp/lib_pnt.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/$R/prof_pa_${name}_$v --output-format csv -- python3 bench.py --no-cpu --steps 5 --warmup 2 $args \
        > gpurun_out/$R/pa_${name}_$v.log 2>&1 || exit $?
      f=$(find gpurun_out/$R/prof_pa_${name}_$v -name '*kernel_stats.csv' | head -1)
      echo "$name nt $v: $(grep prefix_locator "$f" | awk -F'",' '{print $2}' | cut -d, -f3) ns"
    done
  done
}

"$@"
