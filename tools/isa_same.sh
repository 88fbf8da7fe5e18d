#!/bin/bash
# Compiles every kernel file to gfx950 assembly in $1 and compares it with the
# assembly in $2 (ignoring the per-compile __hip_cuid symbols): a
# behaviour-preserving source change (e.g. removing an experiment switch at its
# default) leaves the code objects identical.  Not product code.
out=$1; base=$2; mkdir -p $out
cd "$(dirname "$0")/../reed-solomon-novelpoly_amd/csrc"
for f in kernels_fast kernels_big kernels_res kernels_huge kernels_small kernels_generic kernels_systematic; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Wno-unused-function -munsafe-fp-atomics --cuda-device-only -S -o $out/$f.s $f.hip 2>/dev/null &
done
wait
rc=0
for f in kernels_fast kernels_big kernels_res kernels_huge kernels_small kernels_generic kernels_systematic; do
  if diff <(grep -v "__hip_cuid\|\.file\|\.ident" $base/$f.s) <(grep -v "__hip_cuid\|\.file\|\.ident" $out/$f.s) > /dev/null; then
    echo "same $f"
  else
    echo "DIFF $f"; rc=1
  fi
done
exit $rc
