#!/bin/bash
# Round-4 probe 9: the generic kernels' rate at 2-21 validators (k = 1, 2, 4;
# smallmin8 = NP_SMALL_MINK=8) against the small kernels of the product.
set -o pipefail
cd $GRAFT_REPO_ROOT
for vc in 2 3 6 10 20; do
  TAG=p9v${vc}_ ARGS="--n-wanted $vc --batch 1024 --erase $(( (vc - 1) / 3 + 1 ))" bash tools/exp_one.sh base smallmin8 || exit $?
done
