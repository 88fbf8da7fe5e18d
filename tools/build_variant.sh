#!/bin/bash
# Builds an experiment variant of the library: tools/build_variant.sh NAME "-DFLAG=1 ..."
# -> tools/exp/lib_NAME.so (never the product)
cd "$(dirname "$0")/.."
make -s -j8 -C reed-solomon-novelpoly_amd OUT=$PWD/tools/exp/lib_$1.so OBJDIR=$PWD/tools/exp/build_$1 EXTRA="$2" 2>&1 | grep -iE "error" ; ls -la tools/exp/lib_$1.so
