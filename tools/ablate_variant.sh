#!/bin/bash
# Traffic attribution builds: the working tree's sources with one store removed (sed on a copy under
# matching_engine_amd/build/src_NAME; the product sources are untouched), built into build/ab/libme_NAME.so.
# The outputs of such a build are wrong by construction: use them only for byte counts
# (ME_ENGINE_LIB=... tools/gpu/record.sh TAG traffic). The removed stores must leave every address
# the kernels compute in bounds.
#   usage: tools/ablate_variant.sh NAME FILE SED_EXPR
set -e
NAME=$1; FILE=$2; EXPR=$3
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/matching_engine_amd/build
S=$B/src_$NAME
rm -rf $S && mkdir -p $S/csrc $S/include $B/ab
cp $R/matching_engine_amd/csrc/* $S/csrc/; cp $R/include/* $S/include/
sed -i "$EXPR" $S/csrc/$FILE
cmp -s $S/csrc/$FILE $R/matching_engine_amd/csrc/$FILE && { echo "ablation matched nothing"; exit 1; }
make -s -C $R/matching_engine_amd CSRC=$S/csrc OBJDIR=$B/obj_$NAME OUT=$B/ab/libme_$NAME.so \
  CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I$S/include -I$S/csrc" -j8 >/dev/null
echo built $B/ab/libme_$NAME.so
