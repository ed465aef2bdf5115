#!/bin/bash
# Build libme_engine.so from the sources at a git revision (default: the working tree) into
# matching_engine_amd/build/ab/libme_NAME.so, for same-box A/B runs (ME_ENGINE_LIB; build/ab travels with
# the gpurun snapshot).
# usage: tools/build_variant.sh NAME [REV] [extra HIP flags]
set -e
NAME=$1; REV=${2:-WORKTREE}; shift; shift || true
R=$(cd "$(dirname "$0")/.." && pwd)
B=$R/matching_engine_amd/build
S=$B/src_$NAME
rm -rf $S && mkdir -p $S/csrc $S/include $B/ab
if [ "$REV" = "WORKTREE" ]; then
  cp $R/matching_engine_amd/csrc/* $S/csrc/; cp $R/include/* $S/include/
else
  git -C $R archive $REV matching_engine_amd/csrc include | tar -x -C $S --strip-components=0
  mv $S/matching_engine_amd/csrc/* $S/csrc/; cp $S/include/* $S/include/ 2>/dev/null || true
fi
make -s -C $R/matching_engine_amd CSRC=$S/csrc OBJDIR=$B/obj_$NAME OUT=$B/ab/libme_$NAME.so ${REGFLAGS+REGFLAGS="$REGFLAGS"} ${KERNFLAGS+KERNFLAGS="$KERNFLAGS"} \
  CXXFLAGS="-O3 -std=c++17 -fPIC -Wall -Wno-unused-function -I$S/include -I$S/csrc $*" -j8 >/dev/null
echo built $B/ab/libme_$NAME.so
