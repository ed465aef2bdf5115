#!/bin/bash
# Quick GPU iteration: parity tests, a short bench (no CPU baseline), phase stamps of config 2.
# usage: tools/gpu/quick.sh TAG [notests]
set -o pipefail
TAG=${1:-quick}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ "$2" != "notests" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo TESTS_FAIL; grep -E "^E |Error|FAILED" $O/pytest_gpu.log | head -30; exit 1; fi
fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
ME_ENGINE_LIB=matching_engine_amd/build/libme_engine_stamps.so timeout -k 10 200 python tools/stamp_probe.py --batches 210 --skip 180 > $O/stamps.txt 2>&1 || { echo STAMPS_FAIL; tail -20 $O/stamps.txt; exit 1; }
cat $O/stamps.txt
