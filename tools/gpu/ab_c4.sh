#!/bin/bash
# Same-box A/B of library variants on config 4 (hot-path experiments): the hot-path parity tests on
# each variant, then R interleaved rounds of the c4 bench line. usage: tools/gpu/ab_c4.sh TAG R lib...
set -o pipefail
TAG=$1; RN=$2; shift; shift
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for LIB in "$@"; do
  V=$(basename $LIB .so)
  ME_ENGINE_LIB=$PWD/$LIB timeout -k 10 300 python -u -m pytest tests/test_hot_path.py -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > $O/$V.pytest.log 2>&1 || { echo "TEST_FAIL $V"; tail -20 $O/$V.pytest.log; exit 1; }
  echo "$V tests: $(tail -1 $O/$V.pytest.log)"
done
for r in $(seq 1 $RN); do
  for LIB in "$@"; do
    V=$(basename $LIB .so)
    ME_ENGINE_LIB=$PWD/$LIB timeout -k 10 300 python bench.py --workload c4 --steps 24 --warmup 4 --no-cpu-baseline --no-e2e > $O/$V.$r.json 2> $O/$V.$r.err || { echo "BENCH_FAIL $V"; tail -5 $O/$V.$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$V.$r.json')); print('%-18s r%d %6.3f M/s  %.3f ms/step' % ('$V', $r, d['value']/1e6, d['ms_per_step']))"
  done
done
