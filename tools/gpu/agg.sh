#!/bin/bash
# The aggregate hot-symbol path (me_agg.hip): its parity tests, then the c1 / c4 bench lines.
# usage: tools/gpu/agg.sh TAG [bench]
set -o pipefail
TAG=${1:-agg}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_hot_path.py tests/test_agg_groups.py -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_hot.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_hot.log | tail -30
if [ $rc -ne 0 ]; then grep -E "^E " $O/pytest_hot.log | head -40; exit 1; fi
[ "$2" = "bench" ] || exit 0
for wl in c1 c4; do
  timeout -k 10 400 python bench.py --workload $wl --steps 12 --warmup 3 --no-e2e --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { echo "BENCH_FAIL $wl"; tail -5 $O/$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', round(d['value']/1e6,2), 'M/s', d['ms_per_step'])"
done
