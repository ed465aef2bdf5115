#!/bin/bash
# Aggregate path: parity tests, configs 1 and 4 (hot symbols), then the config 2/3/5 A/B (agg_ab.sh).
set -o pipefail
TAG=${1:-aggrun}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hot_path.py tests/test_agg_groups.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_agg.log 2>&1
rc=$?; tail -3 $O/pytest_agg.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/pytest_agg.log | head -30; exit 1; fi
for spec in "c1 12 2" "c4 12 3"; do
  set -- $spec; wl=$1
  timeout -k 10 400 python bench.py --workload $wl --steps $2 --warmup $3 --no-e2e --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { echo "BENCH_FAIL $wl"; tail -5 $O/$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', round(d['value']/1e6,2), 'M/s', d['ms_per_step'])"
done
bash tools/gpu/agg_ab.sh $TAG/ab
