#!/bin/bash
# One GPU iteration: the named -m gpu test files (or all), then bench lines with environment overrides.
#   tools/gpu/iter.sh TAG "tests/test_a.py tests/test_b.py|all|none" "ENV=.. WL K W" ["ENV=.. WL K W" ...]
# (each bench spec: space-separated KEY=VAL overrides, then workload, steps, warmup)
set -o pipefail
TAG=$1; TESTS=$2; shift 2
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
if [ "$TESTS" != none ]; then
  [ "$TESTS" = all ] && TESTS=tests
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -3 $O/pytest.log
  if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $O/pytest.log | head -30; exit 1; fi
fi
i=0
for spec in "$@"; do
  i=$((i + 1))
  envs=(); rest=()
  for t in $spec; do if [[ $t == *=* ]]; then envs+=("$t"); else rest+=("$t"); fi; done
  wl=${rest[0]:-c2}; k=${rest[1]:-20}; w=${rest[2]:-5}
  env "${envs[@]}" timeout -k 10 400 python3 bench.py --workload $wl --steps $k --warmup $w --no-cpu-baseline --no-e2e $BENCH_ARGS > $O/b$i.json 2> $O/b$i.err || { echo "BENCH_FAIL $spec"; tail -20 $O/b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/b$i.json')); print('$spec:', round(d['value']/1e6,2), 'M/s', 'kernel_ms', round(d['kernel_match_ms_avg'],3), d['build'])"
done
