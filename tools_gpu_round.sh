#!/bin/bash
# One GPU session: gpu tests, smoke, default bench, rocprofv3 kernel-trace stats of a short bench.
# usage: tools_gpu_round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -m pytest tests -m gpu -x -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo TESTS_FAIL; grep -E "^E |Error" $O/pytest_gpu.log | head -20; exit 1; fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_kt -o kt -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-e2e > $O/prof_kt.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_kt.log; exit 1; }
python3 - <<PY
import csv,glob
for f in glob.glob("$O/prof_kt/*kernel_stats.csv"):
    for r in csv.DictReader(open(f)):
        print(f"{r['Name'][:32]:32s} calls={r['Calls']:>5} avg_us={float(r['AverageNs'])/1e3:8.2f} pct={float(r['Percentage']):6.2f}")
PY
