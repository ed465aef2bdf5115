#!/bin/bash
# One GPU session for the record: gpu tests, smoke, rocprofv3 kernel-trace stats of a short bench,
# the HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE, one counter per pass) on k_match, and the
# default bench line carrying that traffic. Every GPU step has its own time limit; the first
# failure ends the session.   usage: tools/gpu/round.sh TAG [skip-tests]
set -o pipefail
TAG=${1:-run}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; tail -3 $O/pytest_gpu.log
  if [ $rc -ne 0 ]; then echo TESTS_FAIL; grep -E "^E |Error|FAILED" $O/pytest_gpu.log | head -20; exit 1; fi
fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
B="python3 $R/bench.py --steps 320 --warmup 32 --no-cpu-baseline --no-e2e"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_kt -o kt -- $B > $O/prof_kt.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_kt.log; exit 1; }
python3 $R/tools/trace_gaps.py $O/prof_kt > $O/trace_gaps.txt && cat $O/trace_gaps.txt
bash $R/tools/gpu_pmc_traffic.sh $TAG/traffic || { echo PMC_FAIL; exit 1; }
cp $O/traffic/traffic.json $O/traffic.json
timeout -k 10 600 python bench.py --traffic-from $O/traffic.json > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
