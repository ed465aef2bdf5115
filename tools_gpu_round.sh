#!/bin/bash
# One GPU session: smoke, default bench, rocprofv3 kernel-trace stats of a short bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_kt -o kt -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-e2e > $O/prof_kt.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_kt.log; exit 1; }
find $O/prof_kt -name "*stats*" | head
