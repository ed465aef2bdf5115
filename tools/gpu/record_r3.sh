#!/bin/bash
# Round-3 record, part 1: smoke, the whole -m gpu suite, the default bench line (as the driver runs it)
# and its rocprofv3 kernel-trace summary. usage: tools/gpu/record_r3.sh TAG
set -o pipefail
TAG=${1:-r3rec}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -40; exit 1; fi
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -5 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; cut -d, -f1-6 $O/kernel_stats.csv | head -12
