#!/bin/bash
# Round-3 record, part A: the whole GPU suite, smoke, the metric line and its kernel trace.
set -o pipefail
TAG=${1:-r3_v5}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/pytest_gpu.log | head -30; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver_shape.json 2> $O/bench_driver_shape.err || { echo BENCH_FAIL; tail -5 $O/bench_driver_shape.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_driver_shape.json')); print('c2 driver shape', round(d['value']/1e6,1), 'M/s')"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -5 $O/bench_prof.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_prof.json')); print('c2 640 steps (under rocprof)', round(d['value']/1e6,1), 'M/s')"
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; cut -d, -f1-4 $O/kernel_stats.csv | head -8
