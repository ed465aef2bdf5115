#!/bin/bash
# Round-3 closing record: the whole GPU suite, smoke, the driver-shape line, the 640-step metric line.
set -o pipefail
TAG=${1:-r3_v13}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/pytest_gpu.log | head -30; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
line() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['value']/1e6,2), 'M/s', 'ms/step', round(d['ms_per_step'],4), d['roofline'].get('paths'), 'traffic B/order', d['roofline'].get('traffic_bytes_per_order'))"; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver_shape.json 2> $O/bench_driver_shape.err && line $O/bench_driver_shape.json "c2 driver shape" || { echo BENCH_FAIL; tail -5 $O/bench_driver_shape.err; exit 1; }
timeout -k 10 400 python bench.py > $O/bench_640.json 2> $O/bench_640.err && line $O/bench_640.json "c2 640 steps" || { echo BENCH_FAIL; tail -5 $O/bench_640.err; exit 1; }
