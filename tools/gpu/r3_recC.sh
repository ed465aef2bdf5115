#!/bin/bash
# Round-3 record after the walk changes: the whole GPU suite, smoke, the driver-shape line, the metric line
# under a kernel trace, configs 3 and 5 with the engine's own path choice. usage: tools/gpu/r3_recC.sh TAG
set -o pipefail
TAG=${1:-r3_v9}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/pytest_gpu.log | head -30; exit 1; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { echo SMOKE_FAIL; tail -5 $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
line() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['value']/1e6,2), 'M/s', 'ms/step', round(d['ms_per_step'],4), d['roofline'].get('paths'))"; }
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver_shape.json 2> $O/bench_driver_shape.err && line $O/bench_driver_shape.json "c2 driver shape" || { echo BENCH_FAIL; tail -5 $O/bench_driver_shape.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err && line $O/bench_prof.json "c2 640 steps (rocprof)" || { echo PROF_FAIL; tail -5 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; cut -d, -f1-4 $O/kernel_stats.csv | head -12
for w in c3 c5; do
  timeout -k 10 300 python bench.py --workload $w --no-e2e > $O/workload_$w.json 2> $O/workload_$w.err && line $O/workload_$w.json $w || { echo BENCH_FAIL $w; exit 1; }
done
timeout -k 10 300 python bench.py --workload c1 > $O/workload_c1.json 2> $O/workload_c1.err && line $O/workload_c1.json c1 || { echo BENCH_FAIL c1; exit 1; }
timeout -k 10 300 python bench.py --workload c4 > $O/workload_c4.json 2> $O/workload_c4.err && line $O/workload_c4.json c4 || { echo BENCH_FAIL c4; exit 1; }
ME_REG_AGG=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -k "cancelled_chunks or capacity_exhaustion" -m gpu -q -p no:cacheprovider --timeout 100 --timeout-method thread > $O/diag_agg_tiny_pool.log 2>&1; tail -3 $O/diag_agg_tiny_pool.log
