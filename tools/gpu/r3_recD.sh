#!/bin/bash
# Round-3 record, the secondary lines with the engine's own path choice (c3 / c5 at 320 timed batches as
# in r3_recB: the bench sizes max_resting from the whole run), c1 / c4 with CPU baselines, the tiny-pool
# diagnostic of the grouped aggregate path, SQ counters of the config-1 walk. usage: TAG
set -o pipefail
TAG=${1:-r3_v10}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
line() { python -c "import json; d=json.load(open('$1')); c=d.get('cpu_baseline') or {}; print('$2', round(d['value']/1e6,2), 'M/s', 'ms/step', round(d['ms_per_step'],4), d['roofline'].get('paths'), 'cpu', c.get('value'), c.get('cores'))"; }
for spec in "c3 320 32" "c5 320 32" "c1 16 2" "c4 20 5"; do
  set -- $spec
  timeout -k 10 400 python bench.py --workload $1 --steps $2 --warmup $3 > $O/workload_$1.json 2> $O/workload_$1.err && line $O/workload_$1.json $1 || { echo BENCH_FAIL $1; tail -3 $O/workload_$1.err; exit 1; }
done
ME_REG_AGG=1 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -k "cancelled_chunks or capacity_exhaustion" -m gpu -q -p no:cacheprovider --timeout 100 --timeout-method thread > $O/diag_agg_tiny_pool.log 2>&1; tail -3 $O/diag_agg_tiny_pool.log
bash tools/gpu/pmc_walk_c1.sh $TAG/pmc_c1
