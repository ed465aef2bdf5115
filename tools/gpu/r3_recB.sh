#!/bin/bash
# Round-3 record, part B: configs 1, 4, 3, 5 with their CPU baselines; traces of the aggregate path.
set -o pipefail
TAG=${1:-r3_v5}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for spec in "c1 16 2" "c4 20 5" "c3 320 32" "c5 320 32"; do
  set -- $spec; wl=$1
  timeout -k 10 500 python bench.py --workload $wl --steps $2 --warmup $3 --no-e2e > $O/workload_$wl.json 2> $O/workload_$wl.err || { echo "WL_FAIL $wl"; tail -5 $O/workload_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/workload_$wl.json')); print('$wl', round(d['value']/1e6,2), 'M/s; cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
for wl in c1 c4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- python3 bench.py --workload $wl --steps 8 --warmup 2 --no-e2e --no-cpu-baseline > $O/prof_$wl.json 2> $O/prof_$wl.err || { echo "PROF_FAIL $wl"; exit 1; }
  echo "== $wl"; python3 tools/trace_summary.py $(find $O/prof_$wl -name "*kernel_trace.csv" | head -1) | head -12
done
bash tools/gpu/pmc_agg.sh $TAG/pmc
