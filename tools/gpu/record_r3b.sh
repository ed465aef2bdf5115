#!/bin/bash
# Round-3 record, part 2: the steady-state headline (config 2 at 640 timed batches) and configs 1, 3, 4,
# 5 with their CPU baselines. usage: tools/gpu/record_r3b.sh TAG
set -o pipefail
TAG=${1:-r3rec}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp

for spec in "c3 320 32" "c5 320 32" "c4 20 5" "c1 16 2"; do
  set -- $spec; wl=$1
  timeout -k 10 600 python bench.py --workload $wl --steps $2 --warmup $3 --no-e2e > $O/workload_$wl.json 2> $O/workload_$wl.err || { echo "WL_FAIL $wl"; tail -5 $O/workload_$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/workload_$wl.json')); print('$wl', round(d['value']/1e6,2), 'M/s; cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
