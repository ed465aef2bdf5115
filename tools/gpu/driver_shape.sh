#!/bin/bash
# The driver's bench shape (--steps 20 --warmup 5), three runs, then one under rocprofv3 --kernel-trace.
set -o pipefail
O=gpurun_out/${1:-drv}; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b$r.json 2> $O/b$r.err || { echo BENCH_FAIL; tail -5 $O/b$r.err; exit 1; }
  python -c "import json; d=json.load(open('$O/b$r.json')); print('driver shape', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step']*1e3,2), 'us/step')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/bp.json 2> $O/bp.err || { echo PROF_FAIL; exit 1; }
f=$(find $O/prof -name "*kernel_trace.csv" | head -1); cp $f $O/kernel_trace.csv
python3 - <<PY
import csv
rows=list(csv.DictReader(open("$O/kernel_trace.csv")))
rows.sort(key=lambda r:int(r["Start_Timestamp"]))
last=rows[-12:]
t0=int(last[0]["Start_Timestamp"])
for r in last:
    s=int(r["Start_Timestamp"]); e=int(r["End_Timestamp"])
    print(f"{(s-t0)/1e3:9.1f} us +{(e-s)/1e3:8.1f} us  {r['Kernel_Name'][:60]}")
PY
