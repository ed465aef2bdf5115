#!/bin/bash
set -o pipefail
O=gpurun_out/${1:-trace_c1}; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload c1 --steps 8 --warmup 2 --no-e2e --no-cpu-baseline > $O/c1.json 2> $O/c1.err || { echo PROF_FAIL; tail -5 $O/c1.err; exit 1; }
python3 tools/trace_summary.py $(find $O/prof -name "*kernel_trace.csv" | head -1) | head -16
