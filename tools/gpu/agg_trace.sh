#!/bin/bash
# Kernel durations of the aggregate hot-symbol path on configs 1 and 4 (rocprofv3 --kernel-trace --stats).
# usage: tools/gpu/agg_trace.sh TAG
set -o pipefail
TAG=${1:-agg_trace}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
for spec in "c1 8 2" "c4 10 3"; do
  set -- $spec; wl=$1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$wl -o run -- python3 bench.py --workload $wl --steps $2 --warmup $3 --no-e2e --no-cpu-baseline > $O/bench_$wl.json 2> $O/bench_$wl.err || { echo "PROF_FAIL $wl"; tail -5 $O/bench_$wl.err; exit 1; }
  f=$(find $O/prof_$wl -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_$wl.csv
  echo "== $wl"; head -14 $O/kernel_stats_$wl.csv | cut -d, -f1-4
done
# config 2's shape with every symbol on the aggregate path (L = 256, ME_HOT_MIN=1): the walk's cost per
# record at ~64 records per symbol and batch
ME_HOT_MIN=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2agg -o run -- python3 bench.py --workload c2 --levels 256 --steps 10 --warmup 3 --no-e2e --no-cpu-baseline > $O/bench_c2agg.json 2> $O/bench_c2agg.err || { echo "PROF_FAIL c2agg"; tail -5 $O/bench_c2agg.err; exit 1; }
f=$(find $O/prof_c2agg -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_c2agg.csv
echo "== c2agg"; head -14 $O/kernel_stats_c2agg.csv | cut -d, -f1-4
