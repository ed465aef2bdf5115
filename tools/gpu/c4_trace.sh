# Kernel durations of config 4 (k_match vs k_match_hot and the rest): rocprofv3 --kernel-trace --stats.
set -o pipefail
O=gpurun_out/c4_trace; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --workload c4 --steps 10 --warmup 3 --no-e2e --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -5 $O/bench.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; head -12 $O/kernel_stats.csv | cut -d, -f1-8
