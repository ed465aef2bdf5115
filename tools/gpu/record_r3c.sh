set -o pipefail
O=gpurun_out/r3_v2; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --no-cpu-baseline > $O/bench_prof.json 2> $O/bench_prof.err || { echo PROF_FAIL; tail -5 $O/bench_prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; cut -d, -f1-6 $O/kernel_stats.csv | head -12
bash tools/gpu/record_r3b.sh r3_v2
