#!/bin/bash
# Same-box A/B of the grouped aggregate path (ME_REG_AGG=1) against k_match_reg on configs 2, 3 and 5,
# plus configs 1 and 4 (hot symbols, aggregate path by default), and a kernel trace of config 2 on the
# aggregate path. usage: tools/gpu/agg_ab.sh TAG
set -o pipefail
TAG=${1:-agg_ab}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
line() { python -c "import json,sys; d=json.load(open('$1')); print('$2', round(d['value']/1e6,1), 'M/s', 'ms/step', round(d['ms_per_step'],4), 'frac', d['roofline']['frac'])"; }
for spec in "c2 0 160 32" "c2 1 160 32" "c3 0 96 32" "c3 1 96 32" "c5 0 96 32" "c5 1 96 32"; do
  set -- $spec; wl=$1; ag=$2
  ME_REG_AGG=$ag timeout -k 10 300 python bench.py --workload $wl --steps $3 --warmup $4 --no-e2e --no-cpu-baseline > $O/${wl}_agg$ag.json 2> $O/${wl}_agg$ag.err || { echo "BENCH_FAIL $wl agg=$ag"; tail -5 $O/${wl}_agg$ag.err; exit 1; }
  line $O/${wl}_agg$ag.json "$wl agg=$ag"
done
ME_REG_AGG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2agg -o run -- python3 bench.py --workload c2 --steps 64 --warmup 32 --no-e2e --no-cpu-baseline > $O/c2agg_prof.json 2> $O/c2agg_prof.err || { echo PROF_FAIL; tail -5 $O/c2agg_prof.err; exit 1; }
f=$(find $O/prof_c2agg -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats_c2agg.csv; head -16 $O/kernel_stats_c2agg.csv | cut -d, -f1-4
