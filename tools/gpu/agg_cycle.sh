#!/bin/bash
# One iteration on the aggregate path: parity tests, c1/c4 lines, c2 A/B (k_match_reg vs grouped), kernel
# trace of c1 and c2-grouped, SQ counters of the grouped walk. usage: tools/gpu/agg_cycle.sh TAG
set -o pipefail
TAG=${1:-aggcyc}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hot_path.py tests/test_agg_groups.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_agg.log 2>&1
rc=$?; tail -2 $O/pytest_agg.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/pytest_agg.log | head -30; exit 1; fi
line() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['value']/1e6,2), 'M/s', 'ms/step', round(d['ms_per_step'],4))"; }
timeout -k 10 300 python bench.py --workload c4 --steps 12 --warmup 3 --no-e2e --no-cpu-baseline > $O/c4.json 2> $O/c4.err && line $O/c4.json c4 || { echo BENCH_FAIL c4; exit 1; }
for ag in 0 1; do
  ME_REG_AGG=$ag timeout -k 10 300 python bench.py --workload c2 --steps 160 --warmup 32 --no-e2e --no-cpu-baseline > $O/c2_agg$ag.json 2> $O/c2_agg$ag.err && line $O/c2_agg$ag.json "c2 agg=$ag" || { echo BENCH_FAIL c2 $ag; exit 1; }
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c1 -o run -- python3 bench.py --workload c1 --steps 8 --warmup 2 --no-e2e --no-cpu-baseline > $O/c1.json 2> $O/c1.err || { echo PROF_FAIL c1; tail -5 $O/c1.err; exit 1; }
line $O/c1.json c1; python3 tools/trace_summary.py $(find $O/prof_c1 -name "*kernel_trace.csv" | head -1) | head -10
ME_REG_AGG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2agg -o run -- python3 bench.py --workload c2 --steps 64 --warmup 32 --no-e2e --no-cpu-baseline > $O/c2agg_prof.json 2> $O/c2agg_prof.err || { echo PROF_FAIL c2agg; exit 1; }
python3 tools/trace_summary.py $(find $O/prof_c2agg -name "*kernel_trace.csv" | head -1) | head -10
bash tools/gpu/pmc_agg.sh $TAG/pmc
