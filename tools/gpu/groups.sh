#!/bin/bash
# GPU parity tests, then the default bench line at 1, 4 and 8 batches per launch (same box).
set -o pipefail
TAG=${1:-grp}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then echo TESTS_FAIL; grep -E "^E |Error|FAILED" $O/pytest_gpu.log | head -30; exit 1; fi
for g in ${GROUPS_TO_RUN:-1 4 8}; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --batches-per-launch $g > $O/bench_g$g.json 2> $O/bench_g$g.err || { echo BENCH_FAIL; tail -20 $O/bench_g$g.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_g$g.json'));print('G=$g', round(d['value']/1e6,1),'M/s', 'k_match', round(d['kernel_match_ms_avg']*1e3,1),'us/launch', 'frac', round(d['roofline']['frac'],5))"
done
