#!/bin/bash
# Deep-window hot-symbol path: GPU parity tests, then the config-4 bench line with and without the
# k_match_hot hand-off (ME_HOT_MIN=0). usage: tools/gpu/hot.sh TAG [tests-filter]
set -o pipefail
TAG=${1:-hot}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread ${2:+-k "$2"} > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then echo TESTS_FAIL; grep -E "^E |Error|FAILED" $O/pytest_gpu.log | head -20; exit 1; fi
timeout -k 10 400 python bench.py --workload c4 --steps 20 --warmup 5 --no-e2e --no-cpu-baseline --traffic-from '' > $O/c4.json 2> $O/c4.err || { echo BENCH_FAIL; tail -20 $O/c4.err; exit 1; }
cat $O/c4.json
