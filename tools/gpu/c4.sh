#!/bin/bash
# GPU parity tests, then the config-4 secondary line with its CPU baseline (seeded oracle).
set -o pipefail
TAG=${1:-c4}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then echo TESTS_FAIL; grep -E "^E |Error|FAILED" $O/pytest_gpu.log | head -20; exit 1; fi
timeout -k 10 600 python bench.py --workload c4 --steps 20 --warmup 5 --no-e2e --traffic-from '' > $O/c4.json 2> $O/c4.err || { echo BENCH_FAIL; tail -20 $O/c4.err; exit 1; }
cat $O/c4.json
