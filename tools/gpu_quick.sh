#!/bin/bash
# Selected GPU tests (args = pytest node ids / -k filters) and then the default bench.
# usage: tools/gpu_quick.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-quick}
shift
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1; rc=$?
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -40; exit 1; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
