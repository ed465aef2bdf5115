#!/bin/bash
# One GPU iteration: smoke, the -m gpu parity suite (extra pytest args pass through), a short bench.
# usage: tools/gpu_iter.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-iter}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1
rc=$?
tail -5 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -40; exit 1; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
