#!/bin/bash
# Validation of the current build: smoke, the -m gpu suite, then bench lines (a failure of either ends the call).   tools/gpu/val.sh TAG [bench specs as record.sh: bench:WL:K:W ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then
  grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -30
  exit 1
fi
exec_steps="$@"
[ -n "$exec_steps" ] && bash tools/gpu/record.sh $TAG $exec_steps
