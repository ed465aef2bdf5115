#!/bin/bash
# Kernel timeline of a short bench run (rocprofv3 kernel trace) -> per-kernel averages and gaps.
# usage: tools/gpu/trace.sh TAG [extra bench args]
set -o pipefail
TAG=${1:-trace}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof_kt -o kt -- python3 $R/bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-e2e "$@" > $O/prof_kt.log 2>&1 || { echo PROF_FAIL; tail -20 $O/prof_kt.log; exit 1; }
python3 $R/tools/trace_gaps.py $O/prof_kt
