#!/bin/bash
# HBM traffic of the pipelined match launches (k_match_reg<false> + its continuation <true>): one
# rocprofv3 pass per counter (FETCH_SIZE, WRITE_SIZE), never combined with tracing domains.
# usage: tools/gpu_pmc_traffic.sh TAG [bench args...]
set -o pipefail
TAG=${1:-traffic}
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
run() { timeout -k 10 300 rocprofv3 --pmc $2 --kernel-include-regex k_match_reg --output-format csv -d $O/$1 -o pmc -- python3 $R/bench.py --steps 320 --warmup 32 --no-cpu-baseline --no-e2e "${@:3}" > $O/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $O/$1.log; exit 1; }; }
run fetch FETCH_SIZE "$@"
run write WRITE_SIZE "$@"
python3 $R/tools/pmc_traffic.py $O/fetch $O/write --kernel k_match_reg --orders-per-launch $((32*65536)) > $O/traffic.json
cat $O/traffic.json
