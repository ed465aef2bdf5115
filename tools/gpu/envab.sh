#!/bin/bash
# Same-box A/B of engine environment switches on one library: the bench per setting, R rounds interleaved.
#   usage: [WL=c2] [K=20] [W=5] tools/gpu/envab.sh TAG ROUNDS VAR VALUE1 [VALUE2 ...]
set -o pipefail
TAG=$1; RN=$2; VAR=$3; shift 3
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for r in $(seq 1 $RN); do
  for V in "$@"; do
    env $VAR=$V timeout -k 10 120 python3 bench.py --workload ${WL:-c2} --steps ${K:-20} --warmup ${W:-5} --no-cpu-baseline --no-e2e > $O/$VAR-$V.$r.json 2> $O/$VAR-$V.$r.err || { echo "BENCH_FAIL $VAR=$V"; tail -5 $O/$VAR-$V.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$VAR-$V.$r.json')); print('%s=%-4s r%d %8.1f M/s  step %.2f us' % ('$VAR', '$V', $r, d['value']/1e6, d['ms_per_step']*1e3))"
  done
done
