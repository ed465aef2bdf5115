#!/bin/bash
# Same-box A/B of library variants without the post-run fills check (measurement-only variants whose
# outputs are knowingly wrong).   usage: [WL=c2] [K=20] [W=5] tools/gpu/ab_nofc.sh TAG ROUNDS lib1.so [lib2.so ...]
set -o pipefail
TAG=$1; RN=$2; shift; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
for r in $(seq 1 $RN); do
  for LIB in "$@"; do
    V=$(basename $LIB .so)
    ME_ENGINE_LIB=$R/$LIB timeout -k 10 120 python3 bench.py --workload ${WL:-c2} --steps ${K:-20} --warmup ${W:-5} --no-cpu-baseline --no-e2e --no-fills-check > $O/$V.$r.json 2> $O/$V.$r.err || { echo "BENCH_FAIL $V"; tail -5 $O/$V.$r.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$O/$V.$r.json')); print('%-14s r%d %8.1f M/s  step %.2f us  dev %.2f us' % ('$V', $r, d['value']/1e6, d['ms_per_step']*1e3, (d.get('device_ms_per_step') or 0)*1e3))"
  done
done
