#!/bin/bash
# k_match PMC counter sets (one rocprofv3 pass per set) for one library variant.
# usage: tools/gpu/pmc_sets.sh TAG LIB "CNT1 CNT2 ..." ["..."]
set -o pipefail
TAG=$1; LIB=$2; shift; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
export ME_ENGINE_LIB=$R/$LIB
B="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e"
k=0
for SET in "$@"; do
  k=$((k+1))
  timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex k_match --output-format csv -d $O/s$k -o pmc -- $B > $O/s$k.log 2>&1 || { echo "PMC_FAIL set $k"; tail -5 $O/s$k.log; exit 1; }
done
python3 - $O <<'PY'
import csv,glob,collections,sys
acc=collections.defaultdict(list)
for f in glob.glob(sys.argv[1]+"/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
n=65536
for k,v in sorted(acc.items()):
    a=sum(v)/len(v)
    print(f"  {k:30s} avg={a:.4g}  per_order={a/n:.2f}")
PY
