#!/bin/bash
set -o pipefail
TAG=${1:-pmcsq}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
B="python3 $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-e2e"
run() { timeout -k 10 300 rocprofv3 --pmc $2 --kernel-include-regex k_match --output-format csv -d $O/$1 -o pmc -- $B > $O/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $O/$1.log; exit 1; }; }
run sq1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES GRBM_GUI_ACTIVE"
python3 - <<PY
import csv,glob,collections
acc=collections.defaultdict(list)
for f in glob.glob("$O/*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
n=65536
for k,v in sorted(acc.items()):
    a=sum(v)/len(v)
    print(f"{k:24s} avg={a:.4g}  per_order={a/n:.1f}")
PY
