#!/bin/bash
# SQ counters of k_match_hot on config 4 (the busy symbols only). usage: tools/gpu/pmc_hot.sh TAG
set -o pipefail
TAG=${1:-pmchot}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
B="python3 $R/bench.py --workload c4 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e --traffic-from ''"
run() { timeout -s KILL 300 rocprofv3 --pmc $2 --kernel-include-regex k_match_hot --output-format csv -d $O/$1 -o pmc -- $B > $O/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $O/$1.log; exit 1; }; }
run sq1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" &&
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_WAIT_INST_LDS" || exit 1
run ic "SQ_IFETCH SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE" || echo "icache pass failed"
python3 tools/pmc_last.py $O 3 34500; exit 0
python3 - <<PY
import csv,glob,collections
acc=collections.defaultdict(list)
for f in glob.glob("$O/*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k,v in sorted(acc.items()):
    a=sum(v)/len(v)
    print(f"{k:24s} n={len(v)} avg={a:.4g}")
PY
