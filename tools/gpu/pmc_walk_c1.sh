#!/bin/bash
# SQ counters of the hot-symbol aggregate walk (k_agg_walk, ladder form) on config 1. usage: TAG
set -o pipefail
TAG=${1:-pmcc1}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
B="python3 bench.py --workload c1 --steps 6 --warmup 2 --no-cpu-baseline --no-e2e"
run() { timeout -s KILL 200 rocprofv3 --pmc $2 --kernel-include-regex "$3" --output-format csv -d $O/$1 -o pmc -- $B > $O/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $O/$1.log; exit 1; }; }
run c1w1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" k_agg_walk &&
run c1w2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" k_agg_walk || exit 1
python3 - <<PY
import csv,glob,collections
for tag in ("c1w1","c1w2"):
    acc=collections.defaultdict(list)
    for f in glob.glob("$O/"+tag+"/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k,v in sorted(acc.items()):
        v=sorted(v)
        print(f"{tag} {k:24s} n={len(v)} med={v[len(v)//2]:.6g} per_record={v[len(v)//2]/62500:.1f}")
PY
