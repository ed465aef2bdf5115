#!/bin/bash
# SQ counters of the grouped aggregate walk (k_agg_gwalk) and the per-level kernel on config 2
# (ME_REG_AGG=1). usage: tools/gpu/pmc_agg.sh TAG
set -o pipefail
TAG=${1:-pmcagg}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
B="python3 bench.py --workload c2 --steps 64 --warmup 32 --no-cpu-baseline --no-e2e --traffic-from ''"
run() { ME_REG_AGG=1 timeout -s KILL 200 rocprofv3 --pmc $2 --kernel-include-regex "$3" --output-format csv -d $O/$1 -o pmc -- $B > $O/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $O/$1.log; exit 1; }; }
run w1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" k_agg_gwalk &&
run w2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS" k_agg_gwalk &&
run l1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES" k_agg_levels || exit 1
python3 - <<PY
import csv,glob,collections
for tag in ("w1","w2","l1"):
    acc=collections.defaultdict(list)
    for f in glob.glob("$O/"+tag+"/**/*counter_collection*.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k,v in sorted(acc.items()):
        print(f"{tag} {k:24s} n={len(v)} med={sorted(v)[len(v)//2]:.6g}")
PY
