#!/bin/bash
# PMC passes on k_match (one counter group per pass; never combined with tracing domains).
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
B="python3 $R/bench.py --steps 320 --warmup 32 --no-cpu-baseline --no-e2e"
run() { timeout -k 10 300 rocprofv3 --pmc $2 --kernel-include-regex k_match --output-format csv -d $O/$1 -o pmc -- $B > $O/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $O/$1.log; exit 1; }; }
run sq1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM"
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG SQ_INSTS_VALU_TRANS_32"
run fetch "FETCH_SIZE"
run write "WRITE_SIZE"
run lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
python3 - <<PY
import csv,glob,collections,statistics
# per counter: the median dispatch (a steady full-group launch), per order (32 x 65,536 per launch)
acc=collections.defaultdict(list)
for f in glob.glob("$O/*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
n=32*65536
for k,v in sorted(acc.items()):
    m=statistics.median(v)
    print(f"{k:28s} dispatches={len(v):3d} median={m:.4g}  per_order={m/n:.2f}")
PY
python3 $R/tools/pmc_traffic.py $O/fetch $O/write > $O/traffic.json; cat $O/traffic.json
