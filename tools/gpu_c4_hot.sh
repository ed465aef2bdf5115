#!/bin/bash
# Config 4's hot symbol alone (tools/c4_hot_probe.py): time per hot record, then SQ counters per hot
# record (two rocprofv3 --pmc passes on k_match, within the per-pass counter limits).
set -o pipefail
TAG=${1:-c4hot}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
timeout -k 10 300 python3 tools/c4_hot_probe.py > $O/probe.json 2> $O/probe.err || { echo PROBE_FAIL; tail -5 $O/probe.err; exit 1; }
cat $O/probe.json
run() { timeout -s KILL 200 rocprofv3 --pmc $2 --kernel-include-regex "k_match<" --output-format csv -d $O/$1 -o pmc -- python3 $R/tools/c4_hot_probe.py > $O/$1.log 2>&1 || { echo "PMC_FAIL $1"; tail -5 $O/$1.log; exit 1; }; }
run sq1 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM" &&
run sq2 "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_SENDMSG SQ_INSTS_VALU_TRANS_32" || exit 1
python3 - <<PY
import csv, glob, json, collections, statistics
n = json.load(open("$O/probe.json"))["records_per_batch"]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob("$O/sq*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]][(f, int(r["Dispatch_Id"]))] += float(r["Counter_Value"])
print(f"SQ counters of k_match per hot record (median dispatch of one hot-symbol batch, {n:.0f} records)")
for k in sorted(acc):
    v = sorted(acc[k].values())
    big = [x for x in v if x >= 0.3 * v[-1]]
    print(f"  {k:26s} per_record={statistics.median(big) / n:10.2f}")
PY
