#!/bin/bash
# SQ instruction-mix counters of k_match for several library variants (ME_ENGINE_LIB).
# usage: tools/gpu/pmc_cmp.sh TAG lib1.so [lib2.so ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
for LIB in "$@"; do
  V=$(basename $LIB .so)
  export ME_ENGINE_LIB=$R/$LIB
  B="python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e"
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM --kernel-include-regex k_match --output-format csv -d $O/$V/sq1 -o pmc -- $B > $O/$V.sq1.log 2>&1 || { echo "PMC_FAIL $V sq1"; tail -5 $O/$V.sq1.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_INSTS_SENDMSG SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU SQ_INSTS_VALU_TRANS_32 --kernel-include-regex k_match --output-format csv -d $O/$V/sq2 -o pmc -- $B > $O/$V.sq2.log 2>&1 || { echo "PMC_FAIL $V sq2"; tail -5 $O/$V.sq2.log; exit 1; }
  python3 - $O/$V <<'PY'
import csv,glob,collections,sys
acc=collections.defaultdict(list)
for f in glob.glob(sys.argv[1]+"/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
n=65536
print(sys.argv[1])
for k,v in sorted(acc.items()):
    a=sum(v)/len(v)
    print(f"  {k:24s} avg={a:.4g}  per_order={a/n:.1f}")
PY
done
