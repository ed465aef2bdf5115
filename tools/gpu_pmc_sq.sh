#!/bin/bash
# SQ instruction / cycle counters of the common match kernel, per order, for library variants.
# One rocprofv3 pass per counter set per library; the median full-group dispatch is reported.
# usage: tools/gpu_pmc_sq.sh TAG lib1.so [lib2.so ...]
set -o pipefail
TAG=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
SETS=("SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_WAIT_ANY"
      "SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INSTS_SMEM")
for LIB in "$@"; do
  V=$(basename $LIB .so)
  k=0
  for SET in "${SETS[@]}"; do
    k=$((k+1))
    ME_ENGINE_LIB=$R/$LIB timeout -s KILL 120 rocprofv3 --pmc $SET --kernel-include-regex k_match --output-format csv -d $O/$V.s$k -o pmc -- python3 $R/bench.py --steps 96 --warmup 32 --no-cpu-baseline --no-e2e > $O/$V.s$k.log 2>&1 || { echo "PMC_FAIL $V set $k"; tail -5 $O/$V.s$k.log; exit 1; }
  done
  python3 - $O $V <<'PY'
import csv, glob, collections, sys
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for f in glob.glob(f"{sys.argv[1]}/{sys.argv[2]}.s*/**/*counter_collection*.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r.get("Kernel_Name", "")
        if "true" in name:  # the continuation launch
            continue
        acc[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
orders = 32 * 65536
print(f"== {sys.argv[2]}: median full-group dispatch, per order")
for k in sorted(acc):
    v = sorted(acc[k].values())
    big = [x for x in v if x > 0.5 * v[-1]]
    m = big[len(big) // 2]
    print(f"  {k:24s} per_order={m / orders:9.2f}")
PY
done
