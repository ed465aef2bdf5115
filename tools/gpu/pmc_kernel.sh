#!/bin/bash
# SQ counters (two passes) of the kernels matching REGEX on a workload's bench run, summarised per kernel
# by tools/prof_summary.py sq.   usage: tools/gpu/pmc_kernel.sh TAG WL REGEX [STEPS] [WARMUP]
set -o pipefail
TAG=$1; WL=$2; RE=$3; K=${4:-6}; W=${5:-2}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
B="python3 $R/bench.py --workload $WL --steps $K --warmup $W --no-cpu-baseline --no-e2e --no-fills-check"
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
  i=$((i + 1))
  timeout -s KILL 400 rocprofv3 --pmc $set --kernel-include-regex "$RE" --output-format csv -d $O/sq_$i -o pmc -- $B > $O/sq_$i.log 2>&1 || { echo "SQ_FAIL $i"; tail -5 $O/sq_$i.log; exit 1; }
done
python3 $R/tools/prof_summary.py sq $O/sq_1 $O/sq_2 > $O/sq.txt && cat $O/sq.txt
