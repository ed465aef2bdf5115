#!/bin/bash
# SQ counters (instruction mix, wait / issue cycles, LDS bank conflicts) of the round-3 kernels on
# their workloads, steady dispatches only: k_match_reg rc128 (config 2), k_match_reg rc64 (config 3),
# k_side (config 2's fill / drain launches), k_match and k_match_hot (config 4).
# usage: tools/gpu/pmc_sq_r3.sh TAG   -> gpurun_out/TAG/summary.txt
set -o pipefail
TAG=${1:-pmcsq3}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
run() {  # name workload kernel-regex steps
  for p in 1 2; do
    C=$([ $p = 1 ] && echo "$P1" || echo "$P2")
    timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "$3" --output-format csv -d $O/$1_p$p -o pmc -- python3 $R/bench.py --workload $2 --steps $4 --warmup 4 --no-cpu-baseline --no-e2e > $O/$1_p$p.log 2>&1 || { echo "PMC_FAIL $1 $p"; tail -5 $O/$1_p$p.log; return 1; }
  done
}
summ() {  # name orders-per-dispatch last-n
  echo "== $1 (last $3 dispatches, per order = / $2)"
  python3 $R/tools/pmc_last.py $O/$1_p1 $3 $2; python3 $R/tools/pmc_last.py $O/$1_p2 $3 $2
}
run reg128_c2 c2 "k_match_reg<false>" 320 && run reg64_c3 c3 "k_match_reg<false>" 160 && run side_c2 c2 k_side 20 &&
run match_c4 c4 "k_match<" 12 && run hot_c4 c4 k_match_hot 12 || exit 1
{
summ reg128_c2 $((32*65536)) 6
summ reg64_c3 $((32*131072)) 3
summ side_c2 65536 2
summ match_c4 65536 8
summ hot_c4 34500 8
} > $O/summary.txt
cat $O/summary.txt
