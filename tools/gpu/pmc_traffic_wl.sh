#!/bin/bash
# HBM traffic per order of one workload's match launches (rocprofv3 FETCH_SIZE / WRITE_SIZE, one
# counter per pass, never with tracing) -> gpurun_out/TAG/pmc_traffic_WL.json (bench.py reads
# profiles/pmc_traffic_WL.json for roofline.traffic).
# usage: tools/gpu/pmc_traffic_wl.sh TAG WL KERNEL_REGEX ORDERS_PER_LAUNCH STEPS [MERGE_NEXT_REGEX [LAST_N]]
set -o pipefail
TAG=$1; WL=$2; K=$3; OPL=$4; STEPS=$5; MN=$6; LAST=$7
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG/$WL
mkdir -p $O
export TMPDIR=/tmp
cd $R
run() { timeout -k 10 400 rocprofv3 --pmc $2 --kernel-include-regex "$K" --output-format csv -d $O/$1 -o pmc -- python3 $R/bench.py --workload $WL --steps $STEPS --warmup 4 --no-cpu-baseline --no-e2e > $O/$1.log 2>&1 || { echo "PMC_FAIL $WL $1"; tail -5 $O/$1.log; exit 1; }; }
run fetch FETCH_SIZE && run write WRITE_SIZE || exit 1
python3 $R/tools/pmc_traffic.py $O/fetch $O/write --kernel "$K" --orders-per-launch $OPL ${MN:+--merge-next $MN} ${LAST:+--last $LAST} > $R/gpurun_out/$TAG/pmc_traffic_$WL.json
python3 -c "import json; d=json.load(open('$R/gpurun_out/$TAG/pmc_traffic_$WL.json')); print('$WL', d.get('bytes_per_order'), 'B/order', d.get('dispatches'))"
