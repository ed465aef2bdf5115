#!/bin/bash
# config-4 A/B of the deep-window hand-off: old path (ME_HOT_MIN=0), hot kernel with / without
# its head-chunk cache. usage: tools/gpu/hotab.sh TAG
set -o pipefail
TAG=${1:-hotab}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
cd $R
B="python bench.py --workload c4 --steps 12 --warmup 3 --no-e2e --no-cpu-baseline --traffic-from ''"
for V in "ME_HOT_MIN=0" "ME_HOT_MIN=64 ME_HOT_CACHE=1" "ME_HOT_MIN=64 ME_HOT_CACHE=0"; do
  F=$(echo $V | tr " =" "__")
  env $V timeout -k 10 300 $B > $O/$F.json 2> $O/$F.err || { echo BENCH_FAIL $V; tail -5 $O/$F.err; exit 1; }
  python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], round(d['value']/1e6,3), 'M orders/s', round(d['kernel_match_ms_avg'],3), 'ms')" $O/$F.json "$V"
done
