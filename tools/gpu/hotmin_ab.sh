#!/bin/bash
# config 4: the hot threshold (ME_HOT_MIN) A/B, and a kernel trace at each setting
set -o pipefail
O=gpurun_out/hm; mkdir -p $O
export TMPDIR=/tmp
for v in 512 1024 2048 4096; do
  ME_HOT_MIN=$v timeout -k 10 300 python3 bench.py --workload c4 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --no-fills-check > $O/c4_hm$v.json 2> $O/c4_hm$v.err || { echo FAIL $v; tail -5 $O/c4_hm$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_hm$v.json')); print('hot_min=$v %.2f M/s step %.3f ms' % (d['value']/1e6, d['ms_per_step']))"
done
for v in 512 4096; do
  ME_HOT_MIN=$v timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr$v -o kt -- python3 bench.py --workload c4 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-fills-check > $O/tr$v.json 2> $O/tr$v.err || { echo TRFAIL $v; exit 1; }
done
