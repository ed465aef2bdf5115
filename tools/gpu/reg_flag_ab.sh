#!/bin/bash
# k_match_reg built with uniform regions left unstructurized: the whole GPU suite, then configs 3 / 5 and
# config 2 on k_match_reg (ME_REG_AGG=0). usage: TAG
set -o pipefail
TAG=${1:-regflag}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/pytest_gpu.log | head -20; exit 1; fi
line() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['value']/1e6,2), 'M/s', 'ms/step', round(d['ms_per_step'],4), d['roofline'].get('paths'))"; }
for spec in "c3 320 32" "c5 320 32"; do
  set -- $spec
  timeout -k 10 400 python bench.py --workload $1 --steps $2 --warmup $3 --no-cpu-baseline --no-e2e > $O/$1.json 2> $O/$1.err && line $O/$1.json $1 || { echo BENCH_FAIL $1; exit 1; }
done
ME_REG_AGG=0 timeout -k 10 300 python bench.py --workload c2 --steps 160 --warmup 32 --no-e2e --no-cpu-baseline > $O/c2_agg0.json 2> $O/c2_agg0.err && line $O/c2_agg0.json "c2 k_match_reg" || { echo BENCH_FAIL c2; exit 1; }
