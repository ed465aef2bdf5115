#!/bin/bash
# Aggregate-path A/B after a walk change: parity (hot path + grouped), c1, c4 on both walk forms, and
# configs 2/3/5 with grouped launches off / on. usage: tools/gpu/agg_ab2.sh TAG
set -o pipefail
TAG=${1:-aggab2}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_hot_path.py tests/test_agg_groups.py -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_agg.log 2>&1
rc=$?; tail -2 $O/pytest_agg.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" $O/pytest_agg.log | head -30; exit 1; fi
line() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['value']/1e6,2), 'M/s', 'ms/step', round(d['ms_per_step'],4))"; }
timeout -k 10 300 python bench.py --workload c1 --steps 8 --warmup 2 --no-e2e --no-cpu-baseline > $O/c1.json 2> $O/c1.err && line $O/c1.json c1 || { echo BENCH_FAIL c1; exit 1; }
for lm in 256 32768; do
  ME_AGG_LADDER=$lm timeout -k 10 300 python bench.py --workload c4 --steps 12 --warmup 3 --no-e2e --no-cpu-baseline > $O/c4_l$lm.json 2> $O/c4_l$lm.err && line $O/c4_l$lm.json "c4 ladder<=$lm" || { echo BENCH_FAIL c4 $lm; exit 1; }
done
for w in c2 c3 c5; do
  for ag in 0 1; do
    ME_REG_AGG=$ag timeout -k 10 300 python bench.py --workload $w --steps 160 --warmup 32 --no-e2e --no-cpu-baseline > $O/${w}_agg$ag.json 2> $O/${w}_agg$ag.err && line $O/${w}_agg$ag.json "$w agg=$ag" || { echo BENCH_FAIL $w $ag; exit 1; }
  done
done
