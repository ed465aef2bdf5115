#!/bin/bash
# Hot path iteration: its parity tests, the deep-window parity tests, then config 4 (hot path, and the
# generic kernel alone for the same-box comparison). usage: tools/gpu_hot.sh TAG
set -o pipefail
TAG=${1:-hot}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_hot_path.py tests/test_gpu_parity.py -k "hot or config4 or deep or fixture" -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_hot.log 2>&1
rc=$?
tail -3 $O/pytest_hot.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $O/pytest_hot.log | head -40; exit 1; fi
timeout -k 10 400 python bench.py --workload c4 --steps 20 --warmup 5 --no-e2e > $O/c4.json 2> $O/c4.err || { echo C4_FAIL; tail -20 $O/c4.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4.json')); print('c4 hot', d['value'], d['ms_per_step'], (d['cpu_baseline'] or {}).get('value'))"
ME_HOT_MIN=0 timeout -k 10 400 python bench.py --workload c4 --steps 20 --warmup 5 --no-e2e --no-cpu-baseline > $O/c4_generic.json 2> $O/c4_generic.err || { echo C4G_FAIL; tail -20 $O/c4_generic.err; exit 1; }
python -c "import json; d=json.load(open('$O/c4_generic.json')); print('c4 generic', d['value'], d['ms_per_step'])"
