#!/bin/bash
# Deep-window check: the -m gpu suite, config 4's hot symbol alone (time per hot record), the c4
# bench line. usage: tools/gpu_c4.sh TAG [pytest -k filter]
set -o pipefail
TAG=${1:-c4}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
K=${2:-}
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
else
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
fi
tail -1 $O/pytest.log
timeout -k 10 300 python3 tools/c4_hot_probe.py > $O/probe.json 2> $O/probe.err || { tail -5 $O/probe.err; exit 1; }
cat $O/probe.json
timeout -k 10 400 python bench.py --workload c4 --steps 20 --warmup 5 --no-cpu-baseline > $O/c4.json 2>$O/c4.err || { tail $O/c4.err; exit 1; }
python3 -c "import json; d=json.load(open('$O/c4.json')); print('c4', round(d['value']/1e6,3), 'M orders/s, kernel ms', round(d['kernel_match_ms_avg'],3))"
