#!/bin/bash
# me_kernels.hip built with uniform regions left unstructurized: the whole GPU suite, configs 4 and 1, and
# config 2's metric line. usage: TAG
set -o pipefail
TAG=${1:-kernflag}; O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/pytest_gpu.log | head -20; exit 1; fi
line() { python -c "import json; d=json.load(open('$1')); print('$2', round(d['value']/1e6,2), 'M/s', 'ms/step', round(d['ms_per_step'],4))"; }
timeout -k 10 300 python bench.py --workload c4 --steps 12 --warmup 3 --no-e2e --no-cpu-baseline > $O/c4.json 2> $O/c4.err && line $O/c4.json c4 || { echo BENCH_FAIL c4; exit 1; }
timeout -k 10 300 python bench.py --workload c1 --steps 8 --warmup 2 --no-e2e --no-cpu-baseline > $O/c1.json 2> $O/c1.err && line $O/c1.json c1 || { echo BENCH_FAIL c1; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err && line $O/c2_driver.json "c2 driver shape" || { echo BENCH_FAIL c2; exit 1; }
