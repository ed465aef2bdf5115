# Round-3 iteration: the whole GPU suite, then the bench lines of configs 2, 3 and 4.
set -o pipefail
TAG=${1:-r3it}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^FAILED|^E " $O/pytest_gpu.log | head -30; exit 1; fi
for wl in c2 c3 c4; do
  timeout -k 10 400 python bench.py --workload $wl --steps 40 --warmup 8 --no-e2e --no-cpu-baseline > $O/$wl.json 2> $O/$wl.err || { echo "BENCH_FAIL $wl"; tail -5 $O/$wl.err; exit 1; }
  python -c "import json; d=json.load(open('$O/$wl.json')); print('$wl', round(d['value']/1e6,1), 'M/s', d['ms_per_step'])"
done
