#!/bin/bash
# Round-3 iteration: smoke, the -m gpu suite, the default bench, and a short N=1 bench with the cluster
# leg (RCCL at world size 1). usage: tools/gpu_r3.sh TAG [pytest args...]
set -o pipefail
TAG=${1:-r3}
shift
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 240 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1
rc=$?
tail -3 $O/pytest_gpu.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -40; exit 1; fi
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python bench.py --steps 64 --warmup 8 --no-cpu-baseline --no-e2e --cluster-steps 12 > $O/bench_cluster.json 2> $O/bench_cluster.err || { echo CLUSTER_BENCH_FAIL; tail -20 $O/bench_cluster.err; exit 1; }
python -c "import json; print(json.load(open('$O/bench_cluster.json'))['cluster'])"
