#!/bin/bash
# Round record on one MI355X box: full GPU tests, smoke, default bench (with CPU baseline), a 2-rank
# gloo rehearsal of the N>1 bench path on the one GPU. usage: tools/gpu_round.sh TAG
set -o pipefail
TAG=${1:-round}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
cat $O/smoke.log | tail -1
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 --steps 64 --warmup 4 --dist-backend gloo --no-cpu-baseline > $O/bench_n2_gloo.json 2> $O/bench_n2_gloo.err || { tail -20 $O/bench_n2_gloo.err; exit 1; }
cat $O/bench_n2_gloo.json
