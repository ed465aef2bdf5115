#!/bin/bash
# Rehearsal of the N>1 bench path on a one-GPU box: 2 ranks (gloo collectives) sharing the card.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/n2
mkdir -p $O
cd $R
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo > $O/n2.json 2> $O/n2.err || { echo N2_FAIL; tail -30 $O/n2.err; exit 1; }
cat $O/n2.json
