#!/bin/bash
# Walk build A/B (tools/gpu/agg_ab2.sh) then the HBM traffic per order of config 2's grouped aggregate
# launches: k_seq_sweep + k_side + the k_agg kernels + the continuation summed per 32-batch group.
set -o pipefail
bash tools/gpu/agg_ab2.sh $1 &&
bash tools/gpu/pmc_traffic_wl.sh $1 c2 'k_seq_sweep|k_side|k_agg|k_match_reg' 2097152 252 'k_side|k_agg' 4
