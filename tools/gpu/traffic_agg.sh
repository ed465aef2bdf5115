#!/bin/bash
# HBM traffic per batch of configs 1 and 4 with the aggregate hot path: k_match plus the batch's k_agg_*
# kernels (and k_match_hot_cont) summed per batch (FETCH_SIZE / WRITE_SIZE passes).
set -o pipefail
TAG=${1:-traffic_agg}
bash tools/gpu/pmc_traffic_wl.sh $TAG c4 'k_match|k_agg' 65536 12 'k_agg|k_match_hot_cont' 12 &&
bash tools/gpu/pmc_traffic_wl.sh $TAG c1 'k_match|k_agg' 62500 10 'k_agg|k_match_hot_cont' 10
