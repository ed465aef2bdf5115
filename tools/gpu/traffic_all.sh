set -o pipefail
T=traffic3
bash tools/gpu/pmc_traffic_wl.sh $T c2 k_match_reg $((32*65536)) 320 &&
bash tools/gpu/pmc_traffic_wl.sh $T c3 k_match_reg $((32*131072)) 160 &&
bash tools/gpu/pmc_traffic_wl.sh $T c5 k_match_reg $((32*65536)) 320 &&
bash tools/gpu/pmc_traffic_wl.sh $T c4 "k_match" 65536 12 k_match_hot 12
