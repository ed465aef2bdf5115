#!/bin/bash
# PC samples (host-trap, time-based) of config 4's hot wave: where the k_match_hot record loop spends
# its time, instruction by instruction. usage: tools/gpu/pcsamp_c4.sh TAG
set -o pipefail
TAG=${1:-pcs}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 --kernel-include-regex k_match_hot --output-format csv -d $O/pcs -o pcs -- python3 bench.py --workload c4 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e > $O/run.log 2>&1 || { echo PCS_FAIL; tail -20 $O/run.log; exit 1; }
find $O/pcs -name "*.csv" | head; ls -la $(find $O/pcs -name "*pc_sampling*" | head -3)
