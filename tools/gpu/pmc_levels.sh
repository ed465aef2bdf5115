#!/bin/bash
# SQ counters of config 4's post-walk kernels (instruction mix, waves, waits), one pass
set -o pipefail
O=gpurun_out/pl; mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS --kernel-include-regex "k_agg_levels|k_agg_group|k_agg_walk" --output-format csv -d $O/pmc -o pmc -- python3 bench.py --workload c4 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-fills-check > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
ls $O/pmc
