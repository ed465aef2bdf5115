#!/bin/bash
# Driver-shaped bench (--steps 20 --warmup 5), alternating the in-tree library and a variant
# (matching_engine_amd/build/ab/libme_$1.so), N rounds: value, kernel ms, ms per step.
V=$1; N=${2:-6}
for i in $(seq 1 $N); do
  for v in base $V; do
    if [ $v = base ]; then L=""; else L=matching_engine_amd/build/ab/libme_$v.so; fi
    ME_ENGINE_LIB=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e 2>/dev/null | python3 -c "import json,sys; d=json.load(sys.stdin); print('$v', round(d['value']/1e6,1), round(d['kernel_match_ms_avg'],3), round(d['ms_per_step'],4))" || exit 1
  done
done
