#!/bin/bash
# Session check: full -m gpu suite, two driver-shaped benches (--steps 20 --warmup 5), one default
# bench, and a kernel trace of the driver shape. usage: tools/gpu_s2.sh TAG
set -o pipefail
TAG=${1:-s2}
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b20_$i.json 2>$O/b20.err || { tail $O/b20.err; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2>$O/bench.err || { tail $O/bench.err; exit 1; }
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/bench_prof.json 2>$O/err.log || exit 1
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("b20_1", "b20_2", "bench"):
    d = json.load(open(f"{o}/{f}.json"))
    print(f, round(d["value"] / 1e6, 1), "M orders/s; e2e", round((d.get("e2e_host_path_orders_per_s_rank0") or 0) / 1e6, 1))
PY
