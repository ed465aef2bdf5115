set -o pipefail
O=gpurun_out/occ1; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hot_path.py -m gpu -k "occ" > $O/pytest_hot.log 2>&1 || { tail -30 $O/pytest_hot.log; exit 1; }
tail -3 $O/pytest_hot.log
for r in 1 2; do
 for cfg in "list:ME_AGG_LADDER=256" "scan:ME_AGG_LADDER=32768 ME_LW_OCC=0" "occ:ME_AGG_LADDER=32768 ME_LW_OCC=256"; do
  n=${cfg%%:*}; e=${cfg#*:}
  env $e timeout -k 10 300 python3 bench.py --workload c4 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --no-fills-check > $O/c4_$n.$r.json 2> $O/c4_$n.$r.err || { echo FAIL $n; tail -5 $O/c4_$n.$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4_$n.$r.json')); print('$n r$r %.2f M/s step %.3f ms' % (d['value']/1e6, d['ms_per_step']))"
 done
done
