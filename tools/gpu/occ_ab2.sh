set -o pipefail
O=gpurun_out/occ2; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hot_path.py tests/test_gpu_parity.py -m gpu -k "hot or agg or config4 or config1" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
 for v in 0 64; do
  ME_LW_OCC=$v timeout -k 10 300 python3 bench.py --workload c1 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-fills-check > $O/c1_occ$v.$r.json 2> $O/c1_occ$v.$r.err || { echo FAIL c1 $v; tail -5 $O/c1_occ$v.$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c1_occ$v.$r.json')); print('c1 occ=$v r$r %.3f M/s step %.3f ms' % (d['value']/1e6, d['ms_per_step']))"
 done
done
bash tools/gpu/record.sh occ2 trace:c4:4:2
