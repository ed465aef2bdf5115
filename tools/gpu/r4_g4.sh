# round-4 iteration: parity (agg groups, fuzz, parity, cluster), then same-box A/Bs and the c3 cluster leg
set -o pipefail
O=gpurun_out/r4_g4; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -m gpu tests/test_agg_groups.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_multirank.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "^E |FAILED" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
bash tools/gpu/ab.sh r4_g4/wpe 2 matching_engine_amd/build/ab/libme_wpe5.so matching_engine_amd/build/ab/libme_wpe6.so matching_engine_amd/build/ab/libme_wpe8.so || exit 1
for r in 1 2; do
  for side in 0 1; do
    ME_SIDE_STREAM=$side timeout -k 10 120 python3 bench.py --steps 320 --warmup 32 --no-cpu-baseline --no-e2e > $O/side$side.$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('$O/side$side.$r.json')); print('side=$side r$r', round(d['value']/1e6,1), 'M/s')"
  done
  K=320 W=32 bash tools/gpu/ab.sh r4_g4/prio 1 matching_engine_amd/build/ab/libme_prio0.so || exit 1
done
timeout -k 10 400 python bench.py --workload c3 --steps 20 --warmup 4 --no-cpu-baseline --no-e2e > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print(round(d['value']/1e6,1), json.dumps(d['cluster']))"
