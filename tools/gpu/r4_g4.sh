set -o pipefail
O=gpurun_out/r4_g4; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q -p no:cacheprovider --timeout 240 --timeout-method thread -m gpu tests/test_agg_groups.py tests/test_gpu_fuzz.py tests/test_gpu_parity.py tests/test_multirank.py > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; grep -E "^E |FAILED" $O/pytest.log | head -20
[ $rc -eq 0 ] || exit 1
bash tools/gpu/ab.sh r4_g4 2 matching_engine_amd/build/ab/libme_wpe5.so matching_engine_amd/build/ab/libme_wpe6.so matching_engine_amd/build/ab/libme_wpe8.so || exit 1
timeout -k 10 400 python bench.py --workload c3 --steps 20 --warmup 4 --no-cpu-baseline --no-e2e > $O/c3.json 2> $O/c3.err || { tail -20 $O/c3.err; exit 1; }
python -c "import json;d=json.load(open('$O/c3.json'));print(round(d['value']/1e6,1), json.dumps(d['cluster']))"
