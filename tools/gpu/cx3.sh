set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cx3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_agg_cancels.py -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/cx3/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/cx3/pytest.log; grep -E "^E |FAILED" gpurun_out/cx3/pytest.log | head -20; [ $rc -ne 0 ] && exit $rc
ME_GW_CANCEL=1 timeout -k 10 300 python3 bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/cx3/b5.json 2> gpurun_out/cx3/b5.err || { tail -5 gpurun_out/cx3/b5.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/cx3/b5.json')); print('c5', round(d['value']/1e6,1), 'M/s handoffs', d['handoffs_rank0'], 'fills_ok', d['fills_check_rank0']['mismatched_batches'])"
export ME_ENGINE_LIB=$GRAFT_REPO_ROOT/matching_engine_amd/build/libme_engine_stamps.so
for c in 5 2; do
ME_GW_CANCEL=1 timeout -k 10 300 python tools/cx_probe.py --config $c > gpurun_out/cx3/st$c.txt 2>&1 || { cat gpurun_out/cx3/st$c.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/cx3/st$c.txt
done
