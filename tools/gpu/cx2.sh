set -o pipefail
mkdir -p gpurun_out/cx2
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_agg_cancels.py -m gpu -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/cx2/pytest.log 2>&1
rc=$?; tail -5 gpurun_out/cx2/pytest.log; grep -E "^E |FAILED" gpurun_out/cx2/pytest.log | head -20; [ $rc -ne 0 ] && exit $rc
for spec in "ME_GW_CANCEL=1 c5" "ME_GW_CANCEL=0 c5" "c5" "c2"; do
  envs=(); rest=()
  for t in $spec; do if [[ $t == *=* ]]; then envs+=("$t"); else rest+=("$t"); fi; done
  n=$(echo "$spec" | tr ' =' '__')
  env "${envs[@]}" timeout -k 10 300 python3 bench.py --workload ${rest[0]} --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > gpurun_out/cx2/b_$n.json 2> gpurun_out/cx2/b_$n.err || { echo "BENCH_FAIL $spec"; tail -5 gpurun_out/cx2/b_$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/cx2/b_$n.json')); print('$spec', round(d['value']/1e6,1), 'M/s handoffs', d['handoffs_rank0'], d['roofline']['paths'], 'fills_ok', d['fills_check_rank0']['mismatched_batches'] if d['fills_check_rank0'] else None)"
done
