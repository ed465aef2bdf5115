set -o pipefail
bash tools/gpu/record.sh close4c traffic:c2 dram:c2 || exit 1
mkdir -p gpurun_out/close4c
ME_FUZZ_SEEDS=200 timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread tests/test_gpu_fuzz.py tests/test_far_arena.py tests/test_hot_path.py -m gpu > gpurun_out/close4c/fuzz200.log 2>&1; rc=$?; tail -2 gpurun_out/close4c/fuzz200.log; exit $rc
