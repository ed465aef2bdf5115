# Randomized GPU soak of the round-6 build: the cancel-walk fuzz, the agg / pool / far-arena fuzzers and the
# hot-path tests at ME_FUZZ_SEEDS seeds (default 200), one pytest process.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}
T=${1:-soak6}; mkdir -p gpurun_out/$T
ME_FUZZ_SEEDS=${SEEDS:-200} timeout -k 10 1000 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  tests/test_agg_cancels.py tests/test_gpu_fuzz.py tests/test_chunk_pool.py tests/test_far_arena.py tests/test_hot_path.py -m gpu \
  > gpurun_out/$T/fuzz.log 2>&1; rc=$?; tail -2 gpurun_out/$T/fuzz.log; exit $rc
