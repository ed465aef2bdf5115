set -o pipefail
mkdir -p gpurun_out/cx1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_agg_cancels.py -m gpu -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > gpurun_out/cx1/pytest.log 2>&1
rc=$?; tail -30 gpurun_out/cx1/pytest.log | grep -E "PASS|FAIL|Error|passed|failed|^E " | head -40; exit $rc
