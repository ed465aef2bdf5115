#!/bin/bash
# Hot path diagnosis: its parity tests on the checking build (libme_engine_hotcheck.so: the lists and
# lane states against the HBM book after every record). usage: tools/gpu_hotcheck.sh TAG [-k EXPR]
set -o pipefail
TAG=${1:-hotcheck}; shift
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp
ME_ENGINE_LIB=$PWD/matching_engine_amd/build/libme_engine_hotcheck.so timeout -k 10 300 python -u -m pytest tests/test_hot_path.py -v -s -p no:cacheprovider --timeout 120 --timeout-method thread "$@" > $O/pytest.log 2>&1
rc=$?
grep -E "HOTCHECK|PASSED|FAILED|Error" $O/pytest.log | head -40
exit $rc
