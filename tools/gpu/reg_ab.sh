set -o pipefail
mkdir -p gpurun_out/regab
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_hot_path.py -x -q -p no:cacheprovider --timeout 240 --timeout-method thread > gpurun_out/regab/pytest.log 2>&1 || { tail -30 gpurun_out/regab/pytest.log; exit 1; }
tail -2 gpurun_out/regab/pytest.log
WL=c3 bash tools/gpu/ab.sh c3ab 2 matching_engine_amd/build/libme_ab_base.so matching_engine_amd/build/libme_ab_cur.so matching_engine_amd/build/libme_ab_g32.so &&
WL=c2 bash tools/gpu/ab.sh c2ab 1 matching_engine_amd/build/libme_ab_base.so matching_engine_amd/build/libme_ab_cur.so matching_engine_amd/build/libme_ab_g32.so
