set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/st4b
export ME_ENGINE_LIB=$GRAFT_REPO_ROOT/matching_engine_amd/build/libme_engine_stamps.so
timeout -k 10 400 python tools/stamp_probe.py --config 4 --seed-top 1000 --batches 8 --skip 2 > gpurun_out/st4b/c4.txt 2>&1; rc=$?; cat gpurun_out/st4b/c4.txt; exit $rc
