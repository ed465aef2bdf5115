set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/st4
export ME_ENGINE_LIB=$GRAFT_REPO_ROOT/matching_engine_amd/build/libme_engine_stamps.so
timeout -k 10 400 python tools/stamp_probe.py --config 4 --seed-top 1000 --batches 12 --skip 2 > gpurun_out/st4/c4.txt 2>&1; rc=$?; cat gpurun_out/st4/c4.txt; [ $rc -eq 0 ] &&
timeout -k 10 200 python tools/stamp_probe.py --config 2 --batches 30 --skip 5 > gpurun_out/st4/c2.txt 2>&1; rc=$?; cat gpurun_out/st4/c2.txt; exit $rc
