set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/hotst
export ME_ENGINE_LIB=$GRAFT_REPO_ROOT/matching_engine_amd/build/libme_engine_stamps.so
for c in 1 4; do
timeout -k 10 300 python tools/hot_probe.py --config $c > gpurun_out/hotst/c$c.txt 2>&1 || { cat gpurun_out/hotst/c$c.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/hotst/c$c.txt
done
