set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/grst
export ME_ENGINE_LIB=$GRAFT_REPO_ROOT/matching_engine_amd/build/libme_engine_stamps.so
for c in 2 5; do
timeout -k 10 300 python tools/gres_probe.py --config $c > gpurun_out/grst/c$c.txt 2>&1 || { cat gpurun_out/grst/c$c.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/grst/c$c.txt
done
