set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/cxst
export ME_ENGINE_LIB=$GRAFT_REPO_ROOT/matching_engine_amd/build/libme_engine_stamps.so
for c in 5 2; do
ME_GW_CANCEL=1 timeout -k 10 300 python tools/cx_probe.py --config $c > gpurun_out/cxst/c$c.txt 2>&1 || { cat gpurun_out/cxst/c$c.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/cxst/c$c.txt
done
