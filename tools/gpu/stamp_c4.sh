# Phase stamps of config 4 (stamps build): the hot path, then (GENERIC=1) the generic kernel alone.
set -o pipefail
O=gpurun_out/stamp_c4; mkdir -p $O
export ME_ENGINE_LIB=$PWD/matching_engine_amd/build/libme_engine_stamps.so
timeout -k 10 300 python tools/stamp_probe.py --config 4 --seed-top 20 --batches 12 --skip 4 > $O/hot.txt 2>&1
rc=$?
if [ $rc -eq 0 ] && [ -n "$GENERIC" ]; then
  ME_HOT_MIN=0 timeout -k 10 300 python tools/stamp_probe.py --config 4 --seed-top 20 --batches 12 --skip 4 > $O/generic.txt 2>&1
  rc=$?
fi
cat $O/*.txt | grep -v amdgpu.ids; exit $rc
