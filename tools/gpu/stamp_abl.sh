# Config-4 hot-wave cycles of the ablation builds (stamps + HOT_ABL bits): what each class of HBM
# stores costs the chain. usage: tools/gpu/stamp_abl.sh "0 31 3 4"
set -o pipefail
O=gpurun_out/stamp_abl; mkdir -p $O
for v in $1; do
  ME_ENGINE_LIB=$PWD/matching_engine_amd/build/libme_engine_stamps_abl$v.so timeout -k 10 200 python tools/stamp_probe.py --config 4 --seed-top 20 --batches 10 --skip 4 > $O/abl$v.txt 2>&1 || { echo "abl$v failed"; tail -5 $O/abl$v.txt; exit 1; }
  echo "abl$v: $(grep 'slowest wave per batch' $O/abl$v.txt)"
done
