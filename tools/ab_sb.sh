set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/absb; mkdir -p $O
for v in base sba sbb sbc sbd; do
  if [ $v = base ]; then L=""; else L=matching_engine_amd/build/ab/libme_$v.so; fi
  ME_ENGINE_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/p_$v -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/$v.json 2>$O/$v.err || exit 1
  python3 tools/last_trace.py $O/p_$v 8 | grep k_side > $O/$v.side
  echo $v $(python3 -c "import json; print(round(json.load(open('$O/$v.json'))['value']/1e6,1))") $(cat $O/$v.side | awk '{print $2}' | tr '\n' ' ')
done
