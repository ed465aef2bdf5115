#!/bin/bash
# deep-window parity (hot path, configs 1 and 4, agg fuzz) + config 4 bench and kernel trace
set -o pipefail
O=gpurun_out/${1:-lv}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_hot_path.py tests/test_gpu_parity.py tests/test_gpu_fuzz.py -m gpu -k "hot or agg or config4 or config1 or fuzz" > $O/pytest.log 2>&1 || { grep -E "^E |FAILED" $O/pytest.log | head -20; tail -3 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --workload c4 --steps 8 --warmup 2 --no-cpu-baseline --no-e2e --no-fills-check > $O/c4.$r.json 2> $O/c4.$r.err || { echo FAIL c4; tail -5 $O/c4.$r.err; exit 1; }
  python3 -c "import json; d=json.load(open('$O/c4.$r.json')); print('c4 r$r %.2f M/s step %.3f ms' % (d['value']/1e6, d['ms_per_step']))"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o kt -- python3 bench.py --workload c4 --steps 4 --warmup 2 --no-cpu-baseline --no-e2e --no-fills-check > $O/tr.json 2> $O/tr.err || { echo TRFAIL; exit 1; }
python3 - $O <<'PY'
import csv,collections,re,sys
rows=list(csv.DictReader(open(sys.argv[1]+'/tr/kt_kernel_trace.csv')))
rows.sort(key=lambda r:int(r['Start_Timestamp']))
d=collections.defaultdict(list)
for r in rows:
    m=re.search(r'(k_\w+(<\w+>)?)\(',r['Kernel_Name'])
    if m: d[m.group(1)].append((int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1e3)
for k in d:
    if k.startswith('k_agg') or 'k_match' in k: print(k, [round(x) for x in d[k][-4:]])
PY
