# rank 0's split + merge on the GPU box's host (no GPU work): library A vs B, alternating
set -o pipefail
cd ${GRAFT_REPO_ROOT:-.}; mkdir -p gpurun_out/r0ab
for r in 1 2 3; do
  for L in "$@"; do
    ME_ENGINE_LIB=$PWD/$L timeout -k 10 300 python tools/rank0_probe.py > gpurun_out/r0ab/$(basename $L .so).$r.json 2>/dev/null || exit 1
    python3 -c "import json; d=json.load(open('gpurun_out/r0ab/$(basename $L .so).$r.json')); print('$(basename $L .so) r$r', ' '.join('W%d %.2f ms' % (x['world'], x['split_plus_merge_ms']) for x in d['rows']))"
  done
done
