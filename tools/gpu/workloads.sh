set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out/${WL_TAG:-wl}
timeout -k 10 300 python bench.py --workload c3 --steps 320 --warmup 32 --no-e2e --traffic-from '' > gpurun_out/${WL_TAG:-wl}/c3.json 2> gpurun_out/${WL_TAG:-wl}/c3.err && cat gpurun_out/${WL_TAG:-wl}/c3.json &&
timeout -k 10 300 python bench.py --workload c5 --steps 320 --warmup 32 --no-e2e --traffic-from '' > gpurun_out/${WL_TAG:-wl}/c5.json 2> gpurun_out/${WL_TAG:-wl}/c5.err && cat gpurun_out/${WL_TAG:-wl}/c5.json &&
timeout -k 10 400 python bench.py --workload c4 --steps 20 --warmup 5 --no-e2e --traffic-from '' > gpurun_out/${WL_TAG:-wl}/c4.json 2> gpurun_out/${WL_TAG:-wl}/c4.err && cat gpurun_out/${WL_TAG:-wl}/c4.json
