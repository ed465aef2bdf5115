#!/bin/bash
# The measurement record of the current build, in parameterised steps (each GPU step under its own time
# limit; the first failure ends the call). Outputs under gpurun_out/TAG/; copy what DESIGN.md cites into
# profiles/ (profiles/INDEX.md lists them with the build digest).
#
#   tools/gpu/record.sh TAG STEP [STEP ...]
#   STEP:  tests                 the -m gpu suite (pytest -x, per-test timeout) + smoke
#          bench[:WL[:K[:W]]]    bench.py line (default c2, the driver's --steps 20 --warmup 5)
#          trace[:WL[:K[:W]]]    rocprofv3 --kernel-trace --stats of that bench; per-kernel summary
#          traffic[:WL]          FETCH_SIZE and WRITE_SIZE passes (one counter each) over the match group's
#                                kernels -> pmc_traffic_WL.json (bytes per order, gfx950 FETCH x2 correction)
#          dram[:WL]             byte-exact EA traffic (32-B-unit read / write / atomic request counters, one pass)
#          sq[:WL]               SQ counters (instructions, waits, LDS bank conflicts) of the agg kernels
#          cpu[:WL]              bench.py with the CPU baseline at the host's cores (and 1 core)
# env: BENCH_ARGS (extra bench.py args), ME_* engine switches pass through.
set -o pipefail
TAG=$1
shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $R
# the match group's kernels (the grouped aggregate path and k_match_reg) + the pipeline's side launches
KRE='k_agg|k_match_reg|k_side|k_seq_sweep|k_match|k_sort|k_tape|k_hot'

bench_cmd() {  # WL K W
  echo "python3 $R/bench.py --workload $1 --steps $2 --warmup $3 --no-cpu-baseline --no-e2e --no-fills-check $BENCH_ARGS"
}

for step in "$@"; do
  IFS=: read -r what wl k w <<< "$step"
  wl=${wl:-c2}; k=${k:-20}; w=${w:-5}
  case $what in
  tests)
    timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
    tail -1 $O/smoke.log
    timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
    rc=$?; tail -2 $O/pytest_gpu.log
    if [ $rc -ne 0 ]; then echo TESTS_FAIL; grep -E "^E |FAILED|Error" $O/pytest_gpu.log | head -30; exit 1; fi
    ;;
  bench)
    timeout -k 10 400 python3 bench.py --workload $wl --steps $k --warmup $w $BENCH_ARGS > $O/bench_${wl}_$k.json 2> $O/bench_${wl}_$k.err || { echo "BENCH_FAIL $wl"; tail -20 $O/bench_${wl}_$k.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/bench_${wl}_$k.json')); print('$wl K=$k', round(d['value']/1e6,1), 'M/s', d['build'], 'frac', round(d['roofline']['frac'],4))"
    ;;
  trace)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace_${wl}_$k -o kt -- $(bench_cmd $wl $k $w) > $O/trace_${wl}_$k.json 2> $O/trace_${wl}_$k.err || { echo "TRACE_FAIL $wl"; tail -20 $O/trace_${wl}_$k.err; exit 1; }
    python3 $R/tools/prof_summary.py trace $O/trace_${wl}_$k --steps $k > $O/trace_${wl}_$k.txt && cat $O/trace_${wl}_$k.txt
    ;;
  traffic)
    # (config 4: its 20 seeding batches run through the same kernels before the warmup — dropped with
    # --from-sweep 20; config 3: no cluster leg, whose separate engines would add their dispatches)
    FS=""; XA=""
    [ $wl = c4 ] && FS="--from-sweep 20"
    [ $wl = c3 ] && XA="--cluster-steps 0"
    for c in FETCH_SIZE WRITE_SIZE; do
      timeout -s KILL 300 rocprofv3 --pmc $c --kernel-include-regex "$KRE" --output-format csv -d $O/pmc_${wl}_$c -o pmc -- $(bench_cmd $wl 64 32) $XA > $O/pmc_${wl}_$c.log 2>&1 || { echo "PMC_FAIL $wl $c"; tail -5 $O/pmc_${wl}_$c.log; exit 1; }
    done
    python3 $R/tools/prof_summary.py traffic $O/pmc_${wl}_FETCH_SIZE $O/pmc_${wl}_WRITE_SIZE --bench $O/pmc_${wl}_WRITE_SIZE.log $FS > $O/pmc_traffic_$wl.json && cat $O/pmc_traffic_$wl.json
    ;;
  dram)
    timeout -s KILL 300 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B TCC_EA0_WRREQ_WRITE_ATOMIC_32B TCC_EA0_RDREQ --kernel-include-regex "$KRE" --output-format csv -d $O/dram_$wl -o pmc -- $(bench_cmd $wl 64 32) > $O/dram_$wl.log 2>&1 || { echo "DRAM_FAIL $wl"; tail -5 $O/dram_$wl.log; exit 1; }
    python3 $R/tools/prof_summary.py dram $O/dram_$wl --bench $O/dram_$wl.log > $O/dram_traffic_$wl.json && head -8 $O/dram_traffic_$wl.json
    ;;
  sq)
    KA='k_agg_|k_side|k_match_reg'
    i=0
    for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
               "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_WAVES SQ_WAIT_INST_LDS SQ_INSTS_SMEM SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"; do
      i=$((i + 1))
      timeout -s KILL 300 rocprofv3 --pmc $set --kernel-include-regex "$KA" --output-format csv -d $O/sq_${wl}_$i -o pmc -- $(bench_cmd $wl 64 32) > $O/sq_${wl}_$i.log 2>&1 || { echo "SQ_FAIL $wl $i"; tail -5 $O/sq_${wl}_$i.log; exit 1; }
    done
    python3 $R/tools/prof_summary.py sq $O/sq_${wl}_1 $O/sq_${wl}_2 > $O/sq_$wl.txt && cat $O/sq_$wl.txt
    ;;
  cpu)
    timeout -k 10 600 python3 bench.py --workload $wl --steps $k --warmup $w --no-e2e $BENCH_ARGS > $O/cpu_$wl.json 2> $O/cpu_$wl.err || { echo "CPU_FAIL $wl"; tail -20 $O/cpu_$wl.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/cpu_$wl.json')); c=d['cpu_baseline']; print('$wl GPU', round(d['value']/1e6,1), 'M/s; CPU', round(c['value']/1e6,2), 'M/s on', c['cores'], 'threads; 1 core', round(c.get('single_core_value', c['value'])/1e6,2))"
    ;;
  *) echo "unknown step $step"; exit 2 ;;
  esac
done
