#!/usr/bin/env python3
"""bench.py — orders matched/sec of the MI355X batched matching core (BASELINE.json metric).

Workload (BASELINE.json configs[1]): 1,024 symbols per GPU, uniform
synthetic stream (80% LIMIT at mid +-32 ticks / 20% MARKET, qty U[1,100]), 65,536-order batches
per GPU. With N GPUs the global stream has 1,024*N symbols and 65,536*N-order batches,
hash-sharded by symbol (splitmix64(symbol) % N) with no cross-GPU matching: weak scaling.

One step = one batch through the whole device pipeline (bucket by symbol -> match -> tape
compaction; L > 128: sort -> match -> compaction) with the batch already resident in HBM. W warmup
steps, then K timed steps bracketed by barrier + device sync; the max over ranks is the job time.
--workload c1|c3|c4|c5 runs the other BASELINE configs as secondary lines (same JSON shape); c1 adds
c1_paths: the reference's per-order SubmitOrder + SQLite path, the build's SubmitOrder -> slice ->
GPU -> batched-ingest path and the CPU oracle, on the C1 1M-order stream.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c1|c2|c3|c4|c5]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N   (one rank per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import matching_engine_amd as me  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
BYTES_PER_ORDER = 48   # 32 B record read + 16 B resting insert / cancel
BYTES_PER_FILL = 48    # 32 B tape record + 16 B maker-slot RMW


# Per-workload shape. Weak scaling: symbols and batch grow with N, except config 4
# whose 100k Zipf symbols are global (symbol 0 alone draws ~13 % of the stream at every N).
WORKLOADS = {
    # c1: one book carries every record, so the engine runs it as a hot symbol of a 256-level window
    # (the sort path, the aggregate hot-symbol kernels of me_agg.hip) instead of the 128-level register
    # kernel, whose one wave per symbol is a serial chain of ~0.8 us per record
    "c1": dict(preset=1, symbols_per_gpu=1, batch_per_gpu=62500, levels=256,
               text="BASELINE configs[0]: one symbol 'SYM', 80% LIMIT +-32 ticks / 20% MARKET, qty U[1,100], "
                    "62,500-order batches (the C1 1M-order stream); with the reference-path, service-path and "
                    "oracle timings of SURVEY.md \u00a78(d) C1 in c1_paths"),
    "c2": dict(preset=2, symbols_per_gpu=1024, batch_per_gpu=65536,
               text="BASELINE configs[1]: 1,024 symbols/GPU x uniform stream, 65,536-order batches/GPU, "
                    "80% LIMIT +-32 ticks / 20% MARKET, qty U[1,100]"),
    "c3": dict(preset=3, symbols_per_gpu=12500, batch_per_gpu=131072,
               text="BASELINE configs[2] per-GPU share: 12,500 symbols/GPU (100k at N=8), 131,072-order "
                    "batches/GPU (1M at N=8), uniform stream, hash-sharded"),
    "c4": dict(preset=4, symbols=100_000, batch_per_gpu=65536, seeded=1000, per_side=10_000,
               text="BASELINE configs[3]: Zipf(1.1) popularity over 100k symbols, L=32,768-level windows, "
                    "LIMIT +-5,000 ticks; the 1,000 most popular books pre-seeded to 10,000 levels/side "
                    "(20M resting orders) before warmup"),
    "c5": dict(preset=5, symbols_per_gpu=1024, batch_per_gpu=65536,
               text="BASELINE configs[4]: 1,024 symbols/GPU, 60% cancels of live orders, 25% LIMIT, "
                    "15% MARKET sweeping U[1,20] x 100 qty"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=640)
    ap.add_argument("--warmup", type=int, default=32)
    ap.add_argument("--workload", default="c2", choices=sorted(WORKLOADS),
                    help="c2 (default) = BASELINE configs[1], the metric's workload; c3/c4/c5 = the other "
                         "BASELINE configs as secondary lines (DESIGN.md §7)")
    ap.add_argument("--symbols-per-gpu", type=int, default=None)
    ap.add_argument("--levels", type=int, default=None,
                    help="window L override (experiments: L > 128 runs the sort path; with ME_HOT_MIN=1 every "
                         "symbol takes the aggregate hot-symbol path)")
    ap.add_argument("--batch-per-gpu", type=int, default=None)
    ap.add_argument("--seq-ring", type=int, default=1 << 28,
                    help="me_config.seq_ring (seq-ring entries for cancels; 2^28 is the engine default)")
    ap.add_argument("--batches-per-launch", type=int, default=0,
                    help="batches matched per kernel launch (me_config.batches_per_launch; 0 = engine default 32)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="bounded CPU-baseline sample")
    ap.add_argument("--cpu-threads-sweep", default="1,16,64,128,256",
                    help="thread counts of the native CPU baseline (every core of the affinity mask is added, "
                         "SURVEY.md §8(d)); value = the best")
    ap.add_argument("--cpu-warmup", type=int, default=4, help="untimed stream batches before the CPU sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-fills-check", action="store_true", help="skip the post-run oracle check of the last group")
    ap.add_argument("--fills-check-max", type=int, default=24_000_000,
                    help="largest oracle replay (orders) to check (config 4's 20M seeded orders included)")
    ap.add_argument("--e2e-steps", type=int, default=384,
                    help="batches through the pipelined host path (me_submit_host/me_collect) after the timed loop")
    ap.add_argument("--timing-every", type=int, default=4,
                    help="HIP events on every k-th match launch of the timed loop (each timed launch costs "
                         "the stream a few us; 1 = every launch, 0 = off)")
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="nccl (RCCL, one rank per GPU: the real run); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--cluster-steps", type=int, default=None,
                    help="global slices run after the timed loop through the C++ sharded deployment "
                         "(include/me_cluster.h: split on rank 0, RCCL scatter, match, RCCL gather of tapes and "
                         "results, merge by taker seq); reported beside value, never in it. Default: 16 at N > 1 "
                         "or with --workload c3, else 0. c3's slices have config 3's global shape (1,048,576 "
                         "orders over 100,000 symbols) at every N")
    ap.add_argument("--traffic-from", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"),
                    help="JSON {bytes_per_order: ...} from tools/gpu/pmc_traffic_wl.sh for roofline.traffic (c2; the "
                         "k_match_reg measurement when the engine runs c2 without grouped aggregate launches)")
    args = ap.parse_args()
    args.cpu_threads_sweep = [int(t) for t in args.cpu_threads_sweep.split(",") if t]
    # a shape override makes a c3 run an experiment: its cluster leg (config 3's fixed global slice shape)
    # then runs only when asked for with --cluster-steps
    args.shape_override = any(v is not None for v in (args.symbols_per_gpu, args.batch_per_gpu, args.levels))
    w = WORKLOADS[args.workload]
    if args.symbols_per_gpu is None:
        args.symbols_per_gpu = w.get("symbols_per_gpu", 0)
    if args.batch_per_gpu is None:
        args.batch_per_gpu = w["batch_per_gpu"]
    if args.levels is not None:
        w["levels"] = args.levels
    return args


def _wl_levels(w):
    """The workload's window override (c1), else the preset's."""
    return {"levels": w["levels"]} if "levels" in w else {}


def global_symbols(args, world):
    w = WORKLOADS[args.workload]
    return w["symbols"] if "symbols" in w else args.symbols_per_gpu * world


def progress(msg):
    """A progress line on stderr (long phases — config 4's seeding, the CPU sweep — print as they go)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def dist_setup(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    import torch

    if world > 1:
        import torch.distributed as dist

        if args.dist_backend == "gloo":  # rehearsal of the N>1 path with ranks sharing one GPU
            local = local % max(torch.cuda.device_count(), 1)
            torch.cuda.set_device(local)
            dist.init_process_group("gloo")
        else:  # one rank per GPU over RCCL
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    return world, rank, local


def barrier_sync(world, local):
    import torch

    torch.cuda.synchronize(local)
    if world > 1:
        import torch.distributed as dist

        dist.barrier()
        torch.cuda.synchronize(local)


def allreduce(v, world, op, local):
    if world == 1:
        return v
    import torch
    import torch.distributed as dist

    dev = "cpu" if dist.get_backend() == "gloo" else f"cuda:{local}"
    t = torch.tensor([v], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=op)
    return float(t.item())


def build_rank_batches(args, world, rank, nbatches, n_whole=0):
    """Global stream, hash-sharded; this rank's batches with local symbol ids (and, per batch, the
    positions of its records in the global batch); then n_whole more global batches left whole (the
    cluster leg's slices)."""
    w = WORKLOADS[args.workload]
    S = global_symbols(args, world)
    sc = me.preset(w["preset"], num_symbols=S, batch=args.batch_per_gpu * world, **_wl_levels(w))
    st = me.Stream(sc)
    base = st.base_prices()
    shard, local, members = me.shard_table(S, world)
    ids = members[rank]
    seeds = []
    if w.get("seeded"):  # config 4: deep pre-seeded books of the most popular symbols (not timed)
        progress(f"generating the seeded books of {w['seeded']} symbols")
        sb = st.seed_books(range(w["seeded"]), w["per_side"])
        sel = np.nonzero(shard[sb.symbol] == rank)[0]
        sb = sb.take(sel)
        sb.symbol = np.ascontiguousarray(local[sb.symbol], dtype=np.uint32)
        step = 1 << 20
        seeds = [sb.take(slice(i, i + step)) for i in range(0, len(sb), step)]
    out, pos = [], []
    for _ in range(nbatches):
        b = st.next(sc.batch)
        sel = np.nonzero(shard[b.symbol] == rank)[0]
        lb = b.take(sel)
        lb.symbol = np.ascontiguousarray(local[lb.symbol], dtype=np.uint32)
        out.append(lb)
        pos.append(sel)
    whole = [st.next(sc.batch) for _ in range(n_whole)]
    return sc, base, ids, out, pos, sc.batch * nbatches, seeds, whole


def check_fills(eng, seeds, batches, ids, args):
    """The last launch group's batches (results and tapes) against the oracle replaying the whole stream
    (tests/_parity.py's fields; the oracle is the checker here, after the timed region). Skipped above
    --fills-check-max orders of replay (long runs)."""
    n_replay = sum(len(b) for b in seeds) + sum(len(b) for b in batches)
    if n_replay > args.fills_check_max:
        return {"checked": False, "reason": f"replay of {n_replay} orders > --fills-check-max {args.fills_check_max}"}
    from oracle.oracle import OracleBook

    progress(f"fills check: oracle replay of {n_replay} orders")
    g = eng.last_group_size()
    first = len(batches) - g
    fields = ("filled_qty", "remaining_qty", "fill_count", "tape_offset", "status", "reason")
    ob = OracleBook(len(ids), symbol_ids=ids)  # (fills carry global symbol ids, as the engine's)
    bad, orders, fills = 0, 0, 0
    try:
        for b in seeds:
            ob.submit(b)
        for i, b in enumerate(batches):
            ro, fo = ob.submit(b)
            if i < first:
                continue
            r, f = eng.fetch_group_outputs(i - first, len(b))
            same = len(f) == len(fo) and bool(np.all(f == fo)) and all(bool(np.all(r[x] == ro[x])) for x in fields)
            bad += 0 if same else 1
            orders += len(b)
            fills += len(f)
    finally:
        ob.close()
    return {"checked": True, "batches": g, "orders": orders, "fills": fills, "mismatched_batches": bad,
            "how": "the last launch group's results and tapes vs oracle/oracle_book.cpp replaying the stream"}


def cpu_baseline(args):
    """CPU oracle (oracle/, the scalar price-time book of the build-defined semantics; the reference
    itself has no matcher) on a bounded prefix of the same N=1 stream, natively multi-threaded
    (oracle_book.cpp orc_run_sharded: one std::thread and one book per shard, symbols hash-sharded
    across threads exactly as across GPUs, batches split per thread before the clock starts like the
    GPU's HBM-resident inputs, no Python in the timed loop). Swept over --cpu-threads-sweep thread
    counts (plus every core of the affinity mask); `value` is the best, `sweep` lists them all.
    Every leg first runs the stream's first --cpu-warmup batches (and config 4's seeded books) untimed."""
    from oracle.oracle import OracleBook, run_sharded

    from matching_engine_amd.sharding import ShardPlan

    w = WORKLOADS[args.workload]
    S = global_symbols(args, 1)
    sc = me.preset(w["preset"], num_symbols=S, batch=args.batch_per_gpu, **_wl_levels(w))
    st = me.Stream(sc)
    seeds = st.seed_books(range(w["seeded"]), w["per_side"]) if w.get("seeded") else None
    warm = [st.next(sc.batch) for _ in range(args.cpu_warmup)]
    pre = []  # untimed batches: the seeded books (config 4), then the warm-up batches
    if seeds is not None:
        pre += [seeds.take(np.arange(i, min(i + (1 << 20), len(seeds)))) for i in range(0, len(seeds), 1 << 20)]
    pre += warm
    # k = the batches one thread matches in about --cpu-seconds (the single-core sample, timed per batch)
    progress(f"cpu baseline: {sum(len(b) for b in pre)} untimed orders, then a ~{args.cpu_seconds} s sample on 1 core")
    ob = OracleBook(S)
    for b in pre:
        ob.submit(b)
    timed, t_cpu = [], 0.0
    while t_cpu < args.cpu_seconds:
        b = st.next(sc.batch)
        t0 = time.perf_counter()
        ob.submit(b)
        t_cpu += time.perf_counter() - t0
        timed.append(b)
    ob.close()
    k, done = len(timed), sum(len(b) for b in timed)

    def sharded(T):
        plan = ShardPlan(S, T)
        parts = [[] for _ in range(T)]
        for b in pre + timed:
            for r, (lb, _) in enumerate(plan.split(b)):
                parts[r].append(lb)
        books = [OracleBook(len(plan.members[r])) for r in range(T)]
        wall, _ = run_sharded(books, parts, nwarm=len(pre))
        for bk in books:
            bk.close()
        return done / wall, wall

    allowed = len(os.sched_getaffinity(0))
    ts = sorted({t for t in args.cpu_threads_sweep + [allowed] if 1 <= t <= min(S, allowed)})
    sweep = {}
    for T in ts:
        progress(f"cpu baseline: {T} threads")
        v, wall = sharded(T)
        sweep[str(T)] = {"value": v, "wall_s": round(wall, 4)}
    best = max(sweep, key=lambda t: sweep[t]["value"])
    seeded = f", after seeding {len(seeds)} resting orders" if seeds is not None else ""
    qcpu = cgroup_cpus()
    # the CPUs the threads actually had: never more than the threads, the affinity mask or the job's quota
    cores = min(int(best), allowed, qcpu if qcpu else allowed)
    for t in sweep:
        sweep[t]["cores"] = min(int(t), allowed, qcpu if qcpu else allowed)
    quota = f"a cgroup CPU quota of {qcpu} CPUs" if qcpu else "no cgroup CPU quota"
    return {"value": sweep[best]["value"], "unit": "orders/s", "cores": cores, "threads": int(best), "kind": "port",
            "single_core_value": sweep["1"]["value"] if "1" in sweep else None, "sweep": sweep,
            "sample": f"{k} batches ({done} orders) of the {args.workload} stream after {args.cpu_warmup} untimed "
                      f"warm-up batches{seeded}; oracle/oracle_book.cpp scalar price-time book, one book and one "
                      f"std::thread per shard (orc_run_sharded), symbols hash-sharded; best of threads {ts}, "
                      f"run on {allowed} CPUs of the affinity mask under {quota} (cores = min(threads, quota, mask))"}


def cgroup_cpus():
    """CPUs the job's cgroup quota allows (cpu.max "quota period", rounded up), or None without a quota."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q == "max":
            return None
        return max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        return None


def c1_requests(n: int):
    """The C1 request stream: me_gen config 1 on 'SYM' as raw OrderRequests — 1% of the
    LIMITs re-expressed at scale 2 or 8 to exercise normalisation — and the Q4 records they normalise
    to (seq = the OID each gets on a fresh DB)."""
    sc = me.preset(1, batch=n)
    st = me.Stream(sc)
    base = st.base_prices()
    b = st.next(n)
    otype = ((b.kind >> 2) & 1).astype(np.int32)
    side = (b.kind & 3).astype(np.int32)
    rng = np.random.default_rng(1)
    price, scale = b.price_q4.copy(), np.full(n, 4, dtype=np.int32)
    sel, half = rng.random(n) < 0.01, rng.random(n) < 0.5
    s2, s8 = sel & half & (otype == 0), sel & ~half & (otype == 0)
    price[s2], scale[s2] = b.price_q4[s2] // 100, 2
    price[s8], scale[s8] = b.price_q4[s8] * 10000, 8
    price[otype == 1] = 0
    q4 = price.copy()
    q4[s2] = price[s2] * 100
    q4[s8] = price[s8] // 10000
    rec = me.Batch(np.arange(1, n + 1, dtype=np.uint64), q4, b.qty, np.zeros(n, dtype=np.uint32), b.kind)
    return otype, side, price, scale, b.qty.astype(np.int32), rec, base


def c1_paths(args):
    """C1's three CPU-side timings (rank 0, N = 1): the reference's per-order SubmitOrder with one SQLite
    transaction per order on one core (oracle/ref_submit.cpp, a bounded sample), the build's SubmitOrder
    -> time slices -> GPU match -> one transaction per slice (me_service with its background flusher),
    and the CPU oracle matcher alone on the same records."""
    import ctypes as C
    import sqlite3
    import tempfile

    from matching_engine_amd._abi import MeOrderRequest, MeOrderResponse
    from oracle.oracle import OracleBook, ref_submit_run

    n = 1_000_000
    otype, side, price, scale, qty, rec, base = c1_requests(n)
    tmp = tempfile.mkdtemp(prefix="me_c1_")
    devnull = os.open(os.devnull, os.O_WRONLY)
    out = {}
    # (a) the reference path: calibrate on 5,000 orders, then ~cpu_seconds of it on a fresh DB
    t = time.perf_counter()
    ref_submit_run(os.path.join(tmp, "cal.db"), "C1", "SYM", otype[:5000], side[:5000], price[:5000],
                   scale[:5000], qty[:5000], devnull)
    k = int(min(n, max(5000, 5000 / (time.perf_counter() - t) * args.cpu_seconds)))
    t = time.perf_counter()
    rows, _ = ref_submit_run(os.path.join(tmp, "ref.db"), "C1", "SYM", otype[:k], side[:k], price[:k], scale[:k],
                             qty[:k], devnull)
    dt = time.perf_counter() - t
    out["reference_submitorder"] = {
        "value": k / dt, "unit": "orders/s", "cores": 1, "kind": "reference", "orders": k, "rows": int(rows),
        "what": "SubmitOrder as the reference runs it per order (matching_engine_service.cpp:41-121 + "
                "storage.cpp:78-123: logs to /dev/null with its std::endl flushes, OID, normalize_to_q4, one "
                "SQLite transaction + fresh prepared INSERT per order, WAL / synchronous=NORMAL); no matching"}
    # (b) the build: SubmitOrder -> 1 ms / 65,536-order slices -> GPU match -> one transaction per slice
    reqs = (MeOrderRequest * n)()
    a = np.frombuffer(reqs, dtype=np.dtype([("client", "<u8"), ("symbol", "<u8"), ("otype", "<i4"),
                                            ("side", "<i4"), ("price", "<i8"), ("scale", "<i4"), ("qty", "<i4")]))
    cs, ss = C.create_string_buffer(b"C1"), C.create_string_buffer(b"SYM")
    a["client"], a["symbol"] = C.addressof(cs), C.addressof(ss)
    a["otype"], a["side"], a["price"], a["scale"], a["qty"] = otype, side, price, scale, qty
    resps = (MeOrderResponse * n)()
    lib = me.load()
    eng = me.Engine(1, 128, base, max_batch=65536, max_resting=n + 1024, seq_ring=1 << 22)
    svc = me.MatchingEngineService(eng, ["SYM"], db_path=os.path.join(tmp, "build.db"))
    svc.start(interval_us=1000, slice_orders=65536)
    t = time.perf_counter()
    step = 65536
    for i in range(0, n, step):
        lib.me_service_submit_orders(
            svc.h, C.cast(C.addressof(reqs) + i * C.sizeof(MeOrderRequest), C.POINTER(MeOrderRequest)),
            min(step, n - i), C.cast(C.addressof(resps) + i * C.sizeof(MeOrderResponse), C.POINTER(MeOrderResponse)))
    t_sub = time.perf_counter() - t
    while svc.pending or svc.unpersisted:
        time.sleep(0.0005)
    dt = time.perf_counter() - t
    svc.stop()
    err = svc.last_error()
    con = sqlite3.connect(os.path.join(tmp, "build.db"))
    nrows = con.execute("SELECT COUNT(*) FROM orders").fetchone()[0]
    nfills = con.execute("SELECT COUNT(*) FROM fills").fetchone()[0]
    con.close()
    svc.close()
    eng.close()
    # (c) the oracle matcher alone, one core
    ob = OracleBook(1)
    t = time.perf_counter()
    _, fo = ob.submit(rec)
    dto = time.perf_counter() - t
    ob.close()
    out["build_submitorder_batched"] = {
        "value": n / dt, "unit": "orders/s", "orders": n, "rows": int(nrows), "fill_rows": int(nfills),
        "submit_only_orders_per_s": n / t_sub, "error": err,
        "fills_match_oracle": int(nfills) == 2 * len(fo),
        "what": "me_service_submit_order per request (one thread) -> time slices (1 ms / 65,536 orders, "
                "background flusher) -> me_submit_host / me_collect on the GPU -> one SQLite transaction per "
                "slice (orders rows with their matched status, fills rows, maker updates); clock stops when "
                "every order is matched and committed"}
    out["oracle_matcher"] = {"value": n / dto, "unit": "orders/s", "cores": 1, "kind": "port", "orders": n,
                             "fills": len(fo), "what": "oracle/oracle_book.cpp alone (no SubmitOrder, no SQLite)"}
    os.close(devnull)
    return out


def host_info():
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    quota = None
    try:  # the cgroup's CPU quota ("max" = none) and the affinity mask the CPU baseline's threads run on
        quota = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        pass
    aff = sorted(os.sched_getaffinity(0))
    ranges, i = [], 0
    while i < len(aff):
        j = i
        while j + 1 < len(aff) and aff[j + 1] == aff[j] + 1:
            j += 1
        ranges.append(f"{aff[i]}-{aff[j]}" if j > i else str(aff[i]))
        i = j + 1
    return {"nproc": os.cpu_count(), "cpu_model": model, "cpus_allowed": len(aff), "affinity": ",".join(ranges),
            "cgroup_cpu_max": quota, "cgroup_cpus": cgroup_cpus(), "loadavg": os.getloadavg()}


def cluster_leg(args, world, rank, local, sc, base, slices, n_slices):
    """N > 1: the sharded deployment as a server runs it — rank 0 submits each global slice to
    me_cluster (split by symbol owner, parts scattered over RCCL, matched on every GPU, tapes and results
    gathered back over RCCL and merged by taker seq), two slices in flight; the other ranks serve. Its
    own engines (fresh books), informational: orders/s through the whole round trip, never `value`."""
    from matching_engine_amd.cluster import Cluster

    import torch.distributed as tdist

    transport = "rccl" if (world == 1 or tdist.get_backend() == "nccl") else "tcp"
    port = int(os.environ.get("MASTER_PORT", "29500")) + 11
    cl = Cluster(rank, world, len(base), sc.batch, transport=transport, port=port, device=local, levels=sc.levels,
                 base_prices=base, max_resting=sc.batch * (n_slices + 1), timeout_ms=120000,
                 seq_ring=args.seq_ring, batches_per_launch=2)
    out = None
    if rank == 0:
        t0 = time.perf_counter()
        pend, fills, n = [], 0, 0
        for b in slices:
            pend.append((cl.submit(b), len(b)))
            n += len(b)
            if len(pend) == 2:
                t, k = pend.pop(0)
                fills += len(cl.collect(t, k, copy=False)[1])
        for t, k in pend:
            fills += len(cl.collect(t, k, copy=False)[1])
        dt = time.perf_counter() - t0
        st = cl.stats()
        ph = cl.phases()
        cl.stop()
        out = {"transport": transport, "slices": len(slices), "slice_orders": sc.batch, "symbols": len(base),
               "orders": n, "fills": fills, "orders_per_s": n / dt, "ms_per_slice": dt / len(slices) * 1e3,
               "bytes_rank0": st["bytes"],
               "phase_ms_per_slice_rank0": {k: round(v / len(slices) * 1e3, 4) for k, v in ph.items()},
               "what": "me_cluster_submit / me_cluster_collect (C++, include/me_cluster.h), two slices in flight, "
                       "host slices in and merged host outputs out (the persistence root's view): split on rank 0 "
                       "(its own part packed straight into its engine's pinned slot inputs), grouped "
                       "ncclSend/ncclRecv of the other parts, admission vote (MIN all-reduce), match on every GPU, "
                       "gather of tape lengths, grouped send of tapes + results to rank 0, results back to slice "
                       "order and tapes by taker on rank 0's host (world 1: the slot's outputs in place)"}
    else:
        cl.serve()
    cl.close()
    return out


def main():
    args = parse()
    # the contract is ONE JSON line on stdout: whatever the runtimes print there (RCCL's version banner
    # at its first communicator, library notices) goes to stderr, the line to the saved stdout
    sys.stdout.flush()
    json_out = os.dup(1)
    os.dup2(2, 1)
    world, rank, local = dist_setup(args)
    import torch

    nb = args.warmup + args.steps
    n_cluster = args.cluster_steps if args.cluster_steps is not None else (
        16 if world > 1 or (args.workload == "c3" and not args.shape_override) else 0)
    n_e2e = 0 if args.no_e2e else args.e2e_steps
    sc, gbase, ids, batches, positions, global_orders, seeds, whole = build_rank_batches(
        args, world, rank, nb + n_e2e, 0 if args.workload == "c3" else n_cluster)
    csc, cbase = sc, gbase
    if n_cluster and args.workload == "c3":  # config 3's global slice shape, the same at every N
        csc = me.preset(3, num_symbols=100_000, batch=1 << 20)
        cst = me.Stream(csc)
        cbase = cst.base_prices()
        whole = [cst.next(csc.batch) for _ in range(n_cluster)] if rank == 0 else []
    base = gbase[ids]
    e2e_batches = batches[nb:]
    batches = batches[:nb]
    total_local = sum(len(b) for b in batches + e2e_batches)
    n_seed = sum(len(b) for b in seeds)
    eng = me.Engine(len(ids), sc.levels, base,
                    max_batch=max(len(b) for b in batches + e2e_batches + seeds) + 1,
                    max_resting=max(total_local // 3, sum(len(b) for b in batches)) + n_seed + 65536, seq_ring=args.seq_ring,
                    device=local, symbol_ids=ids, batches_per_launch=args.batches_per_launch)
    if seeds:
        progress(f"seeding {n_seed} resting orders (untimed)")
    for b in seeds:
        eng.submit_batch(b, want_fills=False)
    dbs = [eng.upload(b) for b in batches]
    progress(f"{len(dbs)} batches resident; warmup {args.warmup}, timed {args.steps}")
    for db in dbs[: args.warmup]:
        eng.submit_device(db)
    eng.sync()
    eng.timing_enable(args.timing_every)
    barrier_sync(world, local)
    t0 = time.perf_counter()
    for db in dbs[args.warmup:]:
        eng.submit_device(db)
    t_enq = time.perf_counter() - t0
    eng.sync()
    barrier_sync(world, local)
    t1 = time.perf_counter()
    elapsed = t1 - t0
    tm = eng.timing_read()
    handoffs = eng.stats()["handoffs"]
    adm = eng.admission()  # after the timed region: exact counts taken by submits (0 = never drained)
    orders_local = sum(db.n for db in dbs[args.warmup:])
    import torch.distributed as tdist

    MAX = tdist.ReduceOp.MAX if world > 1 else None
    SUM = tdist.ReduceOp.SUM if world > 1 else None
    job_time = allreduce(elapsed, world, MAX, local)
    orders_all = allreduce(float(orders_local), world, SUM, local)
    fills_all = allreduce(float(tm["fills"]), world, SUM, local)

    # roofline of the dominant kernel (k_match) on this rank, from HIP events on its stream
    # (HIP events on every --timing-every-th launch of the timed loop; one launch matches a group of
    # batches_per_launch batches, so its algorithmic bytes are the timed orders' share of all bytes)
    timed = max(tm["launches"], 1)
    avg_match_s = tm["match_ms"] / 1e3 / timed
    bytes_per_order = (BYTES_PER_ORDER * orders_local + BYTES_PER_FILL * tm["fills"]) / max(orders_local, 1)
    bytes_per_launch = bytes_per_order * tm["orders"] / timed
    achieved = bytes_per_launch / avg_match_s / 1e9
    # roofline.traffic: PMC bytes per order of a steady launch of the same workload (rocprofv3 FETCH_SIZE /
    # WRITE_SIZE passes, tools/gpu_pmc_traffic.sh -> profiles/pmc_traffic[_cN].json) scaled to the orders of
    # THIS run's timed launches, so it and algorithmic_bytes_per_launch describe the same launch shape
    traffic = traffic_per_order = traffic_src = None
    paths = eng.paths()
    tfile = args.traffic_from
    if args.workload == "c2" and not paths["grouped_agg"] and tfile == os.path.join(ROOT, "profiles", "pmc_traffic.json"):
        tfile = os.path.join(ROOT, "profiles", "pmc_traffic_k_match_reg.json")  # (ME_REG_AGG=0)
    if args.workload != "c2":
        tfile = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.workload}.json")
    if tfile and os.path.exists(tfile):
        traffic_per_order = json.load(open(tfile)).get("bytes_per_order")
        traffic_src = os.path.relpath(tfile, ROOT)
        if traffic_per_order:
            traffic = traffic_per_order * tm["orders"] / timed

    # fills check (after the timed region, before anything else runs on the engine): the oracle replays
    # this rank's stream from the start (seeded books, warmup, timed batches) and every batch of the last
    # timed launch group — its results and tape — must equal it bit for bit; the metric's "fills bit-exact"
    # is this check plus the -m gpu parity suite
    fills_check = check_fills(eng, seeds, batches, ids, args) if not args.no_fills_check else None
    bad_all = allreduce(float(fills_check["mismatched_batches"] if fills_check and fills_check["checked"] else 0),
                        world, SUM, local)

    # PCIe-inclusive host path (me_submit_host / me_collect: staging copy into a pinned slot, H2D on
    # its own stream, the grouped pipeline, D2H of results + tape into pinned memory), informational.
    # Each ticket is collected when its slot is needed again (host_slots submissions later).
    e2e = None
    if e2e_batches:
        eng.sync()
        slots = eng.config()["host_slots"]
        eng.host_reserve()  # pinned slots are allocated on first use: a server does it at start-up
        t2 = time.perf_counter()
        n2, f2, pend = 0, 0, []
        for b in e2e_batches:
            if len(pend) == slots:
                _, f = eng.collect(pend.pop(0), copy=False)
                f2 += len(f)
            pend.append(eng.submit_host(b))
            n2 += len(b)
        for t in pend:
            _, f = eng.collect(t, copy=False)
            f2 += len(f)
        e2e = n2 / (time.perf_counter() - t2)
    max_resting = eng.config()["max_resting"]
    for db in dbs:
        db.free()
    eng.close()

    line = None
    if rank == 0:
        cpu = None if (args.no_cpu_baseline or world > 1) else cpu_baseline(args)
        c1 = c1_paths(args) if (args.workload == "c1" and world == 1 and not args.no_cpu_baseline) else None
        line = {
            "metric": "orders matched/sec (whole node); fills bit-exact vs CPU oracle",
            "value": orders_all / job_time,
            "unit": "orders/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": job_time / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": f"synthetic (me_gen config {sc.config} stream, seed {sc.seed})",
            "config": {
                "workload": WORKLOADS[args.workload]["text"],
                "symbols": global_symbols(args, world),
                "global_batch": args.batch_per_gpu * world,
                "levels": sc.levels,
                "parallelism": f"symbol-hash shards x{world} (no cross-GPU matching)",
            },
            "fills_per_order": fills_all / max(orders_all, 1),
            "handoffs_rank0": handoffs,
            "admission_rank0": {"exact_counts": adm["exact_counts"], "resting": adm["resting"],
                                "max_resting": max_resting},
            "kernel_match_ms_avg": tm["match_ms"] / timed,
            "kernel_match_launches_timed": tm["launches"],
            "batches_per_launch": args.batches_per_launch or (32 if sc.levels <= 128 else 1),
            # start-to-start device time per batch between the first and last timed launches (needs two)
            # the match pipeline's device time per batch: the steady launch-to-launch time with two or more
            # timed launches, else the one timed launch group's event-timed duration / the batches it matched
            # (no fill or drain launch in either)
            "device_ms_per_step": tm["pipeline_ms"] if tm["launches"] >= 2 else (
                tm["match_ms"] / (tm["orders"] / (orders_local / args.steps)) if tm["orders"] and orders_local else None),
            "host_enqueue_ms_per_step_rank0": t_enq / args.steps * 1e3,
            "e2e_host_path_orders_per_s_rank0": e2e,
            "fills_check_rank0": fills_check,
            "fills_check_mismatched_batches_all_ranks": int(bad_all),
            "cluster": None,
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": traffic,
                # the timed launch: k_match_reg, or with grouped_agg the group's aggregate-path kernels
                # (k_side, k_agg_gwalk ... k_agg_gemit, the continuation) between the same two events
                "kernel": ("k_agg group" if paths["grouped_agg"] else "k_match_reg") if sc.levels <= 128 else "k_match",
                "paths": paths,
                "algorithmic_bytes_per_launch": bytes_per_launch,
                "algorithmic_bytes_per_order": bytes_per_order,
                "traffic_bytes_per_order": traffic_per_order,
                "traffic_source": traffic_src,
            },
            "cpu_baseline": cpu,
            "host": host_info(),
            "build": me._abi.load().me_build_info().decode(),  # source digest of the library that ran
            "c1_paths": c1,
        }
    if n_cluster:
        # the sharded deployment after the timed loop; a watchdog keeps a stuck collective from eating
        # the run: past the limit, rank 0 prints the line without the leg and every rank exits
        import threading

        def expire():
            if rank == 0:
                line["cluster"] = {"error": "cluster leg timed out (180 s)"}
                os.write(json_out, (json.dumps(line) + "\n").encode())
            os._exit(0)

        wd = threading.Timer(180.0, expire)
        wd.daemon = True
        wd.start()
        try:
            got = cluster_leg(args, world, rank, local, csc, cbase, whole, n_cluster)
        except Exception as ex:  # reported, never fatal to the measured line
            got = {"error": f"{type(ex).__name__}: {ex}"}
        wd.cancel()
        if rank == 0:
            line["cluster"] = got
    if rank == 0:
        os.write(json_out, (json.dumps(line) + "\n").encode())
    if world > 1:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
