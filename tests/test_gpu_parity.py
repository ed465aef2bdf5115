"""GPU parity: the HIP engine (through the C-ABI) against the CPU oracle — an unbounded price-time
book — and the committed golden fixtures: bit-exact per-record results, trade tapes and resting
books. Needs an MI355X."""
import os

import numpy as np
import pytest

from tests._parity import (assert_books_equal, assert_fills_equal, assert_results_equal, load_fixture,
                           run_both, side_levels)

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


@pytest.fixture(scope="module")
def orc(built):
    from oracle import oracle

    return oracle


def engine_for(me, S, L, base, max_batch, max_resting, **kw):
    kw.setdefault("seq_ring", 1 << 22)
    return me.Engine(S, L, base, max_batch=max_batch, max_resting=max_resting, **kw)


def no_window_rejects(res, ctx=""):
    """The engine's window and seq ring are invisible: never OUT_OF_WINDOW, BAD_SEQ only for seq 0."""
    assert not np.any(res["reason"] == 3), f"{ctx}: OUT_OF_WINDOW reject"
    assert not np.any(res["reason"] == 6), f"{ctx}: BAD_SEQ reject"


def _rows(me, rows, start_seq=1):
    n = len(rows)
    return me.Batch(np.arange(start_seq, start_seq + n, dtype=np.uint64), [r[4] for r in rows],
                    [r[5] for r in rows], [r[0] for r in rows], [me.kind(r[1], r[2], r[3]) for r in rows])


# ---------------------------------------------------------------- committed fixtures
@pytest.mark.parametrize("cid", [1, 2, 3, 4, 5, 6])
def test_golden_fixture_on_gpu(me, cid):
    meta, batches, res, fills, book = load_fixture(cid)
    mb = max(len(b) for b in batches)
    # deep sparse books (config 4) keep ~one chunk per resting order: size the pool for that
    with engine_for(me, meta["num_symbols"], meta["levels"], meta["base"], mb, 1 << 18, max_chunks=1 << 17) as eng:
        for k, b in enumerate(batches):
            r, f = eng.submit_batch(b)
            assert_results_equal(r, res[k], f"fixture c{cid} b{k}")
            assert_fills_equal(f, fills[k], f"fixture c{cid} b{k}")
        dumps = np.concatenate([eng.dump(s) for s in range(meta["num_symbols"])])
        assert np.array_equal(dumps, book), f"fixture c{cid}: resting book differs"


# ---------------------------------------------------------------- live differential runs
def _stream_run(me, orc, cfg, nbatches, seed_per_side=0, book_symbols=None, eng_kw=None, **over):
    sc = me.preset(cfg, **over)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = []
    if seed_per_side:
        batches.append(st.seed_books(range(sc.num_symbols), seed_per_side))
    batches += [st.next(sc.batch) for _ in range(nbatches)]
    mb = max(len(b) for b in batches)
    total = sum(len(b) for b in batches)
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, mb, total + 1024, max_chunks=total + 2 * sc.num_symbols,
                    **(eng_kw or {})) as eng:
        nf = run_both(eng, ob, batches, book_symbols=book_symbols, ctx=f"config {cfg}")
    return nf, total


def test_config1_single_symbol(me, orc):
    nf, total = _stream_run(me, orc, 1, 4, batch=62500)
    assert nf > 0.5 * total


def test_config2_uniform_1024(me, orc):
    nf, total = _stream_run(me, orc, 2, 8)
    assert nf > 0.5 * total


def test_config3_100k_symbols_two_pass_sort(me, orc):
    nf, total = _stream_run(me, orc, 3, 2, batch=1 << 19, book_symbols=range(0, 100_000, 97))
    assert nf > 0


def test_config4_zipf_deep_books(me, orc):
    nf, total = _stream_run(me, orc, 4, 3, seed_per_side=2000, num_symbols=200, levels=8192, spread_ticks=2500)
    assert nf > 0


def test_config4_bench_shape(me, orc):
    """Config 4 at the bench's shape: L = 32,768-level windows (the HBM-window kernel), the most
    popular books seeded to 10,000 levels per side, Zipf(1.1) symbols, LIMITs +-5,000 ticks."""
    sc = me.preset(4, num_symbols=2000, batch=65536)
    st = me.Stream(sc)
    base = st.base_prices()
    seeds = st.seed_books(range(24), 10_000)
    batches = [seeds.take(slice(i, i + 65536)) for i in range(0, len(seeds), 65536)]
    batches += [st.next(sc.batch) for _ in range(3)]
    total = sum(len(b) for b in batches)
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, 65536, total + 1024, max_chunks=total + 4096) as eng:
        nf = run_both(eng, ob, batches, book_symbols=list(range(24)) + list(range(24, 2000, 61)), ctx="c4 bench")
    assert nf > 0


def test_config4_full_bench_shape(me, orc):
    """Config 4 exactly as the bench runs it on one GPU: 100,000 symbols, the 1,000 most
    popular books seeded to 10,000 levels per side (20M resting orders, matched on both sides without
    comparison), then two 65,536-order batches of the Zipf stream compared record for record and fill for
    fill, and the hot symbols' books."""
    sc = me.preset(4, batch=65536)
    st = me.Stream(sc)
    base = st.base_prices()
    seeds = st.seed_books(range(1000), 10_000)
    step = 1 << 20
    ob = orc.OracleBook(sc.num_symbols)
    total = len(seeds) + 2 * sc.batch
    with engine_for(me, sc.num_symbols, sc.levels, base, step, total + 65536) as eng:
        for i in range(0, len(seeds), step):
            part = seeds.take(slice(i, i + step))
            eng.submit_batch(part, want_fills=False)
            ob.submit(part)
        nf = run_both(eng, ob, [st.next(sc.batch) for _ in range(2)], book_symbols=[0, 1, 2, 3, 500, 999, 54321],
                      ctx="c4 full shape")
    assert nf > 0


def test_deep_window_many_symbols(me, orc):
    """More symbols than one dispatch round of deep-window workgroups, busy and idle alike."""
    nf, total = _stream_run(me, orc, 2, 2, num_symbols=1100, levels=2048, batch=1100 * 80,
                            book_symbols=range(0, 1100, 7))
    assert nf > 0


def test_config5_cancel_heavy_sweeps(me, orc):
    nf, total = _stream_run(me, orc, 5, 8)
    assert nf > 0


# ---------------------------------------------------------------- unbounded prices and seqs
def _drift_stream(me, levels, num_symbols, batch, nbatches, drift_every, drift_step=1, far_pct=1, cancel_pct=10,
                  market_qty_mult=3, seq_start=(1 << 33) + 777):
    sc = me.preset(5, num_symbols=num_symbols, levels=levels, batch=batch, cancel_pct=cancel_pct, market_pct=15,
                   market_qty_mult=market_qty_mult, drift_step=drift_step, drift_every=drift_every,
                   far_pct=far_pct, seq_start=seq_start)
    st = me.Stream(sc)
    return sc, st.base_prices(), [st.next(batch) for _ in range(nbatches)]


def test_drifting_mids_far_limits_big_oids(me, orc):
    """Every symbol's mid trends 10 x L over 200 batches (1 tick every 5 of its records, 32 records
    per symbol per batch), 1 % of LIMITs are priced L..64L away, 10 % cancels, sweeping MARKETs, OIDs
    above 2^33: the 128-level windows re-centre and spill to far levels, and every batch is bit-exact
    against the window-free oracle with no OUT_OF_WINDOW / BAD_SEQ reject."""
    sc, base, batches = _drift_stream(me, 128, 256, 8192, 200, drift_every=5)
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 20) as eng:
        for k, b in enumerate(batches):
            r, f = eng.submit_batch(b)
            ro, fo = ob.submit(b)
            assert_results_equal(r, ro, f"drift b{k}")
            assert_fills_equal(f, fo, f"drift b{k}")
            no_window_rejects(r, f"drift b{k}")
        assert_books_equal(eng, ob, range(sc.num_symbols), "drift")
        assert eng.resting_count() == ob.resting()
    # the stream really left the initial windows: LIMIT prices of the last batch moved ~10 windows
    last = batches[-1]
    lim = ((last.kind >> 2) & 3) == 0
    moved = np.abs(last.price_q4[lim] - base[last.symbol[lim]])
    assert np.median(moved) > 5 * sc.levels


@pytest.mark.parametrize("group", [8, 32])
def test_drifting_stream_device_groups_every_batch(me, orc, group):
    """The drifting far-price stream through back-to-back device batches, `group` per launch: every
    batch of every group is compared with the oracle (me_fetch_group_outputs)."""
    sc, base, batches = _drift_stream(me, 128, 512, 16384, 2 * group, drift_every=3)
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 21, batches_per_launch=group) as eng:
        for g0 in range(0, len(batches), group):
            grp = batches[g0:g0 + group]
            dbs = [eng.upload(b) for b in grp]
            for db in dbs:
                eng.submit_device(db)
            eng.sync()
            assert eng.last_group_size() == len(grp)
            for k, b in enumerate(grp):
                r, f = eng.fetch_group_outputs(k, len(b))
                ro, fo = ob.submit(b)
                assert_results_equal(r, ro, f"group {g0 // group} batch {k}")
                assert_fills_equal(f, fo, f"group {g0 // group} batch {k}")
                no_window_rejects(r)
            for db in dbs:
                db.free()
        assert_books_equal(eng, ob, range(0, sc.num_symbols, 3), "drift groups")
        assert eng.resting_count() == ob.resting()


@pytest.mark.parametrize("group", [16, 32])
def test_symbol_first_seen_late_in_a_group(me, orc, group):
    """A symbol with no records in the first batches of a launch group and records later (a sparse
    symbol): every batch of the group against the oracle. (The per-symbol record count of a group
    once summed only batches 0-7.)"""
    sc = me.preset(2, num_symbols=64, batch=4096)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(group)]
    for k, b in enumerate(batches):
        late = (b.symbol % 8) == 3  # symbols 3, 11, ... only from batch 12 (and 40) on
        if k < 12 or (group > 32 and 20 <= k < 40):
            b.symbol[late] = (b.symbol[late] + 1) % sc.num_symbols
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, (group + 2) * sc.batch,
                    batches_per_launch=group) as eng:
        dbs = [eng.upload(b) for b in batches]
        for db in dbs:
            eng.submit_device(db)
        eng.sync()
        assert eng.last_group_size() == group
        for k, b in enumerate(batches):
            r, f = eng.fetch_group_outputs(k, len(b))
            ro, fo = ob.submit(b)
            assert_results_equal(r, ro, f"late symbols G={group} batch {k}")
            assert_fills_equal(f, fo, f"late symbols G={group} batch {k}")
        assert_books_equal(eng, ob, range(sc.num_symbols), "late symbols")
        for db in dbs:
            db.free()


@pytest.mark.parametrize("levels,nsym,nb,every", [(128, 256, 1200, 100), (1024, 64, 400, 50)])
def test_long_drift_soak(me, orc, levels, nsym, nb, every):
    """A long session: every symbol's mid trends tens of windows (stale orders are left behind as far
    levels, 1 % of LIMITs far away, 10 % cancels, sweeping MARKETs), device batches back to back (32
    per launch on the register kernel; one per launch on the deep-window kernel). Every `every`-th
    batch and the final books against the oracle; no error, no window / seq reject, the far arrays
    never overflow at the default far_levels."""
    sc, base, batches = _drift_stream(me, levels, nsym, 8192, nb, drift_every=5 if levels == 128 else 1,
                                      drift_step=1 if levels == 128 else 8)
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 22, batches_per_launch=32) as eng:
        for g0 in range(0, len(batches), every):
            grp = batches[g0:g0 + every]
            dbs = [eng.upload(b) for b in grp]
            for db in dbs:
                eng.submit_device(db)
            r, f = eng.fetch_outputs(len(grp[-1]))
            for b in grp[:-1]:
                ob.submit(b)
            ro, fo = ob.submit(grp[-1])
            assert_results_equal(r, ro, f"soak batch {g0 + len(grp) - 1}")
            assert_fills_equal(f, fo, f"soak batch {g0 + len(grp) - 1}")
            no_window_rejects(r)
            for db in dbs:
                db.free()
        assert_books_equal(eng, ob, range(sc.num_symbols), "soak")
        assert eng.resting_count() == ob.resting() == eng.admission()["resting"]
    last = batches[-1]
    lim = ((last.kind >> 2) & 3) == 0
    assert np.median(np.abs(last.price_q4[lim] - base[last.symbol[lim]])) > 20 * sc.levels


@pytest.mark.parametrize("levels", [1024, 4096])
def test_drifting_mids_deep_windows(me, orc, levels):
    """The same unbounded semantics on the deep-window kernel (LDS window at 1,024 levels, HBM window
    at 4,096): mids trend 8 ticks per record of their symbol (several windows over the stream), far
    LIMITs up to 64 windows away."""
    sc, base, batches = _drift_stream(me, levels, 64, 4096, 40, drift_every=1, drift_step=8, far_pct=2)
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 18) as eng:
        for k, b in enumerate(batches):
            r, f = eng.submit_batch(b)
            ro, fo = ob.submit(b)
            assert_results_equal(r, ro, f"deep drift L={levels} b{k}")
            assert_fills_equal(f, fo, f"deep drift L={levels} b{k}")
            no_window_rejects(r)
        assert_books_equal(eng, ob, range(sc.num_symbols), f"deep drift L={levels}")
        assert eng.resting_count() == ob.resting()


@pytest.mark.parametrize("levels", [128, 256])
def test_seq_ring_sweeps_and_old_order_cancels(me, orc, levels):
    """A 4,096-entry seq ring under a 60 %-cancel stream of 1,024-record batches: the ring wraps ~20
    times, k_seq_sweep moves the horizon and rebuilds the old-order table each time, and cancels of
    orders older than the ring still find them (or correctly miss dead ones)."""
    sc = me.preset(5, num_symbols=16, levels=levels, batch=1024, seq_start=(1 << 40) + 3)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(80)]
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 16, seq_ring=4096,
                    batches_per_launch=1) as eng:
        nf = run_both(eng, ob, batches, ctx=f"ring L={levels}")
    assert nf > 0


def test_seq_ring_span_and_order_are_loud(me):
    B, L = me.SIDE_BUY, me.TYPE_LIMIT
    with engine_for(me, 1, 128, [1000], 256, 256, seq_ring=1024) as eng:
        b = _rows(me, [(0, B, L, 0, 1000, 1)] * 2, start_seq=10)
        b.seq[1] = 10 + 5000  # one batch spans more than the ring
        with pytest.raises(me.EngineError, match="seq ring"):
            eng.submit_batch(b)
    with engine_for(me, 1, 128, [1000], 256, 256) as eng:
        eng.submit_batch(_rows(me, [(0, B, L, 0, 1000, 1)], start_seq=100))
        with pytest.raises(me.EngineError, match="ascending"):
            eng.submit_batch(_rows(me, [(0, B, L, 0, 1000, 1)], start_seq=50))


# ---------------------------------------------------------------- edge cases
@pytest.mark.parametrize("levels", [64, 128, 512])
def test_edge_semantics_and_rejects(me, orc, levels):
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    I64 = (1 << 63) - 1
    rows = [
        (0, B, L, 0, 1000, 5), (0, B, L, 0, 999, 5), (0, B, L, 0, 1128, 5), (1, 0, L, 0, 5001, 5),
        (0, B, L, 0, 1001, 0), (7, B, L, 0, 1001, 1), (1, S, L, 1, 1, 0), (0, S, L, 1, 1, 0), (0, S, L, 1, 1, 0),
        (0, S, L, 1, 12, 0), (0, B, M, 0, 0, 3), (1, 3, M, 0, 0, 3), (0, S, L, 1, 1 << 40, 0),
        (1, S, L, 0, 5127, 2), (1, B, M, 0, 123, 5), (1, S, L, 0, 5000, 7), (1, B, L, 0, 5127, 9),
        # int64 extremes: asks far above, bids far below, then sweeps through all of them
        (1, S, L, 0, I64, 4), (1, S, L, 0, 10 ** 15, 4), (1, B, L, 0, -(1 << 62), 3), (1, B, L, 0, -(1 << 63), 2),
        (1, B, M, 0, 0, 20), (1, S, L, 0, -(1 << 63), 9), (1, S, L, 1, 19, 0), (1, B, L, 0, 7, 3),
    ]
    b = _rows(me, rows)
    ob = orc.OracleBook(2)
    with engine_for(me, 2, levels, [1000, 5000], 64, 256) as eng:
        run_both(eng, ob, [b], ctx="edge")
        run_both(eng, ob, [_rows(me, [(0, B, L, 0, 1000, 1)], start_seq=1 << 44)], ctx="big seq")
        r, f = eng.submit_batch(_rows(me, [], start_seq=(1 << 44) + 10))
        assert len(r) == 0 and len(f) == 0


def test_edge_deep_sweep_multi_window_multi_chunk(me, orc):
    """Sweeps crossing >64 levels (several ballot windows) and levels holding >32 orders (several
    FIFO chunks), cancels inside chunks, then chunk reuse from the free list; with a deep window
    and with a 128-level window the 300 ask levels mostly live in far levels."""
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    rows = []
    for lvl in range(300):                     # 300 ask levels, 1..3 orders each
        for k in range(1 + lvl % 3):
            rows.append((0, S, L, 0, 10000 + 2 * lvl, 1 + (lvl * 7 + k) % 50))
    for k in range(100):                       # one level with 100 orders (4 chunks)
        rows.append((0, B, L, 0, 9000, 1 + k % 9))
    b1 = _rows(me, rows)
    seq = len(rows) + 1
    cancels = [(0, S, L, 1, s, 0) for s in range(len(rows) - 99, len(rows) + 1, 3)]  # every 3rd bid
    b2 = _rows(me, cancels, start_seq=seq)
    seq += len(cancels)
    sweeps = [(0, B, M, 0, 0, 5000), (0, S, M, 0, 0, 120), (0, B, L, 0, 10500, 900), (0, S, L, 0, 9000, 50)]
    b3 = _rows(me, sweeps, start_seq=seq)
    seq += len(sweeps)
    refill = _rows(me, [(0, B, L, 0, 9000 + (k % 5), 3) for k in range(200)], start_seq=seq)
    for levels, base in ((4096, 8000), (128, 9950)):
        ob = orc.OracleBook(1)
        with engine_for(me, 1, levels, [base], 1024, 4096, max_chunks=4096) as eng:
            run_both(eng, ob, [b1, b2, b3, refill], ctx=f"deep sweep L={levels}")
            bids, asks = eng.snapshot(0, 5)
            obids, oasks = ob.snapshot(0, 5)
            assert np.array_equal(bids, obids) and np.array_equal(asks, oasks)


def test_edge_one_symbol_whole_batch_and_tile_boundaries(me, orc):
    """All records of a max-size batch on one symbol (one wave walks 65536 records) plus batch
    sizes around the sort/tape tile boundaries."""
    sc = me.preset(1)
    st = me.Stream(sc)
    base = st.base_prices()
    sizes = [65536, 4095, 4096, 4097, 1023, 1024, 1025, 1, 63, 64, 65]
    batches = [st.next(n) for n in sizes]
    ob = orc.OracleBook(1)
    with engine_for(me, 1, sc.levels, base, 65536, 1 << 18) as eng:
        run_both(eng, ob, batches, ctx="tiles")


def test_edge_bucket_boundaries(me, orc):
    """Register-window grouping: per-symbol record counts on both sides of one block (64) and of the
    bucket capacity (128; more records take the batch rescan), and more bad-symbol records than a
    bucket holds — interleaved at random, several batches so the bucket counters are reused."""
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    rng = np.random.default_rng(11)
    counts = [1, 63, 64, 65, 127, 128, 129, 300]
    bad = 200
    nsym = len(counts)
    base = [10_000 + 1000 * k for k in range(nsym)]
    batches, seq = [], 1
    for _ in range(3):
        syms = np.concatenate([np.full(c, k) for k, c in enumerate(counts)] +
                              [rng.integers(nsym, nsym + 50, bad)])
        rng.shuffle(syms)
        rows = []
        for sy in syms:
            sy = int(sy)
            side = B if rng.random() < 0.5 else S
            if rng.random() < 0.2:
                rows.append((sy, side, M, 0, 0, int(rng.integers(1, 60))))
            else:
                px = (base[sy] if sy < nsym else 10_000) + 64 + int(rng.integers(-20, 21))
                rows.append((sy, side, L, 0, px, int(rng.integers(1, 60))))
        batches.append(_rows(me, rows, start_seq=seq))
        seq += len(rows)
    ob = orc.OracleBook(nsym)
    with engine_for(me, nsym, 128, base, 4096, 1 << 14) as eng:
        run_both(eng, ob, batches, ctx="buckets")


def test_edge_symbol_count_sort_plans(me, orc):
    """1-pass sort up to 2047 symbols, 2-pass from 2048: exercise both sides of the switch; and the
    fill launch's bucket job (k_side) on both sides of its LDS-histogram limit (16,383 symbols)."""
    for S in (1, 2, 2047, 2048, 16_383, 16_384, 70_000):
        sc = me.preset(2, num_symbols=S, batch=20000)
        st = me.Stream(sc)
        base = st.base_prices()
        batches = [st.next(20000) for _ in range(2)]
        ob = orc.OracleBook(S)
        with engine_for(me, S, sc.levels, base, 20000, 1 << 17) as eng:
            run_both(eng, ob, batches, book_symbols=range(0, S, max(1, S // 50)), ctx=f"S={S}")


@pytest.mark.parametrize("reg_agg", ["0", "1", "cx"])
def test_cancelled_chunks_are_unlinked(me, orc, monkeypatch, reg_agg):
    """A level that never empties, with chunk after chunk filled and then cancelled: dead chunks
    (head, middle, tail) must be unlinked and reused, so a 4-chunk pool suffices for 30 rounds.
    ME_REG_AGG=1: the adds go through the grouped aggregate path and the cancels through k_match_reg's
    continuation, which parks freed chunks in fcache — the walk must reuse them (k_agg_gwalk)."""
    monkeypatch.setenv("ME_REG_AGG", "1" if reg_agg == "cx" else reg_agg)
    monkeypatch.setenv("ME_GW_CANCEL", "1" if reg_agg == "cx" else "0")  # cx: the cancels inside the grouped walk
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    C = me._abi.CHUNK_SLOTS
    ob = orc.OracleBook(1)
    seq = 1
    with engine_for(me, 1, 128, [1000], 4 * C, 4 * C, max_chunks=4) as eng:
        run_both(eng, ob, [_rows(me, [(0, B, L, 0, 1050, 7)], start_seq=seq)], ctx="anchor")
        seq += 1
        for rnd in range(30):
            adds = [(0, B, L, 0, 1050, 1 + k) for k in range(2 * C)]
            b = _rows(me, adds, start_seq=seq)
            first = seq
            seq += len(adds)
            # cancel in an order that kills the middle chunk first, then the tail, then the rest
            order = list(range(C // 2, C + C // 2)) + list(range(C + C // 2, 2 * C)) + list(range(C // 2))
            if rnd % 3 == 2:
                order = order[::-1]
            cancels = _rows(me, [(0, B, L, 1, first + k, 0) for k in order], start_seq=seq)
            seq += len(order)
            run_both(eng, ob, [b, cancels], ctx=f"round {rnd}")
        sweep = _rows(me, [(0, S, M, 0, 0, 5)], start_seq=seq)
        run_both(eng, ob, [sweep], ctx="final sweep")
        assert eng.paths()["grouped_agg"] == (reg_agg != "0")


def test_capacity_exhaustion_is_loud(me):
    """Pools sized below what a batch needs (within max_resting, so admission lets it in) fail the
    engine loudly and stickily; tests/test_admission.py covers the refusals that are not sticky."""
    B, L = me.SIDE_BUY, me.TYPE_LIMIT
    rows = [(0, B, L, 0, 1000 + (k % 64), 1) for k in range(200)]  # 64 levels -> needs >= 64 chunks
    with engine_for(me, 1, 128, [1000], 256, 256, max_chunks=8) as eng:
        with pytest.raises(me.EngineError, match="chunk pool"):
            eng.submit_batch(_rows(me, rows))
        with pytest.raises(me.EngineError):
            eng.submit_batch(_rows(me, rows[:1], start_seq=500))  # failed state is sticky
    # (far levels past their inline region are not a capacity limit any more: tests/test_far_arena.py)


def test_device_resident_path_matches_host_path(me, orc):
    sc = me.preset(2, num_symbols=256, batch=16384)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(6)]
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 18) as eng:
        dbs = [eng.upload(b) for b in batches]
        for b, db in zip(batches, dbs):
            eng.submit_device(db)
            r, f = eng.fetch_outputs(len(b))
            ro, fo = ob.submit(b)
            assert_results_equal(r, ro, "device path")
            assert_fills_equal(f, fo, "device path")
        assert_books_equal(eng, ob, range(sc.num_symbols), "device path")


# ---------------------------------------------------------------- BASELINE sizes
def test_full_size_config2_bitexact(me, orc):
    """BASELINE.json configs[1] at its real size (1,024 symbols, 65,536-record batches): 24
    consecutive batches compared record-for-record and fill-for-fill, plus size-independent
    properties of every tape."""
    sc = me.preset(2)
    st = me.Stream(sc)
    base = st.base_prices()
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 21, seq_ring=1 << 26) as eng:
        for k in range(24):
            b = st.next(sc.batch)
            r, f = eng.submit_batch(b)
            ro, fo = ob.submit(b)
            assert_results_equal(r, ro, f"full c2 b{k}")
            assert_fills_equal(f, fo, f"full c2 b{k}")
            # properties: tape ordered by taker seq; per-taker fill qty sums to filled_qty
            assert np.all(np.diff(f["taker_seq"].astype(np.int64)) >= 0)
            sums = np.bincount(np.repeat(np.arange(len(b)), r["fill_count"]), weights=f["qty"], minlength=len(b))
            assert np.array_equal(sums.astype(np.int64), r["filled_qty"].astype(np.int64))
            assert np.all(f["maker_seq"] < f["taker_seq"])
        assert_books_equal(eng, ob, range(0, sc.num_symbols, 7), "full c2")
        assert eng.resting_count() == ob.resting()


@pytest.mark.parametrize("group", [16, 32])
def test_every_batch_of_full_groups(me, orc, group):
    """The bench's pattern at full config-2 size — device batches back to back, `group` per launch —
    with EVERY batch of two full groups compared against the oracle, record for record."""
    sc = me.preset(2)
    st = me.Stream(sc)
    base = st.base_prices()
    ob = orc.OracleBook(sc.num_symbols)
    # admission control counts every record of a device batch as a possible rest: size max_resting
    # for both groups in flight so no submit has to cut a group short
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, (2 * group + 2) * sc.batch, seq_ring=1 << 26,
                    batches_per_launch=group) as eng:
        for gi in range(2):
            batches = [st.next(sc.batch) for _ in range(group)]
            dbs = [eng.upload(b) for b in batches]
            for db in dbs:
                eng.submit_device(db)
            eng.sync()
            assert eng.last_group_size() == group
            for k, b in enumerate(batches):
                r, f = eng.fetch_group_outputs(k, len(b))
                ro, fo = ob.submit(b)
                assert_results_equal(r, ro, f"G={group} group {gi} batch {k}")
                assert_fills_equal(f, fo, f"G={group} group {gi} batch {k}")
            for db in dbs:
                db.free()
        assert_books_equal(eng, ob, range(0, sc.num_symbols, 5), f"G={group}")
        assert eng.resting_count() == ob.resting()


def test_config3_grouped_bench_shape(me, orc):
    """The bench's config-3 shape per GPU: 12,500 symbols (more than one round of waves), 131,072-
    record batches, 32 per launch; every batch of the group against the oracle."""
    sc = me.preset(3, num_symbols=12_500, batch=131_072)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(32)]
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 22, seq_ring=1 << 26,
                    batches_per_launch=32) as eng:
        dbs = [eng.upload(b) for b in batches]
        for db in dbs:
            eng.submit_device(db)
        eng.sync()
        assert eng.last_group_size() == 32
        for k, b in enumerate(batches):
            r, f = eng.fetch_group_outputs(k, len(b))
            ro, fo = ob.submit(b)
            assert_results_equal(r, ro, f"c3 batch {k}")
            assert_fills_equal(f, fo, f"c3 batch {k}")
        assert_books_equal(eng, ob, range(0, sc.num_symbols, 97), "c3 grouped")
        assert eng.resting_count() == ob.resting()
        for db in dbs:
            db.free()


@pytest.mark.parametrize("group", [1, 3, 8, 17, 32])
@pytest.mark.parametrize("stream", ["uniform", "skewed"])
def test_back_to_back_device_batches(me, orc, group, stream):
    """Device batches submitted back to back without a sync (the bench's pattern), matched
    `group` batches per launch: the final books, the resting count, the fill total and the last
    batch's results/tape equal the oracle's. The skewed stream (Zipf symbols) overfills buckets
    (the rescan path) and carries unknown-symbol records (rejected by the bucket job)."""
    over = {} if stream == "uniform" else dict(zipf_s=1.2)
    sc = me.preset(2, **over)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(max(12, group + 5))]  # >= one full group + a partial one
    if stream == "skewed":
        for k, b in enumerate(batches):
            b.symbol[k * 97 % len(b)::4099] = sc.num_symbols + 3  # unknown symbols
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, (len(batches) + 1) * sc.batch,
                    batches_per_launch=group) as eng:
        dbs = [eng.upload(b) for b in batches]
        eng.timing_enable(True)
        for db in dbs:
            eng.submit_device(db)
        r, f = eng.fetch_outputs(len(batches[-1]))
        nfo = 0
        for b in batches:
            ro, fo = ob.submit(b)
            nfo += len(fo)
        assert_results_equal(r, ro, "back-to-back last batch")
        assert_fills_equal(f, fo, "back-to-back last batch")
        tm = eng.timing_read()
        assert tm["fills"] == nfo and tm["launches"] == -(-len(batches) // group) and tm["match_ms"] > 0
        assert_books_equal(eng, ob, range(0, sc.num_symbols, 5), "back-to-back")
        assert eng.resting_count() == ob.resting()
        for db in dbs:
            db.free()


def test_partial_groups_between_fetches(me, orc):
    """Runs of 1..7 device batches between fetches: every fetch flushes a partial group, and the
    next group starts over; every fetched batch equals the oracle's."""
    sc = me.preset(2, num_symbols=512, batch=8192)
    st = me.Stream(sc)
    base = st.base_prices()
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, 1 << 18) as eng:
        for run in (1, 7, 2, 8, 5, 3):
            batches = [st.next(sc.batch) for _ in range(run)]
            dbs = [eng.upload(b) for b in batches]
            for db in dbs:
                eng.submit_device(db)
            r, f = eng.fetch_outputs(len(batches[-1]))
            for b in batches:
                ro, fo = ob.submit(b)
            assert_results_equal(r, ro, f"run {run}")
            assert_fills_equal(f, fo, f"run {run}")
            for db in dbs:
                db.free()
        assert_books_equal(eng, ob, range(0, sc.num_symbols, 3), "partial groups")
        assert eng.resting_count() == ob.resting()


# ---------------------------------------------------------------- device book snapshots
@pytest.mark.parametrize("levels", [128, 1024])
def test_book_orders_snapshot_kernel(me, orc, levels):
    """GetOrderBook per order (one k_book_snapshot launch): the top-N levels' resting orders in
    priority order and the level aggregates equal the oracle's, window and far levels alike; the
    all-symbol level snapshot equals the per-symbol one."""
    sc = me.preset(2, num_symbols=48, levels=levels, batch=4096, drift_step=3, drift_every=40, far_pct=3)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(6)]
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, total + 1024, max_chunks=total + 256) as eng:
        run_both(eng, ob, batches, ctx="snapshot")
        lv_all, cnt_all = eng.levels_all(7)
        for s in range(sc.num_symbols):
            dump = ob.dump(s)
            for depth in (1, 7, 100000):
                bids, asks, lb, la = eng.book_orders(s, depth)
                eb = side_levels(dump, me.SIDE_BUY, depth)
                ea = side_levels(dump, me.SIDE_SELL, depth)
                assert np.array_equal(bids, eb), f"symbol {s} depth {depth}: bids"
                assert np.array_equal(asks, ea), f"symbol {s} depth {depth}: asks"
                sb, sa = ob.snapshot(s, depth)
                assert np.array_equal(lb, sb) and np.array_equal(la, sa), f"symbol {s} depth {depth}: levels"
                if depth == 7:
                    assert np.array_equal(lv_all[s, 0, : cnt_all[s, 0]], sb)
                    assert np.array_equal(lv_all[s, 1, : cnt_all[s, 1]], sa)


def test_book_orders_ten_thousand_levels_one_launch(me, orc):
    """A 10,000-level-per-side book (config 4's seeded shape, L = 32,768) snapshots per order in one
    launch and equals the oracle."""
    sc = me.preset(4, num_symbols=8, batch=65536)
    st = me.Stream(sc)
    base = st.base_prices()
    seeds = st.seed_books(range(2), 10_000)
    ob = orc.OracleBook(sc.num_symbols)
    with engine_for(me, sc.num_symbols, sc.levels, base, 65536, len(seeds) + 1024, max_chunks=len(seeds) + 64) as eng:
        run_both(eng, ob, [seeds.take(slice(0, 20000)), seeds.take(slice(20000, None))], check_books=False)
        bids, asks, lb, la = eng.book_orders(0, 10_000)
        dump = ob.dump(0)
        assert len(lb) == 10_000 and len(la) == 10_000
        assert np.array_equal(bids, dump[dump["side"] == me.SIDE_BUY])
        assert np.array_equal(asks, dump[dump["side"] == me.SIDE_SELL])


def test_handoffs_only_for_far_events(me, orc):
    """The register-window kernel hands a symbol to its continuation launch only for a far price level
    (or a re-centre / an old order): a cancel-heavy stream whose prices stay in the window never hands
    off (cancel records carry a seq, not a price), a stream with far LIMITs does."""
    for cfg, over, expect_far in ((5, dict(num_symbols=256, batch=16384), False),
                                  (2, dict(num_symbols=64, batch=4096, far_pct=2), True)):
        sc = me.preset(cfg, **over)
        st = me.Stream(sc)
        base = st.base_prices()
        batches = [st.next(sc.batch) for _ in range(6)]
        total = sum(len(b) for b in batches)
        ob = orc.OracleBook(sc.num_symbols)
        old = os.environ.get("ME_REG_AGG")
        os.environ["ME_REG_AGG"] = "0"  # k_match_reg's hand-offs (the grouped aggregate path hands cancels off)
        try:
            eng = engine_for(me, sc.num_symbols, sc.levels, base, sc.batch, total + 1024,
                             max_chunks=total + 2 * sc.num_symbols)
        finally:
            if old is None:
                del os.environ["ME_REG_AGG"]
            else:
                os.environ["ME_REG_AGG"] = old
        with eng:
            run_both(eng, ob, batches, ctx=f"handoffs c{cfg}")
            h = eng.stats()["handoffs"]
        assert (h > 0) == expect_far, (cfg, h)
