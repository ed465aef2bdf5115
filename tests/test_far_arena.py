"""Far levels without a capacity (GPU): price levels outside a symbol's window live in per-side regions
of the far arena (me_far.hpp). A side that outgrows its inline region (me_config.far_levels) moves to a
larger region, and k_seq_sweep's copying collection compacts the arena and brings small sides back
inline. The reference accepts any positive raw price at any scale (src/server/matching_engine_service.cpp:
78-83, include/domain/price.hpp:15-29) and the oracle's book is unbounded, so every stream here must equal
the oracle batch for batch — results, tapes, final books — with the engine never failing."""
import numpy as np
import pytest

from tests._parity import assert_books_equal, assert_fills_equal, assert_results_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


@pytest.fixture(scope="module")
def orc(built):
    from oracle import oracle

    return oracle


def _rows(me, rows, start_seq=1):
    n = len(rows)
    return me.Batch(np.arange(start_seq, start_seq + n, dtype=np.uint64), [r[4] for r in rows],
                    [r[5] for r in rows], [r[0] for r in rows], [me.kind(r[1], r[2], r[3]) for r in rows])


def _check(eng, ob, b, ctx):
    r, f = eng.submit_batch(b)
    ro, fo = ob.submit(b)
    assert_results_equal(r, ro, ctx)
    assert_fills_equal(f, fo, ctx)


def test_far_side_outgrows_inline_region(me, orc):
    """Round 4's loud-failure case (a best bid in the window, then 40 distinct bids far below it, with 16
    inline far levels) now matches the oracle: the bid side moves to the arena twice (16 -> 32 -> 64). Then
    a SELL MARKET sweeps every bid, window and far, best first, and a second far ladder builds again."""
    B, S_, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    ob = orc.OracleBook(1)
    with me.Engine(1, 128, [4990], max_batch=256, max_resting=256, seq_ring=1 << 22, far_levels=16) as eng:
        rows = [(0, B, L, 0, 5000, 1)] + [(0, B, L, 0, 100 + 3 * k, 1 + k % 5) for k in range(40)]
        _check(eng, ob, _rows(me, rows), "40 far bids")
        assert eng.far_stats()["moves"] == 2
        assert_books_equal(eng, ob, [0], "far bids")
        _check(eng, ob, _rows(me, [(0, S_, M, 0, 0, 1000)], start_seq=100), "sweep")
        assert eng.resting_count() == ob.resting() == 0
        rows = [(0, S_, L, 0, 9000 + 7 * k, 2) for k in range(70)] + [(0, B, L, 0, 8000, 3)]
        _check(eng, ob, _rows(me, rows, start_seq=200), "far asks above a re-centred window")
        assert_books_equal(eng, ob, [0], "far asks")
        assert eng.resting_count() == ob.resting()


def _drift(me, levels, S, batch, nb, far_pct, cancel_pct=10, drift_step=4, drift_every=3):
    sc = me.preset(5, num_symbols=S, levels=levels, batch=batch, cancel_pct=cancel_pct, market_pct=15,
                   market_qty_mult=3, drift_step=drift_step, drift_every=drift_every, far_pct=far_pct,
                   seq_start=(1 << 33) + 5)
    st = me.Stream(sc)
    return sc, st.base_prices(), [st.next(batch) for _ in range(nb)]


@pytest.mark.parametrize("levels,path", [(128, "reg"), (128, "agg"), (1024, "deep")])
def test_far_arena_collections(me, orc, monkeypatch, levels, path):
    """A drifting market with 20 % far LIMITs over few symbols, 8 inline far levels and a collection
    trigger of 64 arena entries (ME_FAR_GC_AT): sides move again and again and the arena is collected
    between launch groups many times — the register kernel's continuation, the grouped aggregate path's
    hand-offs and the deep-window kernel all grow sides. Every batch and the final books equal the
    oracle's."""
    monkeypatch.setenv("ME_FAR_GC_AT", "64")
    monkeypatch.setenv("ME_REG_AGG", "1" if path == "agg" else "0")
    S, batch = (4, 8192) if path == "agg" else (4, 1024)
    sc, base, batches = _drift(me, levels, S, batch, 24, far_pct=20)
    total = sum(len(b) for b in batches)
    ob = orc.OracleBook(S)
    with me.Engine(S, levels, base, max_batch=batch, max_resting=total + 1024, seq_ring=1 << 22,
                   far_levels=8, batches_per_launch=4) as eng:
        assert eng.paths()["grouped_agg"] == (path == "agg")
        for k, b in enumerate(batches):
            _check(eng, ob, b, f"{path} L={levels} batch {k}")
        assert_books_equal(eng, ob, range(S), f"{path} L={levels}")
        assert eng.resting_count() == ob.resting() == eng.admission()["resting"]
        st = eng.far_stats()
        assert st["moves"] > 4 and st["collections"] > 2, st


def test_far_arena_device_groups(me, orc, monkeypatch):
    """Back-to-back device batches (one launch group of 16, so growth and the collection ahead of the next
    group meet mid-stream), every batch compared through me_fetch_group_outputs."""
    monkeypatch.setenv("ME_FAR_GC_AT", "128")
    sc, base, batches = _drift(me, 128, 8, 2048, 48, far_pct=15)
    ob = orc.OracleBook(sc.num_symbols)
    group = 16
    with me.Engine(sc.num_symbols, 128, base, max_batch=sc.batch, max_resting=1 << 18, seq_ring=1 << 22,
                   far_levels=4, batches_per_launch=group) as eng:
        for g0 in range(0, len(batches), group):
            grp = batches[g0:g0 + group]
            dbs = [eng.upload(b) for b in grp]
            for db in dbs:
                eng.submit_device(db)
            eng.sync()
            for k, b in enumerate(grp):
                r, f = eng.fetch_group_outputs(k, len(b))
                ro, fo = ob.submit(b)
                assert_results_equal(r, ro, f"group {g0 // group} batch {k}")
                assert_fills_equal(f, fo, f"group {g0 // group} batch {k}")
            for db in dbs:
                db.free()
        assert_books_equal(eng, ob, range(sc.num_symbols), "device groups")
        st = eng.far_stats()
        assert st["moves"] > 0 and st["collections"] > 0, st


def test_far_levels_in_book_snapshots(me, orc):
    """GetOrderBook's whole-book dump and the level snapshot reach far levels in moved regions: a side of
    600 far levels (inline region 16) is dumped whole, best first."""
    B, L = me.SIDE_BUY, me.TYPE_LIMIT
    ob = orc.OracleBook(1)
    rows = [(0, B, L, 0, 100000, 1)] + [(0, B, L, 0, 1000 + 11 * k, 1 + k % 3) for k in range(600)]
    with me.Engine(1, 64, [99990], max_batch=1024, max_resting=4096, seq_ring=1 << 22, far_levels=16) as eng:
        _check(eng, ob, _rows(me, rows), "600 far bids")
        assert_books_equal(eng, ob, [0], "600 far bids")
        bids, _ = eng.snapshot(0, 1000)
        assert len(bids) == 601
        assert bids["price_q4"][0] == 100000 and bids["price_q4"][-1] == 1000
        assert np.all(np.diff(bids["price_q4"]) < 0)


@pytest.mark.parametrize("path", ["reg", "agg"])
def test_far_arena_worst_case_default_sizing(me, orc, monkeypatch, path):
    """The far arena's bound at its DEFAULT sizing (no ME_FAR_GC_AT, default far_levels) with max_resting
    close to the live count: in ONE launch group four symbols each grow a side far past its inline region
    (300 far asks), cancel every one of them and grow it again. Nothing may fail, every record equals the
    oracle, and the active half's use stays within its size (6 x (max_resting + 64) + 4 x far_levels,
    me_engine.cpp), which the copying collection ahead of the next group brings back down."""
    monkeypatch.delenv("ME_FAR_GC_AT", raising=False)
    monkeypatch.setenv("ME_REG_AGG", "1" if path == "agg" else "0")
    B, S_, L, X = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.OP_CANCEL
    S, nf = 4, 300
    seq = 1
    rows1 = []
    for s in range(S):
        rows1 += [(s, B, L, 0, 1010, 5), (s, S_, L, 0, 1020, 5)]  # a window around the market
        rows1 += [(s, S_, L, 0, 2000 + 3 * k, 1 + k % 4) for k in range(nf)]  # far asks above it
    b1 = _rows(me, rows1, seq)
    first = {s: seq + s * (nf + 2) + 2 for s in range(S)}
    seq += len(rows1)
    rows2 = [(s, B, L, X, first[s] + k, 0) for s in range(S) for k in range(nf)]  # every far ask cancelled
    rows2 += [(s, S_, L, 0, 5000 + 7 * k, 2) for s in range(S) for k in range(nf)]  # and a far side again
    b2 = _rows(me, rows2, seq)
    # admission counts every LIMIT of the batches accepted but not matched yet: both batches of the group
    max_resting = S * (nf + 2) + S * nf + 16
    ob = orc.OracleBook(S)
    with me.Engine(S, 128, [1000] * S, max_batch=len(rows2), max_resting=max_resting, seq_ring=1 << 22,
                   batches_per_launch=4) as eng:
        fcap = eng.config()["far_levels"]
        assert fcap == 256 and nf > fcap
        t1, t2 = eng.submit_host(b1), eng.submit_host(b2)  # one launch group
        outs = [eng.collect(t1), eng.collect(t2)]
        for k, b in enumerate([b1, b2]):
            ro, fo = ob.submit(b)
            assert_results_equal(outs[k][0], ro, f"{path} batch {k}")
            assert_fills_equal(outs[k][1], fo, f"{path} batch {k}")
        assert_books_equal(eng, ob, range(S), f"far worst case {path}")
        st = eng.far_stats()
        assert st["moves"] >= S, st
        assert st["arena_used"] <= 6 * (max_resting + 64) + 4 * fcap, st
        assert eng.resting_count() == ob.resting()
