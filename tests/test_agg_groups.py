"""Grouped launches through the aggregate path (ME_REG_AGG=1, windows of at most 128 levels): every
symbol of a launch group walked on level totals by k_agg_gwalk (me_agg.hip), FIFOs resolved per level,
each batch's fills placed in its own scratch — every batch's outputs bit-exact against the oracle, through
the pipelined host path (per-batch results and tapes) and back-to-back device batches. Cancels, prices
outside the window and overfull buckets hand a symbol's rest of the group to k_match_reg's continuation
launch. Needs an MI355X."""
import os

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


def _engine(me, sc, base, batches, **kw):
    total = sum(len(b) for b in batches)
    old = os.environ.get("ME_REG_AGG")
    os.environ["ME_REG_AGG"] = "1"
    try:
        return me.Engine(sc.num_symbols, sc.levels, base, max_batch=max(len(b) for b in batches),
                         max_resting=total + 1024, max_chunks=total + 2 * sc.num_symbols, seq_ring=1 << 22, **kw)
    finally:
        if old is None:
            del os.environ["ME_REG_AGG"]
        else:
            os.environ["ME_REG_AGG"] = old


def _pipelined(eng, batches, lag):
    out, tickets = [None] * len(batches), []
    for k, b in enumerate(batches):
        tickets.append((k, eng.submit_host(b)))
        while len(tickets) > lag:
            j, t = tickets.pop(0)
            out[j] = eng.collect(t)
    for j, t in tickets:
        out[j] = eng.collect(t)
    return out


def _check(eng, ob, batches, outs, ctx):
    nf = 0
    for k, b in enumerate(batches):
        ro, fo = ob.submit(b)
        assert_results_equal(outs[k][0], ro, f"{ctx} batch {k}")
        assert_fills_equal(outs[k][1], fo, f"{ctx} batch {k}")
        nf += len(fo)
    assert_books_equal(eng, ob, range(eng.num_symbols), ctx)
    assert eng.resting_count() == ob.resting(), f"{ctx}: resting count"
    return nf


@pytest.mark.parametrize("group,lag", [(1, 2), (4, 9), (32, 70)])
def test_agg_groups_config2_every_batch(me, orc, group, lag):
    """Config 2's stream (80 % LIMIT +-32 ticks, 20 % MARKET) on 96 symbols: no record leaves the
    aggregate path; every batch of full and partial groups against the oracle."""
    sc = me.preset(2, num_symbols=96, batch=4096)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(72)]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=group) as eng:
        nf = _check(eng, ob, batches, _pipelined(eng, batches, lag), f"agg G={group}")
        assert eng.stats()["handoffs"] == 0
    assert nf > 0


@pytest.mark.parametrize("spread", [2, 60])
def test_agg_groups_long_fifos_and_sweeps(me, orc, spread):
    """Tight spreads (a few levels with long chunk chains) and wide ones (rests beyond the 64-entry
    lists), sweeping MARKETs of up to 6 x 100 lots, G = 16."""
    sc = me.preset(2, num_symbols=48, batch=4096, spread_ticks=spread, market_qty_mult=6, market_pct=25)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(48)]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=16) as eng:
        assert _check(eng, ob, batches, _pipelined(eng, batches, 20), f"agg spread={spread}") > 0


def test_agg_groups_handoffs(me, orc):
    """Cancels, a drifting mid with far LIMITs (re-centring) and OIDs above 2^33 at G = 32: symbols are
    handed to the register kernel's continuation mid-group; every batch against the oracle."""
    sc = me.preset(5, num_symbols=128, levels=128, batch=4096, cancel_pct=10, market_pct=15, market_qty_mult=3,
                   drift_step=1, drift_every=3, far_pct=1, seq_start=(1 << 33) + 5)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(80)]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=32) as eng:
        _check(eng, ob, batches, _pipelined(eng, batches, 40), "agg handoffs")
        assert eng.stats()["handoffs"] > 0


def test_agg_groups_large_quantities(me, orc):
    """Quantities up to 2^25 at G = 8: books whose sum reaches 2^31 (the ladder's 32-bit limit) hand the
    symbol's rest of the group to the continuation; every batch against the oracle."""
    sc = me.preset(2, num_symbols=32, batch=4096, max_qty=1 << 25)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(24)]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=8) as eng:
        _check(eng, ob, batches, _pipelined(eng, batches, 10), "agg large qty")
        assert eng.stats()["handoffs"] > 0


def test_agg_groups_overfull_buckets(me, orc):
    """A Zipf-skewed stream: the head symbols' buckets overflow BK_CAP records, so the walk hands them to
    the continuation (which rescans the batch); every batch against the oracle."""
    sc = me.preset(2, num_symbols=64, batch=8192, zipf_s=1.3)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(24)]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=8) as eng:
        _check(eng, ob, batches, _pipelined(eng, batches, 10), "agg overfull")
        assert eng.stats()["handoffs"] > 0


def test_agg_groups_device_back_to_back(me, orc):
    """The bench's pattern at config 2's shape (1,024 symbols, 65,536-record batches, G = 32), device
    batches back to back: books, resting count, fill total and the last batch against the oracle."""
    sc = me.preset(2)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(40)]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches) as eng:
        dbs = [eng.upload(b) for b in batches]
        eng.timing_enable(True)
        for db in dbs:
            eng.submit_device(db)
        r, f = eng.fetch_outputs(len(batches[-1]))
        nfo = 0
        for b in batches:
            ro, fo = ob.submit(b)
            nfo += len(fo)
        assert_results_equal(r, ro, "agg back-to-back last batch")
        assert_fills_equal(f, fo, "agg back-to-back last batch")
        assert eng.timing_read()["fills"] == nfo
        assert_books_equal(eng, ob, range(0, sc.num_symbols, 3), "agg back-to-back")
        assert eng.resting_count() == ob.resting()
        for db in dbs:
            db.free()


@pytest.mark.parametrize("early", ["0", "3", "8"])
def test_agg_groups_early_fill_after_flush(me, orc, monkeypatch, early):
    """Groups submitted after a flush bucket every ME_EARLY_FILL batches while the rest are still being
    submitted (me_engine.cpp early_fill); the flush buckets what is left, if anything. Device batches in
    groups of 5, 8, 9, 16, 20, 32 and 3 at G = 32, a sync after each: every batch of every group against
    the oracle."""
    monkeypatch.setenv("ME_EARLY_FILL", early)
    sc = me.preset(2, num_symbols=96, batch=4096)
    st = me.Stream(sc)
    base = st.base_prices()
    sizes = [5, 8, 9, 16, 20, 32, 3]
    batches = [st.next(sc.batch) for _ in range(sum(sizes))]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=32) as eng:
        dbs = [eng.upload(b) for b in batches]
        k0 = 0
        for n in sizes:
            for db in dbs[k0:k0 + n]:
                eng.submit_device(db)
            eng.sync()
            assert eng.last_group_size() == n
            for k in range(n):
                r, f = eng.fetch_group_outputs(k, len(batches[k0 + k]))
                ro, fo = ob.submit(batches[k0 + k])
                assert_results_equal(r, ro, f"early={early} group of {n} batch {k}")
                assert_fills_equal(f, fo, f"early={early} group of {n} batch {k}")
            k0 += n
        assert_books_equal(eng, ob, range(sc.num_symbols), f"early={early}")
        assert eng.resting_count() == ob.resting()
        for db in dbs:
            db.free()


def _peak_resting(orc, sc, batches):
    """The most orders resting at any record of the stream (the oracle fed one record at a time)."""
    ob = orc.OracleBook(sc.num_symbols)
    peak = 0
    for b in batches:
        for i in range(len(b)):
            ob.submit(b.take(slice(i, i + 1)))
            peak = max(peak, ob.resting())
    return peak


@pytest.mark.parametrize("group", [1, 8])
def test_agg_groups_cancels_tight_chunk_pool(me, orc, group):
    """One symbol, 40 % cancels and sweeping MARKETs, ME_REG_AGG=1: adds go through the walk, cancels
    hand the symbol to k_match_reg's continuation, which parks freed chunks in fcache. The pool holds
    only the stream's peak resting orders (+ the 2S slack and a few): every parked chunk must be reused
    by the walk (k_agg_gwalk links them into the free list), or the pool runs dry."""
    sc = me.preset(5, num_symbols=1, levels=128, batch=512, cancel_pct=40, market_pct=15, market_qty_mult=3,
                   spread_ticks=8)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(40)]
    peak = _peak_resting(orc, sc, batches)
    ob = orc.OracleBook(sc.num_symbols)
    old = os.environ.get("ME_REG_AGG")
    os.environ["ME_REG_AGG"] = "1"
    try:
        eng = me.Engine(1, sc.levels, base, max_batch=sc.batch, max_resting=sum(len(b) for b in batches),
                        max_chunks=peak + 2 + 8, seq_ring=1 << 22, batches_per_launch=group)
    finally:
        if old is None:
            del os.environ["ME_REG_AGG"]
        else:
            os.environ["ME_REG_AGG"] = old
    with eng:
        _check(eng, ob, batches, _pipelined(eng, batches, 2 * group + 1), f"agg tight pool G={group}")
        assert eng.stats()["handoffs"] > 0
        assert eng.paths()["grouped_agg"]


@pytest.mark.parametrize("cx", ["auto", "0"])
def test_agg_auto_mode_turns_off_under_cancels(me, orc, monkeypatch, cx):
    """Automatic path choice (ME_REG_AGG unset) at a shape that picks the grouped aggregate path (8,192-
    record batches, 128 records per symbol): a cancel-free first phase runs on it; a second phase with
    30 % cancels hands symbols off. By default the engine then switches to the grouped walk that covers
    cancels (k_agg_gwalk_cx) and stays on the grouped path; with ME_GW_CANCEL=0 it turns the grouped path
    off for good. max_chunks = max_resting + 2S, every batch of both phases against the oracle."""
    if cx == "0":
        monkeypatch.setenv("ME_GW_CANCEL", "0")
    sc = me.preset(5, num_symbols=64, levels=128, batch=8192, cancel_pct=30, market_pct=15, market_qty_mult=3)
    st = me.Stream(sc)
    base = st.base_prices()
    raw = [st.next(sc.batch) for _ in range(40)]
    # phase 1: the first 16 batches with their cancel records dropped (the generator's later cancels
    # never target an order it already cancelled, and the oracle rejects unknown targets anyway)
    batches = [b.take((b.kind & 8) == 0) if k < 16 else b for k, b in enumerate(raw)]
    total = sum(len(b) for b in batches)
    max_resting = total + 1024
    assert os.environ.get("ME_REG_AGG") is None
    ob = orc.OracleBook(sc.num_symbols)
    with me.Engine(sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=max_resting,
                   max_chunks=max_resting + 2 * sc.num_symbols, seq_ring=1 << 22, batches_per_launch=8) as eng:
        outs = _pipelined(eng, batches[:16], 9)
        assert eng.paths()["grouped_agg"], "phase 1 should run on the grouped aggregate path"
        assert eng.stats()["handoffs"] == 0
        assert not eng.paths()["grouped_cancels"]
        outs += _pipelined(eng, batches[16:], 9)
        p = eng.paths()
        if cx == "0":
            assert not p["grouped_agg"], "hand-offs should have turned the aggregate path off"
        else:
            assert p["grouped_agg"] and p["grouped_cancels"], f"the walk with cancels should have taken over: {p}"
        _check(eng, ob, batches, outs, f"agg auto flip (ME_GW_CANCEL={cx})")


@pytest.mark.parametrize("symbols,agg", [(768, True), (2048, False)])
def test_agg_auto_choice_by_records_per_symbol(me, orc, symbols, agg):
    """Automatic path choice (ME_REG_AGG unset) by shape: 8,192-record batches over 768 symbols (~10.7
    records per symbol and batch, ~340 per 32-batch group: config 3's shape) take the grouped aggregate
    path; over 2,048 symbols (4 per batch) they stay on k_match_reg. Every batch against the oracle."""
    sc = me.preset(3, num_symbols=symbols, levels=128, batch=8192)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(40)]
    total = sum(len(b) for b in batches)
    assert os.environ.get("ME_REG_AGG") is None
    ob = orc.OracleBook(sc.num_symbols)
    with me.Engine(sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=total + 1024,
                   seq_ring=1 << 22) as eng:
        outs = _pipelined(eng, batches, 70)
        assert eng.paths()["grouped_agg"] == agg
        _check(eng, ob, batches, outs, f"auto choice S={symbols}")
