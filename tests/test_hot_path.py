"""The hot-symbol paths of deep windows against the CPU oracle, bit-exact per batch: the aggregate path
(me_agg.hip: a level-total walk per hot symbol, FIFO resolution per level in parallel; the default for
128 < L <= 32,768) and k_match_hot (the write-through top-of-book path, me_kernels.hip; ME_HOT_AGG=0).
ME_HOT_MIN (read at me_create) sets the records per batch that make a symbol hot; 1 sends every symbol
through the hot path, so the generic fallbacks (cancels, prices outside the window, far levels,
re-centring: k_match_hot_cont) run behind it too."""
import os

import numpy as np
import pytest

from tests._parity import assert_books_equal, assert_fills_equal, assert_results_equal


def run_both(eng, ob, batches, ctx=""):
    """run_both of tests/_parity.py, naming the batch an engine error came from."""
    total = 0
    for k, b in enumerate(batches):
        try:
            rg, fg = eng.submit_batch(b)
        except Exception as ex:
            raise AssertionError(f"{ctx}: batch {k}: {ex}") from ex
        ro, fo = ob.submit(b)
        assert_results_equal(rg, ro, f"{ctx} batch {k}")
        assert_fills_equal(fg, fo, f"{ctx} batch {k}")
        total += len(fo)
    assert_books_equal(eng, ob, range(eng.num_symbols), ctx)
    assert eng.resting_count() == ob.resting(), f"{ctx}: resting count"
    return total

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


@pytest.fixture(scope="module")
def orc(built):
    from oracle import oracle

    return oracle


def _engine(me, hot_min, *a, agg=1, ladder=None, occ=None, **kw):
    env = {"ME_HOT_MIN": str(hot_min), "ME_HOT_AGG": str(agg)}
    if ladder is not None:  # ME_AGG_LADDER: the largest window k_agg_walk's ladder walk takes (0: lists)
        env["ME_AGG_LADDER"] = str(ladder)
    if occ is not None:  # ME_LW_OCC: ladders deeper than this search through the LDS occupancy bitmap (0: off)
        env["ME_LW_OCC"] = str(occ)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        kw.setdefault("seq_ring", 1 << 22)
        return me.Engine(*a, **kw)
    finally:
        for k, v in old.items():
            if v is None:
                del os.environ[k]
            else:
                os.environ[k] = v


def _drift(me, levels, num_symbols, batch, nbatches, **over):
    kw = dict(num_symbols=num_symbols, levels=levels, batch=batch, cancel_pct=10, market_pct=15, market_qty_mult=3,
              drift_step=1, drift_every=4, far_pct=1, seq_start=(1 << 33) + 99)
    kw.update(over)
    sc = me.preset(5, **kw)
    st = me.Stream(sc)
    return sc, st.base_prices(), [st.next(batch) for _ in range(nbatches)]


@pytest.mark.parametrize("agg", [1, 0])
@pytest.mark.parametrize("hot_min", [1, 64])
def test_hot_drift_far_cancels(me, orc, hot_min, agg):
    """Mids drifting past the 2,048-level windows, 1 % far LIMITs, 10 % cancels, sweeping MARKETs:
    every generic fallback inside the hot path (cancel, out-of-window rest with re-centring, takers while
    far levels exist), list rebuilds and deep rests."""
    sc, base, batches = _drift(me, 2048, 6, 6144, 60)
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, hot_min, sc.num_symbols, sc.levels, base, agg=agg, max_batch=sc.batch,
                 max_resting=total + 64, max_chunks=total + 64) as eng:
        nf = run_both(eng, ob, batches, ctx=f"hot drift min={hot_min} agg={agg}")
    assert nf > 0


@pytest.mark.parametrize("agg", [1, 0])
def test_hot_sweeps_drain_lists(me, orc, agg):
    """MARKETs of up to 40 x 100 qty against thin levels: a sweep consumes more than the 64 listed
    levels and the list is rebuilt mid-sweep (the list walk, ME_AGG_LADDER=0); no cancels, no far prices."""
    sc, base, batches = _drift(me, 4096, 3, 4096, 40, cancel_pct=0, far_pct=0, market_qty_mult=40,
                               market_pct=10, drift_every=0, drift_step=0)
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 1, sc.num_symbols, sc.levels, base, agg=agg, ladder=0, max_batch=sc.batch,
                 max_resting=total + 64, max_chunks=total + 64) as eng:
        nf = run_both(eng, ob, batches, ctx=f"hot sweeps agg={agg}")
    assert nf > 0


@pytest.mark.parametrize("agg", [1, 0])
def test_hot_multichunk_levels(me, orc, agg):
    """A 4-tick spread on a 2,048-level window: levels hold dozens of orders (chunk chains), walks cross
    chunk boundaries (the one load of a walk) and appends open new tail chunks."""
    sc, base, batches = _drift(me, 2048, 2, 4096, 30, cancel_pct=5, far_pct=0, spread_ticks=4, drift_every=0,
                               drift_step=0, market_qty_mult=2)
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 1, sc.num_symbols, sc.levels, base, agg=agg, max_batch=sc.batch, max_resting=total + 64,
                 max_chunks=total + 64) as eng:
        nf = run_both(eng, ob, batches, ctx=f"hot multichunk agg={agg}")
    assert nf > 0


@pytest.mark.parametrize("agg", [1, 0])
def test_hot_equals_generic_config4(me, orc, agg):
    """Config 4's shape (Zipf symbols, L = 32,768, books seeded to 3,000 levels per side): the hot path
    (default threshold) and the generic kernel alone (ME_HOT_MIN=0) give identical outputs, both equal
    to the oracle."""
    sc = me.preset(4, num_symbols=300, batch=32768)
    st = me.Stream(sc)
    base = st.base_prices()
    seeds = st.seed_books(range(8), 3000)
    batches = [seeds.take(slice(i, i + 32768)) for i in range(0, len(seeds), 32768)]
    batches += [st.next(sc.batch) for _ in range(4)]
    total = sum(len(b) for b in batches)
    outs = []
    for hot_min in (512, 0):
        ob = orc.OracleBook(sc.num_symbols)
        with _engine(me, hot_min, sc.num_symbols, sc.levels, base, agg=agg, max_batch=32768,
                     max_resting=total + 1024, max_chunks=total + 1024) as eng:
            got = []
            for b in batches:
                got.append(eng.submit_batch(b))
            for b, (r, f) in zip(batches, got):
                ro, fo = ob.submit(b)
                assert np.array_equal(f, fo) and all(np.array_equal(r[x], ro[x]) for x in
                                                     ("filled_qty", "remaining_qty", "fill_count", "status"))
            outs.append([eng.dump(s) for s in range(0, 300, 7)])
    for a, b in zip(*outs):
        assert np.array_equal(a, b)


@pytest.mark.parametrize("levels", [256, 2048])
def test_agg_single_symbol_config1(me, orc, levels):
    """Config 1's shape (one symbol, 80 % LIMIT +-32 ticks, 20 % MARKET): every record of every batch on
    the aggregate path (no hand-off), deep multi-chunk levels, the walk's list inserts and pops; L = 256
    runs k_match's LDS-ladder build beside it, 2,048 the HBM build."""
    sc = me.preset(1, levels=levels, batch=16384)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(12)]
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 512, sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=total + 64,
                 max_chunks=total + 64) as eng:
        nf = run_both(eng, ob, batches, ctx=f"agg c1 L={levels}")
    assert nf > 0


@pytest.mark.parametrize("levels,ladder", [(256, 0), (2048, 0)])
def test_agg_config1_walk_forms(me, orc, levels, ladder):
    """Config 1's shape on the walk form the default does not pick (ME_AGG_LADDER=0): the top-of-book
    lists, which also take any book the 32-bit ladder cannot hold, at L = 256 and 2,048."""
    sc = me.preset(1, levels=levels, batch=16384)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(8)]
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 512, sc.num_symbols, sc.levels, base, ladder=ladder, max_batch=sc.batch,
                 max_resting=total + 64, max_chunks=total + 64) as eng:
        assert run_both(eng, ob, batches, ctx=f"agg c1 L={levels} ladder<={ladder}") > 0


@pytest.mark.parametrize("levels", [256, 2048])
@pytest.mark.parametrize("max_qty", [1 << 20, 1 << 26])
def test_agg_large_quantities(me, orc, levels, max_qty):
    """Quantities up to 2^20 / 2^26: the ladder's 32-bit totals are exact only while the book's sum stays
    below 2^31, so blocks that could cross it go to the generic loop and books beyond it take the list
    walk (64-bit totals) — level totals past 2^32 included; every batch against the oracle."""
    sc = me.preset(1, levels=levels, batch=8192, max_qty=max_qty)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(10)]
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 512, sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=total + 64,
                 max_chunks=total + 64) as eng:
        assert run_both(eng, ob, batches, ctx=f"agg qty<={max_qty} L={levels}") > 0


@pytest.mark.parametrize("ladder", [None, 0])
@pytest.mark.parametrize("spread", [2, 40, 400])
def test_agg_many_symbols_no_handoff(me, orc, spread, ladder):
    """Every symbol hot (ME_HOT_MIN=1) on a 1,024-level window, no cancels, no far prices: the aggregate
    path alone, with tight spreads (long FIFOs, sweeps through many makers per level) and wide ones
    (deep rests beyond the 64-entry lists, list rebuilds), on the default walk (the bitmap ladder) and on
    the list walk (ME_AGG_LADDER=0)."""
    sc, base, batches = _drift(me, 1024, 40, 8192, 25, cancel_pct=0, far_pct=0, spread_ticks=spread,
                               drift_every=0, drift_step=0, market_qty_mult=4, market_pct=20)
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 1, sc.num_symbols, sc.levels, base, ladder=ladder, max_batch=sc.batch,
                 max_resting=total + 64, max_chunks=total + 64) as eng:
        nf = run_both(eng, ob, batches, ctx=f"agg many spread={spread} ladder={ladder}")
    assert nf > 0


@pytest.mark.parametrize("occ", [256, 0])
@pytest.mark.parametrize("levels", [2048, 32768])
def test_agg_ladder_occ_config1(me, orc, levels, occ):
    """The ladder walk on deep windows (ME_AGG_LADDER=32768) in both next-level forms: the occupancy
    bitmap in LDS (ME_LW_OCC=256: bits set by rests, cleared by the takes that empty a level, one read per
    4,096 levels) and the 64-level scan of the totals (0); config 1's shape, every batch against the
    oracle."""
    sc = me.preset(1, levels=levels, batch=16384)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(8)]
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 512, sc.num_symbols, sc.levels, base, ladder=32768, occ=occ, max_batch=sc.batch,
                 max_resting=total + 64, max_chunks=total + 64) as eng:
        assert run_both(eng, ob, batches, ctx=f"agg c1 L={levels} occ={occ}") > 0


@pytest.mark.parametrize("spread", [2, 400, 3000])
def test_agg_ladder_occ_wide_spreads(me, orc, spread):
    """The bitmap form where it matters: every symbol hot on an 8,192-level window with spreads up to 3,000
    ticks (gaps of hundreds of empty levels between the bests, sweeps emptying level after level, rests at
    the far ends of the window in words no other level shares), no cancels, no far prices."""
    sc, base, batches = _drift(me, 8192, 24, 8192, 20, cancel_pct=0, far_pct=0, spread_ticks=spread,
                               drift_every=0, drift_step=0, market_qty_mult=6, market_pct=20)
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 1, sc.num_symbols, sc.levels, base, ladder=32768, max_batch=sc.batch,
                 max_resting=total + 64, max_chunks=total + 64) as eng:
        assert run_both(eng, ob, batches, ctx=f"agg occ spread={spread}") > 0


def test_agg_ladder_occ_drift_far_cancels(me, orc):
    """The bitmap form behind the generic fallbacks: drifting mids, far LIMITs, cancels and re-centring
    hand symbols to k_match_hot_cont, whose book the next batch's ladder (and bitmap) is rebuilt from."""
    sc, base, batches = _drift(me, 2048, 6, 6144, 40)
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 64, sc.num_symbols, sc.levels, base, ladder=32768, max_batch=sc.batch,
                 max_resting=total + 64, max_chunks=total + 64) as eng:
        assert run_both(eng, ob, batches, ctx="agg occ drift") > 0


def test_agg_ladder_occ_config4(me, orc):
    """Config 4's shape (Zipf symbols, L = 32,768, books seeded to 3,000 levels per side) with the hot
    symbols on the ladder's bitmap form: every batch, and the books, against the oracle."""
    sc = me.preset(4, num_symbols=300, batch=32768)
    st = me.Stream(sc)
    base = st.base_prices()
    seeds = st.seed_books(range(8), 3000)
    batches = [seeds.take(slice(i, i + 32768)) for i in range(0, len(seeds), 32768)]
    batches += [st.next(sc.batch) for _ in range(4)]
    ob = orc.OracleBook(sc.num_symbols)
    total = sum(len(b) for b in batches)
    with _engine(me, 512, sc.num_symbols, sc.levels, base, ladder=32768, max_batch=32768,
                 max_resting=total + 1024, max_chunks=total + 1024) as eng:
        assert run_both(eng, ob, batches, ctx="agg occ c4") > 0
