"""The pipelined host-batch path (me_submit_host / me_collect, include/me_engine.h): host SoA batches
staged in pinned slots, H2D on their own stream, matched in launch groups, results and tapes D2H'd
behind the match — every batch's outputs bit-exact against the oracle, whatever the collect lag,
including tapes longer than a slot (recovered from scratch at collect). Needs an MI355X."""
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


def _stream(me, cfg, nbatches, **over):
    sc = me.preset(cfg, **over)
    st = me.Stream(sc)
    return sc, st.base_prices(), [st.next(sc.batch) for _ in range(nbatches)]


def _engine(me, sc, base, batches, **kw):
    total = sum(len(b) for b in batches)
    return me.Engine(sc.num_symbols, sc.levels, base, max_batch=max(len(b) for b in batches),
                     max_resting=total + 1024, max_chunks=total + 2 * sc.num_symbols, seq_ring=1 << 22, **kw)


def _pipelined(me, eng, batches, lag, zero_copy_every=0):
    """Submit every batch through me_submit_host, collecting each `lag` submissions later (in order);
    returns the outputs per batch. zero_copy_every = k: every k-th batch is written straight into the
    pinned slot (me_host_inputs) instead of being staged by the engine."""
    out, tickets = [None] * len(batches), []
    for k, b in enumerate(batches):
        if zero_copy_every and k % zero_copy_every == 0:
            w = eng.host_inputs(len(b))
            for f in ("seq", "price_q4", "qty", "symbol", "kind"):
                getattr(w, f)[:] = getattr(b, f)
            b = w
        tickets.append((k, eng.submit_host(b)))
        while len(tickets) > lag:
            j, t = tickets.pop(0)
            out[j] = eng.collect(t)
    for j, t in tickets:
        out[j] = eng.collect(t)
    return out


@pytest.mark.parametrize("levels,group,lag", [(128, 4, 1), (128, 4, 12), (128, 32, 96), (128, 8, 32), (512, 1, 3)])
def test_host_pipeline_every_batch(me, orc, levels, group, lag):
    sc, base, batches = _stream(me, 2, 40, num_symbols=64, levels=levels, batch=2048)
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=group) as eng:
        assert eng.config()["host_slots"] == 4 * eng.config()["batches_per_launch"] + 1
        outs = _pipelined(me, eng, batches, lag, zero_copy_every=3)
        for k, b in enumerate(batches):
            ro, fo = ob.submit(b)
            assert_results_equal(outs[k][0], ro, f"L={levels} G={group} lag={lag} batch {k}")
            assert_fills_equal(outs[k][1], fo, f"L={levels} G={group} lag={lag} batch {k}")
        assert_books_equal(eng, ob, range(sc.num_symbols), "host pipeline")


@pytest.mark.parametrize("levels", [128, 512])
def test_host_tape_longer_than_slot(me, orc, levels):
    """host_tape_cap = 64 fills: market sweeps outgrow the slot and the tail comes from scratch."""
    sc, base, batches = _stream(me, 5, 12, num_symbols=16, levels=levels, batch=2048)
    ob = orc.OracleBook(sc.num_symbols)
    spilled = 0
    with _engine(me, sc, base, batches, batches_per_launch=2, host_tape_cap=64) as eng:
        for k, (r, f) in enumerate(_pipelined(me, eng, batches, lag=2)):
            ro, fo = ob.submit(batches[k])
            assert_results_equal(r, ro, f"spill L={levels} batch {k}")
            assert_fills_equal(f, fo, f"spill L={levels} batch {k}")
            spilled += len(fo) > 64
        assert_books_equal(eng, ob, range(sc.num_symbols), "spill")
    assert spilled >= 6


def test_host_tape_longer_than_batch(me, orc):
    """Sweeping MARKETs give batches with more fills than records: the slot's DMA carries the first
    n fills, me_collect copies the rest from the slot's HBM block (below host_tape_cap, no spill)."""
    sc, base, _ = _stream(me, 2, 0, num_symbols=16, batch=1024)
    rng = np.random.default_rng(4)
    batches, seq = [], 1
    for k in range(12):
        if k % 2 == 0:  # 1,024 one-lot LIMITs on both sides, 1..40 ticks from the mid
            n = 1024
            side = rng.integers(1, 3, n)
            off = rng.integers(1, 41, n)
            sym = rng.integers(0, 16, n)
            px = base[sym] + 64 + np.where(side == 1, -off, off)
            kind = [me.kind(int(s)) for s in side]
            qty = np.ones(n, np.int32)
        else:  # 48 MARKETs of 40 lots: ~2,000 fills from 48 records
            n = 48
            side = rng.integers(1, 3, n)
            sym = rng.integers(0, 16, n)
            px = np.zeros(n, np.int64)
            kind = [me.kind(int(s), me.TYPE_MARKET) for s in side]
            qty = np.full(n, 40, np.int32)
        batches.append(me.Batch(np.arange(seq, seq + n, dtype=np.uint64), px, qty, sym, kind))
        seq += n
    ob = orc.OracleBook(sc.num_symbols)
    longer = 0
    with _engine(me, sc, base, batches, batches_per_launch=4) as eng:
        for k, (r, f) in enumerate(_pipelined(me, eng, batches, lag=3)):
            ro, fo = ob.submit(batches[k])
            assert_results_equal(r, ro, f"long tape batch {k}")
            assert_fills_equal(f, fo, f"long tape batch {k}")
            longer += len(fo) > len(batches[k])
        assert_books_equal(eng, ob, range(sc.num_symbols), "long tape")
    assert longer >= 3


def test_host_pipeline_drifting_handoffs(me, orc):
    """Host batches on a drifting far-price stream (hand-offs to the continuation launch, window
    re-centring, far levels, cancels, OIDs above 2^33) at G = 32 with a 40-batch collect lag: every
    batch's outputs from its pinned slot against the oracle."""
    sc = me.preset(5, num_symbols=256, levels=128, batch=4096, cancel_pct=10, market_pct=15, market_qty_mult=3,
                   drift_step=1, drift_every=3, far_pct=1, seq_start=(1 << 33) + 5)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(96)]
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=32) as eng:
        for k, (r, f) in enumerate(_pipelined(me, eng, batches, lag=40)):
            ro, fo = ob.submit(batches[k])
            assert_results_equal(r, ro, f"drift host batch {k}")
            assert_fills_equal(f, fo, f"drift host batch {k}")
        assert_books_equal(eng, ob, range(sc.num_symbols), "drift host")
        assert eng.stats()["handoffs"] > 0


def test_host_slot_reuse_needs_collect(me, orc):
    sc, base, batches = _stream(me, 2, 6, num_symbols=32, batch=512)
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=2, host_slots=3) as eng:
        t = [eng.submit_host(b) for b in batches[:3]]
        with pytest.raises(me.EngineError) as ei:
            eng.submit_host(batches[3])
        assert ei.value.code == me.ME_E_STATE and "collect ticket 0" in str(ei.value)
        with pytest.raises(me.EngineError):
            eng.host_inputs(len(batches[3]))
        outs = [eng.collect(x) for x in t]
        with pytest.raises(me.EngineError):  # collected once only
            eng.collect(t[0])
        outs += [eng.collect(eng.submit_host(b)) for b in batches[3:]]
        for k, b in enumerate(batches):
            ro, fo = ob.submit(b)
            assert_results_equal(outs[k][0], ro, f"reuse batch {k}")
            assert_fills_equal(outs[k][1], fo, f"reuse batch {k}")


def test_host_and_device_batches_interleave(me, orc):
    """Host and device batches share the launch groups and the books; the device-output fetches refuse
    to read a host batch's outputs."""
    sc, base, batches = _stream(me, 2, 8, num_symbols=64, batch=1024)
    ob = orc.OracleBook(sc.num_symbols)
    with _engine(me, sc, base, batches, batches_per_launch=4) as eng:
        for k, b in enumerate(batches):
            ro, fo = ob.submit(b)
            if k % 2:
                db = eng.upload(b)
                eng.submit_device(db)
                r, f = eng.fetch_outputs(len(b))
                db.free()
            else:
                r, f = eng.collect(eng.submit_host(b))
                with pytest.raises(me.EngineError, match="host batch"):
                    eng.fetch_outputs(len(b))
            assert_results_equal(r, ro, f"interleave batch {k}")
            assert_fills_equal(f, fo, f"interleave batch {k}")


def test_collected_outputs_survive_the_next_submit(me, orc):
    """me_collect's outputs (pinned views, copy=False) stay valid until the next me_collect: collect A,
    submit and match C (the LIFO free list would hand C A's slot), then read A — still A's results and
    tape. (the cluster's world-1 direct path hands exactly these views to its caller.)"""
    sc, base, batches = _stream(me, 2, 6, num_symbols=64, batch=2048)
    ob = orc.OracleBook(sc.num_symbols)
    exp = [ob.submit(b) for b in batches]
    with _engine(me, sc, base, batches, batches_per_launch=2) as eng:
        t = [eng.submit_host(b) for b in batches[:2]]
        views = eng.collect(t[0], copy=False)
        t.append(eng.submit_host(batches[2]))
        eng.sync()  # C matched and its outputs written
        assert_results_equal(views[0], exp[0][0], "A after C's submit")
        assert_fills_equal(views[1], exp[0][1], "A after C's submit")
        for k in (1, 2):
            r, f = eng.collect(t[k])
            assert_results_equal(r, exp[k][0], f"batch {k}")
            assert_fills_equal(f, exp[k][1], f"batch {k}")
        # a synchronous caller alternates two warm slots; any lag keeps working
        for k in range(3, 6):
            r, f = eng.collect(eng.submit_host(batches[k]))
            assert_results_equal(r, exp[k][0], f"batch {k}")
            assert_fills_equal(f, exp[k][1], f"batch {k}")
