"""Admission control (me_config.max_resting, me_engine.cpp admit): a batch that could take the
resting orders past max_resting is refused with ME_E_CAPACITY before anything of it is enqueued —
the books are unchanged and the engine keeps matching (the error is not sticky). The device's
resting counter (ST_RESTING, published by k_seq_sweep) equals the per-symbol counts and the oracle.
Needs an MI355X."""
import numpy as np
import pytest

from tests._parity import assert_books_equal, assert_fills_equal, assert_results_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


S, L, MID = 8, 128, 1_000_000


class Seqs:
    def __init__(self):
        self.next = 1

    def take(self, n):
        s = np.arange(self.next, self.next + n, dtype=np.uint64)
        self.next += n
        return s


def _passive(me, seqs, n, rng):
    """n LIMIT orders that never cross: bids below the mid, asks above it."""
    side = rng.choice([me.SIDE_BUY, me.SIDE_SELL], n)
    px = np.where(side == me.SIDE_BUY, MID - rng.integers(1, 40, n), MID + rng.integers(1, 40, n))
    return me.Batch(seqs.take(n), px.astype(np.int64), rng.integers(1, 50, n).astype(np.int32),
                    rng.integers(0, S, n).astype(np.uint32), np.array([me.kind(int(s)) for s in side], np.uint8))


def _market(me, seqs, n, rng):
    side = rng.choice([me.SIDE_BUY, me.SIDE_SELL], n)
    return me.Batch(seqs.take(n), np.zeros(n, np.int64), rng.integers(1, 50, n).astype(np.int32),
                    rng.integers(0, S, n).astype(np.uint32),
                    np.array([me.kind(int(s), me.TYPE_MARKET) for s in side], np.uint8))


def _engine(me, max_resting, **kw):
    return me.Engine(S, L, [MID - 64] * S, max_batch=2048, max_resting=max_resting, seq_ring=1 << 20, **kw)


@pytest.mark.parametrize("mode", ["host", "device", "generic"])
def test_refused_batch_leaves_engine_usable(me, mode):
    from oracle.oracle import OracleBook

    rng = np.random.default_rng(21)
    seqs = Seqs()
    kw = {"levels": 256} if mode == "generic" else {}
    eng = me.Engine(S, kw.get("levels", L), [MID - 128 if mode == "generic" else MID - 64] * S, max_batch=2048,
                    max_resting=5000, seq_ring=1 << 20)
    ob = OracleBook(S)

    def run(b):
        if mode == "device":
            db = eng.upload(b)
            try:
                eng.submit_device(db)
                r, f = eng.fetch_outputs(len(b))
            finally:
                db.free()
        else:
            r, f = eng.submit_batch(b)
        ro, fo = ob.submit(b)
        assert_results_equal(r, ro, mode)
        assert_fills_equal(f, fo, mode)

    for _ in range(3):
        run(_passive(me, seqs, 1500, rng))
    assert eng.admission()["resting"] == 4500 == ob.resting()
    refused = _passive(me, seqs, 1500, rng)  # 4500 + 1500 > 5000
    with pytest.raises(me.EngineError) as ei:
        if mode == "device":
            db = eng.upload(refused)
            try:
                eng.submit_device(db)
            finally:
                db.free()
        else:
            eng.submit_batch(refused)
    assert ei.value.code == me.ME_E_CAPACITY and "refused" in str(ei.value)
    # nothing of it reached the books; the engine keeps going (seqs skip the refused batch's ids)
    assert eng.resting_count() == 4500
    run(_market(me, seqs, 400, rng))  # 4500 + 400 fits; each market order removes makers
    left = ob.resting()
    assert eng.admission()["resting"] == left < 4500
    run(_passive(me, seqs, 5000 - left, rng))  # exactly up to the cap
    assert eng.admission()["resting"] == 5000
    with pytest.raises(me.EngineError):
        run(_passive(me, seqs, 1, rng))
    assert_books_equal(eng, ob, range(S), mode)
    assert eng.admission()["exact_counts"] >= 2
    eng.close()


def test_host_runs_ahead_without_exact_counts(me):
    """Back-to-back device batches far beyond max_resting in total (each market batch removes what
    the passive one adds): the published count keeps the bound honest, so no submit has to drain
    the pipeline, and the books equal the oracle's."""
    from oracle.oracle import OracleBook

    rng = np.random.default_rng(5)
    seqs = Seqs()
    eng = _engine(me, 40_000, batches_per_launch=8)
    ob = OracleBook(S)
    dbs, all_b = [], []
    for k in range(96):
        b = _passive(me, seqs, 1000, rng) if k % 2 == 0 else _market(me, seqs, 1000, rng)
        all_b.append(b)
        dbs.append(eng.upload(b))
    for db in dbs:
        eng.submit_device(db)
    eng.sync()
    for b in all_b:
        ob.submit(b)
    adm = eng.admission()
    assert adm["resting"] == ob.resting() == eng.resting_count()
    assert adm["exact_counts"] <= 2, adm  # 96k records accepted against a 40k cap, by the published count
    assert_books_equal(eng, ob, range(S), "run-ahead")
    for db in dbs:
        db.free()
    eng.close()


def test_admission_check_enqueues_nothing(me):
    """me_admission_check (Engine.admits): the all-or-none question a sharded matcher asks every shard
    before any applies its part — true / false as submit would decide, with nothing enqueued."""
    rng = np.random.default_rng(9)
    seqs = Seqs()
    eng = _engine(me, 3000)
    a = _passive(me, seqs, 2000, rng)
    assert eng.admits(a)
    eng.submit_batch(a)
    big = _passive(me, seqs, 1500, rng)
    assert not eng.admits(big)
    small = _passive(me, seqs, 1000, rng)
    assert eng.admits(small)
    assert eng.admission()["resting"] == 2000  # the checks enqueued nothing
    assert eng.admits(_market(me, seqs, 1500, rng))  # MARKETs never rest
    eng.submit_batch(small)
    assert eng.admission()["resting"] == 3000
    eng.close()
