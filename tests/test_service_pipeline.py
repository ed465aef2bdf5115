"""The service's two stages on CPU: slices are matched on the flushing thread and handed to the
persister thread (OrderUpdates, then one SQLite transaction per slice). The matcher here is the CPU
oracle behind me_service_create_matcher (test infrastructure standing in for the engine), so the
stage hand-off, the stalled-DB retry and the drain on stop run without a GPU."""
import sqlite3
import time

import numpy as np
import pytest


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


class OracleMatcher:
    """The me_matcher contract (match / book_orders) over one OracleBook holding every symbol."""

    def __init__(self, n, max_batch=4096, max_resting=1 << 16):
        from oracle.oracle import OracleBook

        self.ob = OracleBook(n)
        self.num_symbols, self.max_batch, self.max_resting = n, max_batch, max_resting
        self._cmatcher = None
        self.slices = 0

    def match(self, b):
        self.slices += 1
        return self.ob.submit(b)

    def book_orders(self, s, depth):
        from tests._parity import side_levels

        d = self.ob.dump(s)
        lb, la = self.ob.snapshot(s, depth)
        return side_levels(d, 1, depth), side_levels(d, 2, depth), lb, la

    def c_matcher(self):
        from matching_engine_amd.cluster import python_matcher

        return python_matcher(self)


def _stream(rng, syms, mids, n):
    out = []
    for _ in range(n):
        s = syms[int(rng.integers(len(syms)))]
        otype = 1 if rng.random() < 0.2 else 0
        out.append((s, otype, int(rng.choice([1, 2])), 0 if otype else mids[s] + int(rng.integers(-20, 21)),
                    int(rng.integers(1, 50))))
    return out


def _submit(svc, reqs):
    return [int(svc.submit_order("C", *r[:4], 4, r[4])["order_id"][4:]) for r in reqs]


def _expect(me, reqs, oids, sid):
    from oracle.oracle import OracleBook

    ob = OracleBook(len(sid))
    b = me.Batch(oids, [r[3] for r in reqs], [r[4] for r in reqs], [sid[r[0]] for r in reqs],
                 [me.kind(r[2], r[1]) for r in reqs])
    ro, fo = ob.submit(b)
    return ob, ro, fo


def _check_db(db, ob, nsym, n_orders, n_fills):
    con = sqlite3.connect(db)
    assert con.execute("SELECT COUNT(*) FROM orders").fetchone()[0] == n_orders
    assert con.execute("SELECT COUNT(*) FROM fills").fetchone()[0] == 2 * n_fills
    rows = dict(con.execute("SELECT order_id, remaining_quantity FROM orders").fetchall())
    for s in range(nsym):  # every resting order's row carries the oracle's live remainder
        for e in ob.dump(s):
            assert rows[f"OID-{int(e['seq'])}"] == int(e["qty"])
    con.close()


def test_stalled_db_keeps_updates_flowing_and_retries_in_order(me, tmp_path):
    """A slice matched while another connection holds the write lock: its OrderUpdates still go out,
    the flush reports the deferred transaction, and the next flush commits it before the new slice —
    every slice matched exactly once."""
    rng = np.random.default_rng(5)
    syms = ["X", "Y", "Z"]
    mids = {"X": 1_000_000, "Y": 1_500_000, "Z": 2_000_000}
    sid = {s: i for i, s in enumerate(syms)}
    db = str(tmp_path / "stall.sqlite")
    m = OracleMatcher(3)
    svc = me.MatchingEngineService(None, syms, db_path=db, matcher=m)
    reqs, oids = [], []
    r1 = _stream(rng, syms, mids, 900)
    oids += _submit(svc, r1)
    reqs += r1
    svc.flush()
    assert svc.unpersisted == 0
    n_ev1 = len(svc.order_updates())
    locker = sqlite3.connect(db, timeout=0.1)
    locker.execute("BEGIN EXCLUSIVE")
    r2 = _stream(rng, syms, mids, 700)
    oids += _submit(svc, r2)
    reqs += r2
    with pytest.raises(me.ServiceError, match="persistence deferred"):
        svc.flush()
    assert svc.pending == 0 and svc.unpersisted == 700
    assert len(svc.order_updates()) > 0  # slice 2's events are out although its rows are not
    locker.rollback()
    locker.close()
    r3 = _stream(rng, syms, mids, 400)
    oids += _submit(svc, r3)
    reqs += r3
    svc.flush()
    assert svc.unpersisted == 0 and m.slices == 3
    ob, ro, fo = _expect(me, reqs, oids, sid)
    _check_db(db, ob, 3, 2000, len(fo))
    assert n_ev1 > 0
    svc.close()


def test_background_pipeline_drains_on_stop(me, tmp_path):
    """The background flusher runs ahead of the persister (slices of 250): when stop returns, every
    slice it matched is committed and its events are out; the DB equals the oracle's final state."""
    rng = np.random.default_rng(8)
    syms = [f"P{i}" for i in range(8)]
    mids = {s: 3_000_000 + 900 * i for i, s in enumerate(syms)}
    sid = {s: i for i, s in enumerate(syms)}
    db = str(tmp_path / "bg.sqlite")
    m = OracleMatcher(8)
    svc = me.MatchingEngineService(None, syms, db_path=db, matcher=m)
    svc.start(interval_us=500, slice_orders=250)
    reqs = _stream(rng, syms, mids, 5000)
    oids = _submit(svc, reqs)
    t0 = time.time()
    while (svc.pending or svc.unpersisted) and time.time() - t0 < 60:
        time.sleep(0.002)
    svc.stop()
    assert svc.last_error() == "" and svc.pending == 0 and svc.unpersisted == 0
    assert m.slices >= 20
    ob, ro, fo = _expect(me, reqs, oids, sid)
    _check_db(db, ob, 8, 5000, len(fo))
    ev = svc.order_updates(cap=1 << 20)
    assert sum(e["fill_quantity"] for e in ev) == 2 * int(fo["qty"].sum())
    svc.close()
