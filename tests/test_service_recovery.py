"""Restart recovery, book hand-over between symbols and in-band capacity rejection in the SubmitOrder
service (VERDICT r2 items 5, 6 and ADVICE r2: a refused slice must not wedge the service).

  * Restart: the reference resumes only its OID counter from the DB (matching_engine_service.cpp:18-22,
    storage.cpp:254-267); the service also replays every resting order into fresh books, so a run that
    stops and restarts ends with the DB rows and books of an uninterrupted run.
  * Symbols: the reference keeps any non-empty symbol forever (:66-71); the service hands an idle
    symbol's book to a new symbol once every book is taken.
  * Capacity: a slice the backend refuses is split; a LIMIT that still cannot rest is answered in-band
    (REJECTED, ME_RJ_CAPACITY) instead of blocking every later slice.

CPU variants run over one oracle book behind me_service_create_matcher (test infrastructure standing in
for the engine); the GPU variants run the same scenarios on the HIP engine."""
import sqlite3

import numpy as np
import pytest


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


class OracleBackend:
    """me_matcher over ONE oracle book; `cap` emulates admission control (refuse when the resting orders
    plus the slice's LIMIT records could exceed it)."""

    def __init__(self, n, max_batch=4096, max_resting=1 << 16, cap=None):
        from oracle.oracle import OracleBook

        self.ob = OracleBook(n)
        self.num_symbols, self.max_batch, self.max_resting = n, max_batch, max_resting
        self.cap, self.refusals = cap, 0

    def match(self, b):
        from matching_engine_amd.cluster import SliceRefused

        if self.cap is not None and self.ob.resting() + int(np.sum((b.kind & 0x0C) == 0)) > self.cap:
            self.refusals += 1
            raise SliceRefused(-3, "capacity")
        return self.ob.submit(b)

    def book_orders(self, s, depth):
        from tests._parity import side_levels

        depth = depth or (1 << 20)  # 0: the whole book
        d = self.ob.dump(s)
        lb, la = self.ob.snapshot(s, depth)
        return side_levels(d, 1, depth), side_levels(d, 2, depth), lb, la

    def c_matcher(self):
        from matching_engine_amd.cluster import python_matcher

        return python_matcher(self)

    def dump(self, s):
        return self.ob.dump(s)


def _requests(rng, syms, mids, n, live, owner, cancel_p=0.15):
    """SubmitOrder / CancelOrder requests; `live` / `owner` track LIMIT OIDs the caller will assign."""
    out = []
    for _ in range(n):
        if live and rng.random() < cancel_p:
            oid = live[int(rng.integers(len(live)))]
            out.append(("cancel", owner[oid][0], owner[oid][1], oid))
            continue
        s = syms[int(rng.integers(len(syms)))]
        otype = 1 if rng.random() < 0.2 else 0
        out.append(("submit", f"C{int(rng.integers(3))}", s, otype, int(rng.choice([1, 2])),
                    0 if otype else mids[s] + int(rng.integers(-30, 31)), int(rng.integers(1, 60))))
    return out


def _apply(svc, reqs, live, owner):
    for r in reqs:
        if r[0] == "cancel":
            assert svc.cancel_order(r[1], r[2], f"OID-{r[3]}")["success"]
        else:
            resp = svc.submit_order(r[1], r[2], r[3], r[4], r[5], 4, r[6])
            assert resp["success"], resp
            oid = int(resp["order_id"][4:])
            owner[oid] = (r[1], r[2])
            if r[3] == 0:
                live.append(oid)


def _rows(db):
    con = sqlite3.connect(db)
    o = con.execute("SELECT order_id, client_id, symbol, side, order_type, price, quantity, status, "
                    "remaining_quantity FROM orders ORDER BY order_id").fetchall()
    f = con.execute("SELECT id, order_id, symbol, fill_price, fill_quantity FROM fills ORDER BY id").fetchall()
    con.close()
    return o, f


def _scenario(rng_seed, syms, mids):
    """Two request phases generated up front (phase 2 cancels phase-1 orders too). The OIDs are the
    service's: 1, 2, ... for accepted SubmitOrders in request order (cancels consume none)."""
    rng = np.random.default_rng(rng_seed)
    live, owner = [], {}
    # phase 1 needs the OIDs to plan phase-2 cancels: simulate the allocation
    p1 = _requests(rng, syms, mids, 1800, [], {}, cancel_p=0.0)
    oid = 0
    for r in p1:
        oid += 1
        owner[oid] = (r[1], r[2])
        if r[3] == 0:
            live.append(oid)
    p2 = _requests(rng, syms, mids, 1800, live, owner, cancel_p=0.2)
    return p1, p2


def _run_restart(me, tmp_path, make_backend, dump_of, nsym):
    syms = [f"R{i}" for i in range(nsym)]
    mids = {s: 2_000_000 + 700 * i for i, s in enumerate(syms)}
    p1, p2 = _scenario(3, syms, mids)
    # uninterrupted
    db_a = str(tmp_path / "a.sqlite")
    ba = make_backend()
    sa = me.MatchingEngineService(*ba[0], syms[:2], db_path=db_a, **ba[1])
    live, owner = [], {}
    _apply(sa, p1, live, owner)
    sa.flush()
    _apply(sa, p2, live, owner)
    sa.flush()
    ua = sa.order_updates(cap=1 << 20)
    books_a = {s: sa.order_book(s) for s in syms}
    assert sum(len(b) + len(a) for b, a in books_a.values()) > 100  # the comparison below is not vacuous
    # stop after phase 1, restart over fresh books on the same DB, phase 2
    db_b = str(tmp_path / "b.sqlite")
    b1 = make_backend()
    s1 = me.MatchingEngineService(*b1[0], syms[:2], db_path=db_b, **b1[1])
    live, owner = [], {}
    _apply(s1, p1, live, owner)
    s1.flush()
    u1 = s1.order_updates(cap=1 << 20)
    resting = sum(len(dump_of(b1, k)) for k in range(nsym))
    s1.close()
    b2 = make_backend()
    s2 = me.MatchingEngineService(*b2[0], syms[:2], db_path=db_b, **b2[1])
    assert s2.last_error() == ""
    st = s2.stats()
    assert st["recovered_orders"] == resting > 100, (st, resting)
    assert s2.next_oid == s1_next(p1)
    assert s2.order_updates() == []  # the replay of resting orders emits nothing new
    _apply(s2, p2, live, owner)
    s2.flush()
    u2 = s2.order_updates(cap=1 << 20)
    assert _rows(db_a) == _rows(db_b)
    assert u1 + u2 == ua  # the OrderUpdate stream is the uninterrupted run's
    for s in syms:  # books (incl. client ids of recovered orders) equal the uninterrupted run's
        assert s2.order_book(s) == books_a[s], s
    return sa, s2


def s1_next(p1):
    return len(p1) + 1


def test_restart_rebuilds_books_oracle(me, tmp_path):
    """CPU: stop -> recreate over fresh books on the same DB -> match -> cancel recovered orders: DB,
    OrderUpdates and books equal an uninterrupted run's."""
    def make():
        b = OracleBackend(8)
        return (None,), {"matcher": b}
    _run_restart(me, tmp_path, make, lambda b, k: b[1]["matcher"].dump(k), 8)


@pytest.mark.gpu
def test_restart_rebuilds_books_engine(me, tmp_path):
    """GPU: the same on the HIP engine — recovery replays the DB's resting orders
    into a new engine's books before the first new order."""
    base = np.array([2_000_000 + 700 * i - 64 for i in range(8)], dtype=np.int64)

    def make():
        e = me.Engine(8, 128, base, max_batch=4096, max_resting=1 << 14)
        return (e,), {}
    _run_restart(me, tmp_path, make, lambda b, k: b[0][0].dump(k), 8)


def _run_reclaim(me, tmp_path, svc_small, svc_big):
    """Phases of 3 fresh symbols each: orders trade, then every resting order is cancelled, so each
    phase's books end empty and the next phase's symbols take them over (3 books, 15 symbols)."""
    rng = np.random.default_rng(9)
    outs = []
    for svc in (svc_small, svc_big):
        rng = np.random.default_rng(9)
        live_all = []
        for ph in range(5):
            syms = [f"P{ph}_{k}" for k in range(3)]
            mids = {s: 1_000_000 + 5000 * ph + 300 * k for k, s in enumerate(syms)}
            live, owner = [], {}
            _apply(svc, _requests(rng, syms, mids, 400, [], {}, cancel_p=0.0), live, owner)
            svc.flush()
            for oid in live:  # cancel whatever still rests
                c, s = owner[oid]
                assert svc.cancel_order(c, s, f"OID-{oid}")["success"]
            svc.flush()
            live_all += live
        outs.append(svc.order_updates(cap=1 << 20))
    assert outs[0] == outs[1]
    return outs


def test_idle_symbol_books_are_handed_over_oracle(me, tmp_path):
    """CPU: more distinct symbols over time than books — every order matches and
    persists as with room for all of them; a new symbol is refused only while every book holds orders."""
    small, big = OracleBackend(3), OracleBackend(32)
    dbs = [str(tmp_path / "small.sqlite"), str(tmp_path / "big.sqlite")]
    s_small = me.MatchingEngineService(None, [], db_path=dbs[0], matcher=small)
    s_big = me.MatchingEngineService(None, [], db_path=dbs[1], matcher=big)
    _run_reclaim(me, tmp_path, s_small, s_big)
    assert _rows(dbs[0]) == _rows(dbs[1])
    assert s_small.stats()["reclaimed_books"] >= 12
    # every book busy: a resting order on each of 3 symbols, then a 4th symbol is refused (no OID)
    for k in range(3):
        assert s_small.submit_order("C", f"Z{k}", 0, 1, 100, 4, 1)["success"]
    s_small.flush()
    r = s_small.submit_order("C", "Z3", 0, 1, 100, 4, 1)
    assert r["grpc_status"] == 8 and r["order_id"] == "" and not r["success"]
    nxt = s_small.next_oid
    assert s_small.cancel_order("C", "Z0", f"OID-{nxt - 3}")["success"]  # Z0's book empties ...
    s_small.flush()
    assert s_small.submit_order("C", "Z3", 0, 1, 100, 4, 1)["success"]  # ... and Z3 takes it
    s_small.flush()
    assert s_small.order_book("Z3")[0][0]["order_id"] == f"OID-{nxt}"
    assert s_small.order_book("Z0") == ([], [])


@pytest.mark.gpu
def test_idle_symbol_books_are_handed_over_engine(me, tmp_path):
    """GPU: the same with an engine of 3 books (windows re-centre on each new symbol's prices)."""
    small = me.Engine(3, 128, np.full(3, 1_000_000, dtype=np.int64), max_batch=4096, max_resting=1 << 14)
    big = me.Engine(32, 128, np.full(32, 1_000_000, dtype=np.int64), max_batch=4096, max_resting=1 << 14)
    dbs = [str(tmp_path / "small.sqlite"), str(tmp_path / "big.sqlite")]
    s_small = me.MatchingEngineService(small, [], db_path=dbs[0])
    s_big = me.MatchingEngineService(big, [], db_path=dbs[1])
    _run_reclaim(me, tmp_path, s_small, s_big)
    assert _rows(dbs[0]) == _rows(dbs[1])
    assert s_small.stats()["reclaimed_books"] >= 12


def _run_capacity(me, svc, backend_refusals):
    """200 LIMITs that all rest against a capacity of 50: 50 rest, 150 come back REJECTED
    (ME_RJ_CAPACITY) in the same flush; cancels free room and later LIMITs rest again."""
    oids = [int(svc.submit_order("C", "CAP", 0, 1, 1_000_000 - 1 - k, 4, 1)["order_id"][4:]) for k in range(200)]
    seq, res, _ = svc.flush()
    assert svc.last_error() == ""
    st = res["status"]
    assert int(np.sum(st == me.ST_NEW)) == 50 and int(np.sum(st == me.ST_REJECTED)) == 150
    assert np.all(res["reason"][st == me.ST_REJECTED] == 7)  # ME_RJ_CAPACITY
    assert backend_refusals() > 0
    ev = svc.order_updates(cap=1 << 20)
    assert sum(1 for e in ev if e["status"] == me.ST_REJECTED) == 150
    rested = [o for o, s in zip(oids, st) if s == me.ST_NEW]
    for o in rested[:10]:
        assert svc.cancel_order("C", "CAP", f"OID-{o}")["success"]
    for k in range(10):
        svc.submit_order("C", "CAP", 0, 1, 900_000 - k, 4, 1)
    seq, res, _ = svc.flush()
    assert svc.last_error() == ""
    assert int(np.sum(res["status"] == me.ST_CANCELED)) == 10 and int(np.sum(res["status"] == me.ST_NEW)) == 10


def test_capacity_refusal_answers_in_band_oracle(me, tmp_path):
    """CPU: a backend at capacity no longer wedges the service."""
    b = OracleBackend(1, cap=50)
    svc = me.MatchingEngineService(None, ["CAP"], db_path=str(tmp_path / "cap.sqlite"), matcher=b)
    _run_capacity(me, svc, lambda: b.refusals)
    con = sqlite3.connect(str(tmp_path / "cap.sqlite"))
    assert con.execute("SELECT COUNT(*) FROM orders WHERE status = 4").fetchone()[0] == 150
    con.close()


@pytest.mark.gpu
def test_capacity_refusal_answers_in_band_engine(me, tmp_path):
    """GPU: the engine's admission control at max_resting = 50."""
    e = me.Engine(1, 128, np.array([1_000_000 - 64], dtype=np.int64), max_batch=4096, max_resting=50)
    svc = me.MatchingEngineService(e, ["CAP"], db_path=str(tmp_path / "cap.sqlite"))
    _run_capacity(me, svc, lambda: e.admission()["exact_counts"])
