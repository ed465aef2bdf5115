"""SubmitOrder drop-in (include/me_service.h): responses, OID sequence/reseed and persisted rows
against the reference contract (tests/golden/submit_contract.json), and the matched outcome of
requests flowing through SubmitOrder against the oracle."""
import json
import os
import sqlite3

import numpy as np
import pytest

from tests._parity import assert_fills_equal, assert_results_equal, side_levels

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


def _cases():
    return json.load(open(os.path.join(GOLD, "submit_contract.json")))["cases"]


def _submit_all(svc, cases):
    out = []
    for c in cases:
        r = c["request"]
        out.append(svc.submit_order("C1", r["symbol"], r["order_type"], r["side"], r["price"], r["scale"],
                                    r["quantity"]))
    return out


def test_submit_responses_match_reference_contract(me):
    svc = me.MatchingEngineService(None, ["SYM", "ABC"])
    for c, got in zip(_cases(), _submit_all(svc, _cases())):
        exp = dict(c["expect"])
        exp.pop("row")
        assert got == exp, (c["cite"], got, exp)
    # accepted orders wait in the time slice; without an engine the flush fails loudly
    assert svc.pending == sum(1 for c in _cases() if c["expect"]["row"] is not None)
    with pytest.raises(me.ServiceError, match="engine"):
        svc.flush()


def test_oid_reseeded_from_existing_db(me, tmp_path):
    # Impl ctor seeds next_id from MAX(OID)+1 (matching_engine_service.cpp:18-22, storage.cpp:254-267)
    db = str(tmp_path / "seed.sqlite")
    svc = me.MatchingEngineService(None, ["SYM"], db_path=db)
    assert svc.next_oid == 1  # fresh DB
    svc.close()
    con = sqlite3.connect(db)
    con.execute("INSERT INTO orders VALUES ('OID-41','C','SYM',1,1,100,1,0,1,0,0)")
    con.execute("INSERT INTO orders VALUES ('OID-7','C','SYM',1,1,100,1,0,1,0,0)")
    con.execute("INSERT INTO orders VALUES ('X-99','C','SYM',1,1,100,1,0,1,0,0)")
    con.commit()
    con.close()
    svc = me.MatchingEngineService(None, ["SYM"], db_path=db)
    assert svc.next_oid == 42
    r = svc.submit_order("C", "SYM", 0, 1, 100, 4, 1)
    assert r["order_id"] == "OID-42"


def test_schema_matches_reference(me, tmp_path):
    db = str(tmp_path / "schema.sqlite")
    me.MatchingEngineService(None, ["SYM"], db_path=db).close()
    con = sqlite3.connect(db)
    cols = [r[1] for r in con.execute("PRAGMA table_info(orders)")]
    assert cols == ["order_id", "client_id", "symbol", "side", "order_type", "price", "quantity", "status",
                    "remaining_quantity", "created_ts", "updated_ts"]
    cols = [r[1] for r in con.execute("PRAGMA table_info(fills)")]
    assert cols == ["id", "order_id", "symbol", "fill_price", "fill_quantity", "event_ts"]
    assert con.execute("PRAGMA journal_mode").fetchone()[0] == "wal"


@pytest.mark.gpu
def test_persisted_rows_match_reference(me, tmp_path):
    """tests/test_submit_order.cpp:56-79 plus the whole contract: rows as insert_new_order writes them."""
    db = str(tmp_path / "server_test.sqlite")
    # 128-level windows far from the contract's prices (Q4 0 .. 10^9): every order rests through the
    # far levels and window re-centring, as an unbounded book must
    base = [5_000_000, 5_000_000]
    with me.Engine(2, 128, base, max_batch=1024, max_resting=1024) as eng:
        svc = me.MatchingEngineService(eng, ["SYM", "ABC"], db_path=db)
        got = _submit_all(svc, _cases())
        svc.flush()
        con = sqlite3.connect(db)
        for c, g in zip(_cases(), got):
            row = c["expect"]["row"]
            if row is None:
                if g["order_id"]:
                    assert con.execute("SELECT COUNT(*) FROM orders WHERE order_id=?", (g["order_id"],)).fetchone()[0] == 0
                continue
            db_row = con.execute("SELECT price, order_type, side, quantity, symbol, client_id FROM orders "
                                 "WHERE order_id=?", (g["order_id"],)).fetchone()
            assert db_row[:4] == (row["price"], 1, row["side"], row["quantity"]), c["cite"]
        # test_submit_order.cpp:79: 10050 @ scale 8 -> persisted price 1
        assert con.execute("SELECT price FROM orders WHERE order_id='OID-1'").fetchone()[0] == 1
    del base


@pytest.mark.gpu
def test_submitorder_stream_matches_oracle_and_db(me, tmp_path):
    """Raw requests (mixed scales, invalid ones included) through SubmitOrder -> GPU slices ->
    SQLite; the tape/results equal the oracle service + oracle book, and the DB reflects them."""
    from oracle.oracle import OracleBook, OracleService

    rng = np.random.default_rng(7)
    syms = [f"S{i}" for i in range(16)]
    mids = {s: 1_000_000 + 1000 * i for i, s in enumerate(syms)}
    base = np.array([mids[s] - 64 for s in syms], dtype=np.int64)
    db = str(tmp_path / "flow.sqlite")
    eng = me.Engine(len(syms), 128, base, max_batch=4096, max_resting=1 << 14)
    svc = me.MatchingEngineService(eng, syms, db_path=db)
    osvc = OracleService(1)
    ob = OracleBook(len(syms))
    all_fills = 0
    for slice_no in range(4):
        seqs, px, qty, sid, kinds = [], [], [], [], []
        for _ in range(1500):
            s = syms[int(rng.integers(len(syms)))]
            otype = 1 if rng.random() < 0.2 else 0
            side = int(rng.choice([1, 2, 1, 2, 0])) if rng.random() < 0.02 else int(rng.choice([1, 2]))
            q4 = mids[s] + int(rng.integers(-30, 31))
            scale = int(rng.choice([4, 4, 4, 2, 8]))
            price = q4 // 100 if scale == 2 else (q4 * 10000 if scale == 8 else q4)
            if otype == 1:
                price = 0
            qn = int(rng.integers(-2, 100))
            a = svc.submit_order("C", s, otype, side, price, scale, qn)
            b = osvc.submit(s, otype, side, price, scale, qn)
            assert a == {k: b[k] for k in a}, (a, b)
            if b["row"] is not None:
                seqs.append(int(b["order_id"][4:]))
                px.append(b["row"]["price"])
                qty.append(qn)
                sid.append(syms.index(s))
                kinds.append(me.kind(side, otype))
        seq, res, fills = svc.flush()
        ob_b = me.Batch(seqs, px, qty, sid, kinds)
        ro, fo = ob.submit(ob_b)
        assert np.array_equal(seq, np.array(seqs, dtype=np.uint64))
        assert_results_equal(res, ro, f"slice {slice_no}")
        assert_fills_equal(fills, fo, f"slice {slice_no}")
        all_fills += len(fo)
    con = sqlite3.connect(db)
    assert con.execute("SELECT COUNT(*) FROM fills").fetchone()[0] == 2 * all_fills
    # every resting order's row carries its live remainder; fully filled makers are status 2
    for s in range(len(syms)):
        for e in ob.dump(s)[:20]:
            st, rem = con.execute("SELECT status, remaining_quantity FROM orders WHERE order_id=?",
                                  (f"OID-{int(e['seq'])}",)).fetchone()
            assert rem == int(e["qty"]) and st in (0, 1)
    bids, asks = svc.get_order_book("S3", 5)
    obids, oasks = ob.snapshot(3, 5)
    assert np.array_equal(bids, obids) and np.array_equal(asks, oasks)
    # GetOrderBook in the reference's shape: repeated Order {order_id, client_id, price, scale, quantity, side}
    for s in ("S3", "S9"):
        gb, ga = svc.order_book(s)
        d = ob.dump(syms.index(s))
        exp = [{"order_id": f"OID-{int(e['seq'])}", "client_id": "C", "price": int(e["price_q4"]), "scale": 4,
                "quantity": int(e["qty"]), "side": int(e["side"])} for e in d]
        assert gb + ga == exp
    assert svc.order_book("NOPE") == ([], [])
    # StreamMarketData's MarketDataUpdate: the top level of each side
    for s in syms[:4]:
        md = svc.market_data(s)
        ob1, oa1 = ob.snapshot(syms.index(s), 1)
        assert md["has_bid"] == (len(ob1) == 1) and md["has_ask"] == (len(oa1) == 1)
        if len(ob1):
            assert (md["best_bid"], md["bid_size"]) == (int(ob1[0]["price_q4"]), int(ob1[0]["total_qty"]))
        if len(oa1):
            assert (md["best_ask"], md["ask_size"]) == (int(oa1[0]["price_q4"]), int(oa1[0]["total_qty"]))
        assert md["scale"] == 4
    assert svc.market_data("NOPE") == {"symbol": "NOPE", "best_bid": 0, "best_ask": 0, "scale": 4,
                                       "bid_size": 0, "ask_size": 0, "has_bid": False, "has_ask": False}
    svc.close()
    eng.close()


def test_cancel_request_validation(me):
    """CancelOrder (build extension): in-band rejects in SubmitOrder's style; an accepted cancel answers
    with the target's id and consumes NO OID (its stream position repeats the last OID allocated), so
    accepted orders keep the reference's gap-free OID sequence."""
    svc = me.MatchingEngineService(None, ["SYM"])
    assert svc.cancel_order("C", "", "OID-1")["error_message"] == "symbol is required"
    for bad in ("OID-", "OID-0", "OID-x1", "X-3", "OID-3a", ""):
        r = svc.cancel_order("C", "SYM", bad)
        assert r == {"order_id": "", "success": False, "error_message": "order_id is invalid", "grpc_status": 0}
    assert svc.next_oid == 1 and svc.pending == 0
    assert svc.submit_order("C", "SYM", 0, 1, 100, 4, 5)["order_id"] == "OID-1"
    r = svc.cancel_order("C", "SYM", "OID-1")
    assert r == {"order_id": "OID-1", "success": True, "error_message": "", "grpc_status": 0}
    assert svc.next_oid == 2 and svc.pending == 2
    assert svc.submit_order("C", "SYM", 0, 1, 100, 4, 5)["order_id"] == "OID-2"  # no gap
    assert svc.cancel_order("C", "NOSUCH", "OID-2")["success"]  # an unknown symbol takes no book
    assert svc.next_oid == 3 and svc.pending == 4
    assert svc.order_updates() == []  # nothing matched yet


@pytest.mark.gpu
def test_cancels_and_order_update_stream(me, tmp_path):
    """SubmitOrder + CancelOrder slices: results/tapes equal the oracle fed the same records (cancels
    as cancel records), every fill appears as a maker and a taker OrderUpdate, every cancel as one
    CANCELED / REJECTED update, per-client drains partition the stream, and each order's last update
    carries the remaining quantity its DB row holds."""
    from oracle.oracle import OracleBook

    rng = np.random.default_rng(11)
    syms = [f"S{i}" for i in range(8)]
    mids = {s: 1_000_000 + 1000 * i for i, s in enumerate(syms)}
    base = np.array([mids[s] - 64 for s in syms], dtype=np.int64)
    db = str(tmp_path / "cancel.sqlite")
    eng = me.Engine(len(syms), 128, base, max_batch=4096, max_resting=1 << 14)
    svc = me.MatchingEngineService(eng, syms, db_path=db)
    ob = OracleBook(len(syms))
    accepted = []  # (oid, symbol) of LIMIT orders
    owner = {}
    events = []
    for slice_no in range(4):
        seqs, px, qty, sid, kinds = [], [], [], [], []
        nf_expect = 0
        for _ in range(1200):
            if accepted and rng.random() < 0.3:
                oid, s = accepted[int(rng.integers(len(accepted)))]
                if rng.random() < 0.1:
                    s = syms[(syms.index(s) + 1) % len(syms)]  # wrong symbol -> REJECTED
                r = svc.cancel_order(owner[oid], s, f"OID-{oid}")
                assert r["success"] and r["order_id"] == f"OID-{oid}"
                seqs.append(svc.next_oid - 1)
                px.append(oid)
                qty.append(0)
                sid.append(syms.index(s))
                kinds.append(me.kind(me.SIDE_BUY, me.TYPE_LIMIT, 1))
                continue
            s = syms[int(rng.integers(len(syms)))]
            otype = 1 if rng.random() < 0.2 else 0
            side = int(rng.choice([1, 2]))
            q4 = mids[s] + int(rng.integers(-30, 31))
            qn = int(rng.integers(1, 60))
            r = svc.submit_order(f"C{svc.next_oid % 3}", s, otype, side, 0 if otype else q4, 4, qn)
            oid = int(r["order_id"][4:])
            owner[oid] = f"C{oid % 3}"
            if otype == 0:
                accepted.append((oid, s))
            seqs.append(oid)
            px.append(0 if otype else q4)
            qty.append(qn)
            sid.append(syms.index(s))
            kinds.append(me.kind(side, otype))
        seq, res, fills = svc.flush()
        ro, fo = ob.submit(me.Batch(seqs, px, qty, sid, kinds))
        assert np.array_equal(seq, np.array(seqs, dtype=np.uint64))
        assert_results_equal(res, ro, f"slice {slice_no}")
        assert_fills_equal(fills, fo, f"slice {slice_no}")
        # drain per client: the three drains partition the slice's events
        ev = svc.order_updates("C0") + svc.order_updates("C1") + svc.order_updates("C2")
        assert svc.order_updates() == []
        cancels = int(np.sum((np.array(kinds) >> 3) & 1))
        nclose = sum(1 for k, r_ in zip(kinds, ro) if not (k >> 3) & 1 and
                     (r_["status"] in (3, 4) or (r_["fill_count"] == 0 and r_["status"] == 0)))
        assert len(ev) == 2 * len(fo) + cancels + nclose
        assert sum(e["fill_quantity"] for e in ev) == 2 * int(fo["qty"].sum())
        ncanceled = sum(1 for k, r_ in zip(kinds, ro) if (k >> 3) & 1 and r_["status"] == 3)
        assert sum(1 for e in ev if e["status"] == 3 and e["fill_quantity"] == 0
                   and e["remaining_quantity"] > 0) >= ncanceled
        events += ev
    last = {}
    for e in events:
        last[e["order_id"]] = e
    con = sqlite3.connect(db)
    checked = 0
    for oid, e in last.items():
        row = con.execute("SELECT status, remaining_quantity FROM orders WHERE order_id=?", (oid,)).fetchone()
        assert row is not None, oid
        if e["status"] in (0, 1, 2, 3):
            assert row[1] == e["remaining_quantity"], (oid, row, e)
            checked += 1
        if e["status"] == 3:
            assert row[0] == 3
    assert checked > 1000
    for s in syms[:3]:  # the per-order book carries every resting order's own client id
        gb, ga = svc.order_book(s, depth=4)
        for o in gb + ga:
            assert o["client_id"] == owner[int(o["order_id"][4:])]
        d = ob.dump(syms.index(s))
        assert [o["order_id"] for o in gb] == [f"OID-{int(e['seq'])}" for e in
                                               side_levels(d, me.SIDE_BUY, 4)]
    svc.close()
    eng.close()


# ---------------------------------------------------------------- service hardening (round 2)
def _limit_stream(rng, syms, mids, n, market_pct=0.2):
    """(symbol, otype, side, q4 price, qty) requests; every one passes SubmitOrder's validation."""
    out = []
    for _ in range(n):
        s = syms[int(rng.integers(len(syms)))]
        otype = 1 if rng.random() < market_pct else 0
        out.append((s, otype, int(rng.choice([1, 2])), 0 if otype else mids[s] + int(rng.integers(-20, 21)),
                    int(rng.integers(1, 50))))
    return out


def _oracle_batch(me, reqs, oids, sid_of):
    return me.Batch(oids, [r[3] for r in reqs], [r[4] for r in reqs], [sid_of[r[0]] for r in reqs],
                    [me.kind(r[2], r[1]) for r in reqs])


def test_cancel_requires_owner(me):
    """CancelOrder only for the order's own client: another client's cancel is refused
    in-band and consumes no OID."""
    svc = me.MatchingEngineService(None, ["SYM"])
    assert svc.submit_order("alice", "SYM", 0, 1, 100, 4, 5)["order_id"] == "OID-1"
    r = svc.cancel_order("mallory", "SYM", "OID-1")
    assert r == {"order_id": "", "success": False, "error_message": "order belongs to another client",
                 "grpc_status": 0}
    assert svc.next_oid == 2 and svc.pending == 1
    assert svc.cancel_order("alice", "SYM", "OID-1")["success"]
    # an order id nobody holds is queued (the engine answers REJECTED after the flush)
    assert svc.cancel_order("mallory", "SYM", "OID-77")["success"]
    assert svc.pending == 3


def test_unknown_symbols_without_engine(me):
    svc = me.MatchingEngineService(None, ["SYM"])
    for s in ("NEW1", "NEW2", "SYM"):
        assert svc.submit_order("C", s, 0, 1, 100, 4, 5)["success"]
    assert svc.pending == 3


@pytest.mark.gpu
def test_unknown_symbols_interned_matched_and_persisted(me, tmp_path):
    """A never-seen symbol takes the engine's next unused book (its window placed by its first orders)
    and is matched and persisted exactly as the oracle says; past the engine's books SubmitOrder
    answers RESOURCE_EXHAUSTED without an OID."""
    from oracle.oracle import OracleBook

    rng = np.random.default_rng(3)
    syms = ["AAA", "BBB", "CCC", "DDD"]
    mids = {s: 2_000_000 + 50_000 * i for i, s in enumerate(syms)}
    db = str(tmp_path / "intern.sqlite")
    with me.Engine(4, 128, [0, 0, 0, 0], max_batch=4096, max_resting=1 << 14) as eng:
        svc = me.MatchingEngineService(eng, ["AAA"], db_path=db)
        reqs = _limit_stream(rng, syms, mids, 3000)
        oids = []
        for r in reqs:
            resp = svc.submit_order("C", r[0], r[1], r[2], r[3], 4, r[4])
            assert resp["success"], resp
            oids.append(int(resp["order_id"][4:]))
        seq, res, fills = svc.flush()
        sid_of = {"AAA": 0}
        for r in reqs:
            sid_of.setdefault(r[0], len(sid_of))
        ob = OracleBook(4)
        ro, fo = ob.submit(_oracle_batch(me, reqs, oids, sid_of))
        assert_results_equal(res, ro, "interned symbols")
        assert_fills_equal(fills, fo, "interned symbols")
        con = sqlite3.connect(db)
        for s in syms:
            n = con.execute("SELECT COUNT(*) FROM orders WHERE symbol=?", (s,)).fetchone()[0]
            assert n == sum(1 for r in reqs if r[0] == s)
        b0, a0 = svc.get_order_book("DDD", 3)
        ob0, oa0 = ob.snapshot(sid_of["DDD"], 3)
        assert np.array_equal(b0, ob0) and np.array_equal(a0, oa0)
        nxt = svc.next_oid
        r = svc.submit_order("C", "EEE", 0, 1, 100, 4, 1)
        assert r == {"order_id": "", "success": False, "error_message": "symbol capacity exhausted",
                     "grpc_status": 8}
        assert svc.next_oid == nxt
        svc.close()


@pytest.mark.gpu
def test_slices_beyond_max_batch_split(me, tmp_path):
    """More pending orders than the engine's max_batch: the slice closes at max_batch and the flush
    matches every closed slice in order (the service no longer wedges)."""
    from oracle.oracle import OracleBook

    rng = np.random.default_rng(5)
    syms = [f"S{i}" for i in range(8)]
    mids = {s: 1_000_000 + 1000 * i for i, s in enumerate(syms)}
    with me.Engine(8, 128, [mids[s] - 64 for s in syms], max_batch=1000, max_resting=1 << 14) as eng:
        svc = me.MatchingEngineService(eng, syms, db_path=str(tmp_path / "split.sqlite"))
        reqs = _limit_stream(rng, syms, mids, 3500)
        oids = [int(svc.submit_order("C", r[0], r[1], r[2], r[3], 4, r[4])["order_id"][4:]) for r in reqs]
        assert svc.pending == 3500
        seq, res, fills = svc.flush()
        assert svc.pending == 0 and len(seq) == 3500
        ro, fo = OracleBook(8).submit(_oracle_batch(me, reqs, oids, {s: i for i, s in enumerate(syms)}))
        assert_results_equal(res, ro, "split slices")
        assert_fills_equal(fills, fo, "split slices")
        svc.close()


@pytest.mark.gpu
def test_db_failure_keeps_matched_slice_and_retries(me, tmp_path):
    """a failed transaction (another connection holds the write lock past the 5 s busy
    timeout) neither loses nor re-matches the slice: the next flush commits it exactly once."""
    from oracle.oracle import OracleBook

    rng = np.random.default_rng(9)
    syms = ["X", "Y"]
    mids = {"X": 1_000_000, "Y": 1_500_000}
    db = str(tmp_path / "busy.sqlite")
    with me.Engine(2, 128, [mids[s] - 64 for s in syms], max_batch=4096, max_resting=1 << 14) as eng:
        svc = me.MatchingEngineService(eng, syms, db_path=db)
        ob = OracleBook(2)
        sid = {"X": 0, "Y": 1}
        total_fills = 0
        reqs = _limit_stream(rng, syms, mids, 800)
        oids = [int(svc.submit_order("C", *r[:4], 4, r[4])["order_id"][4:]) for r in reqs]
        svc.flush()
        total_fills += len(ob.submit(_oracle_batch(me, reqs, oids, sid))[1])
        # slice 2 while the DB is locked
        locker = sqlite3.connect(db, timeout=0.1)
        locker.execute("BEGIN EXCLUSIVE")
        reqs2 = _limit_stream(rng, syms, mids, 700)
        oids2 = [int(svc.submit_order("C", *r[:4], 4, r[4])["order_id"][4:]) for r in reqs2]
        with pytest.raises(me.ServiceError, match="persistence deferred"):
            svc.flush()
        assert svc.pending == 0 and svc.unpersisted == 700
        ro2, fo2 = ob.submit(_oracle_batch(me, reqs2, oids2, sid))
        total_fills += len(fo2)
        # the engine holds slice 2 (matched once); the book equals the oracle's
        for s in syms:
            gb, ga = svc.get_order_book(s, 5)
            eb, ea = ob.snapshot(sid[s], 5)
            assert np.array_equal(gb, eb) and np.array_equal(ga, ea)
        locker.rollback()
        locker.close()
        # slice 3 flushes after the kept slice 2 commits
        reqs3 = _limit_stream(rng, syms, mids, 300)
        oids3 = [int(svc.submit_order("C", *r[:4], 4, r[4])["order_id"][4:]) for r in reqs3]
        seq, res, fills = svc.flush()
        ro3, fo3 = ob.submit(_oracle_batch(me, reqs3, oids3, sid))
        total_fills += len(fo3)
        assert_results_equal(res, ro3, "after retry")
        assert_fills_equal(fills, fo3, "after retry")
        assert svc.unpersisted == 0
        con = sqlite3.connect(db)
        assert con.execute("SELECT COUNT(*) FROM orders").fetchone()[0] == 1800
        assert con.execute("SELECT COUNT(*) FROM fills").fetchone()[0] == 2 * total_fills
        for s in syms:  # resting rows carry the oracle's live remainders
            for e in ob.dump(sid[s])[:30]:
                rem = con.execute("SELECT remaining_quantity FROM orders WHERE order_id=?",
                                  (f"OID-{int(e['seq'])}",)).fetchone()[0]
                assert rem == int(e["qty"])
        svc.close()


@pytest.mark.gpu
def test_submit_never_waits_for_a_flush(me, tmp_path):
    """SubmitOrder is never blocked by a flush. One thread flushes a 60k-order slice
    (GPU match + a 60k-row SQLite transaction) while this thread keeps submitting; a second thread
    reads books and market data throughout (engine calls are serialized by the service)."""
    import threading
    import time

    from oracle.oracle import OracleBook

    rng = np.random.default_rng(21)
    syms = [f"T{i}" for i in range(64)]
    mids = {s: 3_000_000 + 500 * i for i, s in enumerate(syms)}
    db = str(tmp_path / "concurrent.sqlite")
    with me.Engine(64, 128, [mids[s] - 64 for s in syms], max_batch=65536, max_resting=1 << 18) as eng:
        svc = me.MatchingEngineService(eng, syms, db_path=db)
        reqs = _limit_stream(rng, syms, mids, 60000)
        oids = [int(svc.submit_order("C", *r[:4], 4, r[4])["order_id"][4:]) for r in reqs]
        done = threading.Event()
        span = {}

        def flusher():
            span["t0"] = time.perf_counter()
            svc.flush(outputs=False)
            span["t1"] = time.perf_counter()
            done.set()

        def reader():
            while not done.is_set():
                svc.get_order_book(syms[int(rng.integers(64))], 5)
                svc.market_data(syms[0])

        tf, tr = threading.Thread(target=flusher), threading.Thread(target=reader)
        tf.start()
        tr.start()
        lat, during = [], 0
        reqs2 = _limit_stream(np.random.default_rng(22), syms, mids, 20000)
        oids2 = []
        for r in reqs2:
            a = time.perf_counter()
            oids2.append(int(svc.submit_order("C", *r[:4], 4, r[4])["order_id"][4:]))
            lat.append(time.perf_counter() - a)
            during += not done.is_set()
        tf.join()
        tr.join()
        flush_s = span["t1"] - span["t0"]
        assert during > 1000, "the flush finished before the concurrent submits started"
        assert max(lat) < 0.05 and max(lat) < flush_s / 4, (max(lat), flush_s)
        seq, res, fills = svc.flush()
        ob = OracleBook(64)
        sid = {s: i for i, s in enumerate(syms)}
        ob.submit(_oracle_batch(me, reqs, oids, sid))
        ro, fo = ob.submit(_oracle_batch(me, reqs2, oids2, sid))
        assert_results_equal(res, ro, "after concurrent flush")
        assert_fills_equal(fills, fo, "after concurrent flush")
        con = sqlite3.connect(db)
        assert con.execute("SELECT COUNT(*) FROM orders").fetchone()[0] == 80000
        svc.close()


@pytest.mark.gpu
def test_background_flusher_time_and_size_trigger(me, tmp_path):
    """me_service_start: slices close at 500 records or 2 ms and are matched and persisted with no
    caller; the DB ends up exactly as the oracle's final state says."""
    import time

    from oracle.oracle import OracleBook

    rng = np.random.default_rng(33)
    syms = [f"B{i}" for i in range(16)]
    mids = {s: 4_000_000 + 700 * i for i, s in enumerate(syms)}
    db = str(tmp_path / "bg.sqlite")
    with me.Engine(16, 128, [mids[s] - 64 for s in syms], max_batch=2048, max_resting=1 << 16) as eng:
        svc = me.MatchingEngineService(eng, syms, db_path=db)
        svc.start(interval_us=2000, slice_orders=500)
        reqs = _limit_stream(rng, syms, mids, 6000)
        oids = []
        for k, r in enumerate(reqs):
            oids.append(int(svc.submit_order("C", *r[:4], 4, r[4])["order_id"][4:]))
            if k % 1000 == 999:
                time.sleep(0.01)  # idle gaps: the time trigger closes partial slices
        t0 = time.time()
        while svc.pending and time.time() - t0 < 30:
            time.sleep(0.005)
        assert svc.pending == 0, svc.last_error()
        svc.stop()
        assert svc.last_error() == ""
        ob = OracleBook(16)
        ro, fo = ob.submit(_oracle_batch(me, reqs, oids, {s: i for i, s in enumerate(syms)}))
        con = sqlite3.connect(db)
        assert con.execute("SELECT COUNT(*) FROM orders").fetchone()[0] == 6000
        assert con.execute("SELECT COUNT(*) FROM fills").fetchone()[0] == 2 * len(fo)
        rows = {o: (st, rem) for o, st, rem in
                con.execute("SELECT order_id, status, remaining_quantity FROM orders").fetchall()}
        for k in range(6000):  # a taker that filled completely stays FILLED
            if ro[k]["status"] == me.ST_FILLED:
                assert rows[f"OID-{oids[k]}"] == (me.ST_FILLED, 0)
        for s in range(16):  # every resting order's row carries its live remainder
            for e in ob.dump(s):
                assert rows[f"OID-{int(e['seq'])}"][1] == int(e["qty"])
        ev = svc.order_updates()
        assert sum(e["fill_quantity"] for e in ev) == 2 * int(fo["qty"].sum())
        svc.close()
