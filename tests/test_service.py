"""SubmitOrder drop-in (include/me_service.h): responses, OID sequence/reseed and persisted rows
against the reference contract (tests/golden/submit_contract.json), and the matched outcome of
requests flowing through SubmitOrder against the oracle."""
import json
import os
import sqlite3

import numpy as np
import pytest

from tests._parity import assert_fills_equal, assert_results_equal

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
    """CancelOrder (build extension): in-band rejects in SubmitOrder's style, no OID consumed on a
    reject; an accepted cancel answers with the target's id and takes the next stream position."""
    svc = me.MatchingEngineService(None, ["SYM"])
    assert svc.cancel_order("C", "", "OID-1")["error_message"] == "symbol is required"
    for bad in ("OID-", "OID-0", "OID-x1", "X-3", "OID-3a", ""):
        r = svc.cancel_order("C", "SYM", bad)
        assert r == {"order_id": "", "success": False, "error_message": "order_id is invalid", "grpc_status": 0}
    assert svc.next_oid == 1 and svc.pending == 0
    assert svc.submit_order("C", "SYM", 0, 1, 100, 4, 5)["order_id"] == "OID-1"
    r = svc.cancel_order("C", "SYM", "OID-1")
    assert r == {"order_id": "OID-1", "success": True, "error_message": "", "grpc_status": 0}
    assert svc.next_oid == 3 and svc.pending == 2
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
    events = []
    for slice_no in range(4):
        seqs, px, qty, sid, kinds = [], [], [], [], []
        nf_expect = 0
        for _ in range(1200):
            if accepted and rng.random() < 0.3:
                oid, s = accepted[int(rng.integers(len(accepted)))]
                if rng.random() < 0.1:
                    s = syms[(syms.index(s) + 1) % len(syms)]  # wrong symbol -> REJECTED
                r = svc.cancel_order(f"C{oid % 3}", s, f"OID-{oid}")
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
    svc.close()
    eng.close()
