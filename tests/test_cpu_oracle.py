"""CPU tests: the oracle against the committed golden vectors, the SubmitOrder contract, and the
hand-written matching semantics of DESIGN.md §2. No GPU needed."""
import json
import os

import numpy as np
import pytest

from tests._parity import assert_fills_equal, assert_results_equal, load_fixture

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


@pytest.fixture(scope="module")
def orc(built):
    from oracle import oracle

    return oracle


# ---------------------------------------------------------------- price normalization
def test_reference_test_price_kats(me):
    # tests/test_price.cpp:8-13 and :17-19 (FromRaw(10050, 8) -> price_q4 1)
    assert me.normalize_to_q4(10050, 9) == 0
    assert me.normalize_to_q4(10050, 8) == 1
    assert me.normalize_to_q4(10050, 7) == 10
    assert me.normalize_to_q4(10050, 6) == 100
    assert me.normalize_to_q4(10050, 2) == 1005000
    assert me.normalize_to_q4(10050, 0) == 100500000


def test_price_golden_vectors_product(me):
    cases = json.load(open(os.path.join(GOLD, "price_q4.json")))["cases"]
    assert len(cases) > 200
    for c in cases:
        if c["exception"] is None:
            assert me.normalize_to_q4(c["price"], c["scale"]) == c["q4"], c
        else:
            typ, what = c["exception"]
            exc = ValueError if typ == "invalid_argument" else OverflowError
            with pytest.raises(exc, match=what):
                me.normalize_to_q4(c["price"], c["scale"])


def test_price_golden_vectors_regenerate_from_reference(orc):
    """Re-run the reference's own normalize_to_q4 (oracle/_ref) and compare with the fixture."""
    if not os.path.exists("/root/reference/include/domain/price.hpp"):
        pytest.skip("reference tree absent (GPU box): fixture is the pin")
    cases = json.load(open(os.path.join(GOLD, "price_q4.json")))["cases"]
    outs = orc.ref_normalize_many([(c["price"], c["scale"]) for c in cases])
    for c, o in zip(cases, outs):
        if c["exception"] is None:
            assert o == c["q4"]
        else:
            assert o[1:] == tuple(c["exception"])


# ---------------------------------------------------------------- SubmitOrder contract
def test_submit_contract_oracle(orc):
    cases = json.load(open(os.path.join(GOLD, "submit_contract.json")))["cases"]
    svc = orc.OracleService(next_id=1)
    for c in cases:
        r = c["request"]
        got = svc.submit(r["symbol"], r["order_type"], r["side"], r["price"], r["scale"], r["quantity"])
        assert got == c["expect"], (c["cite"], got, c["expect"])


def test_submit_contract_oid_sequence(orc):
    cases = json.load(open(os.path.join(GOLD, "submit_contract.json")))["cases"]
    # OIDs are allocated exactly by the requests that pass validation (incl. the ones that throw)
    alloc = [c for c in cases if c["expect"]["order_id"] or c["expect"]["grpc_status"]]
    ids = [int(c["expect"]["order_id"][4:]) for c in alloc if c["expect"]["order_id"]]
    assert ids == sorted(ids) and ids[0] == 1
    assert ids[-1] == len(alloc)  # gaps come only from throwing requests


# ---------------------------------------------------------------- oracle matching fixtures
@pytest.mark.parametrize("cid", [1, 2, 3, 4, 5, 6])
def test_oracle_replays_golden_fixture(orc, cid):
    meta, batches, res, fills, book = load_fixture(cid)
    ob = orc.OracleBook(meta["num_symbols"])
    for k, b in enumerate(batches):
        r, f = ob.submit(b)
        assert_results_equal(r, res[k], f"c{cid} b{k}")
        assert_fills_equal(f, fills[k], f"c{cid} b{k}")
    dumps = np.concatenate([ob.dump(s) for s in range(meta["num_symbols"])])
    assert np.array_equal(dumps, book)


def test_fixture_streams_are_deterministic(me):
    from tests.golden.make_golden import fixture_stream

    for cid in (2, 5):
        _, _, b1 = fixture_stream(cid)
        _, _, b2 = fixture_stream(cid)
        for x, y in zip(b1, b2):
            assert np.array_equal(x.seq, y.seq) and np.array_equal(x.price_q4, y.price_q4)
            assert np.array_equal(x.kind, y.kind) and np.array_equal(x.symbol, y.symbol)


# ---------------------------------------------------------------- semantics
def _batch(me, rows, start_seq=1):
    """rows: (symbol, side, type, op, price_or_target, qty)."""
    n = len(rows)
    seq = np.arange(start_seq, start_seq + n, dtype=np.uint64)
    return me.Batch(seq, [r[4] for r in rows], [r[5] for r in rows], [r[0] for r in rows],
                    [me.kind(r[1], r[2], r[3]) for r in rows])


def test_semantics_price_time_priority(me, orc):
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    ob = orc.OracleBook(1)
    rows = [
        (0, S, L, 0, 1010, 5),   # 1 ask 1010
        (0, S, L, 0, 1005, 3),   # 2 ask 1005 (better)
        (0, S, L, 0, 1005, 4),   # 3 ask 1005 (later)
        (0, B, L, 0, 1007, 6),   # 4 crosses 1005: 3 from #2 then 3 from #3 -> FILLED
        (0, B, M, 0, 0, 10),     # 5 market: 1 from #3 @1005, 5 from #1 @1010, rest discarded
        (0, B, L, 0, 999, 2),    # 6 rests as bid
        (0, S, L, 0, 990, 5),    # 7 sells into bid 999 (2), rests 3 @990
    ]
    r, f = ob.submit(_batch(me, rows))
    assert list(r["status"]) == [me.ST_NEW, me.ST_NEW, me.ST_NEW, me.ST_FILLED, me.ST_CANCELED, me.ST_NEW,
                                 me.ST_PARTIALLY_FILLED]
    got = [(int(x["taker_seq"]), int(x["maker_seq"]), int(x["price_q4"]), int(x["qty"])) for x in f]
    assert got == [(4, 2, 1005, 3), (4, 3, 1005, 3), (5, 3, 1005, 1), (5, 1, 1010, 5), (7, 6, 999, 2)]
    assert r["filled_qty"][4] == 6 and r["remaining_qty"][4] == 4
    assert list(r["fill_count"]) == [0, 0, 0, 2, 2, 0, 1]
    assert list(r["tape_offset"]) == [0, 0, 0, 0, 2, 4, 4]
    d = ob.dump(0)
    assert [(int(x["seq"]), int(x["price_q4"]), int(x["qty"]), int(x["side"])) for x in d] == [(7, 990, 3, S)]


def test_semantics_rejects_and_cancel(me, orc):
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    ob = orc.OracleBook(2)
    rows = [
        (0, B, L, 0, 1000, 5),        # 1 rests
        (0, B, L, 0, 999, 5),         # 2 rests (any price: the book is unbounded)
        (0, B, L, 0, 1128, 5),        # 3 rests, best bid
        (1, 0, L, 0, 5001, 5),        # 4 side 0 -> REJECTED bad side
        (0, B, L, 0, 1001, 0),        # 5 qty 0 -> REJECTED bad qty
        (7, B, L, 0, 1001, 1),        # 6 symbol out of range -> REJECTED bad symbol
        (1, S, L, 1, 1, 0),           # 7 cancel #1 from the wrong symbol -> REJECTED unknown
        (0, S, L, 1, 1, 0),           # 8 cancel #1 -> CANCELED, remaining 5
        (0, S, L, 1, 1, 0),           # 9 cancel again -> REJECTED unknown
        (0, S, L, 1, 12, 0),          # 10 cancel a future seq -> REJECTED
        (0, S, M, 0, 0, 3),           # 11 market sell: 3 from #3 @1128 -> FILLED
    ]
    r, f = ob.submit(_batch(me, rows))
    assert [(int(x["taker_seq"]), int(x["maker_seq"]), int(x["price_q4"]), int(x["qty"])) for x in f] == [
        (11, 3, 1128, 3)]
    st = [(int(x["status"]), int(x["reason"]), int(x["remaining_qty"])) for x in r]
    assert st == [
        (me.ST_NEW, 0, 5), (me.ST_NEW, 0, 5), (me.ST_NEW, 0, 5),
        (me.ST_REJECTED, me.RJ_BAD_SIDE, 5), (me.ST_REJECTED, me.RJ_BAD_QTY, 0),
        (me.ST_REJECTED, me.RJ_BAD_SYMBOL, 0), (me.ST_REJECTED, me.RJ_UNKNOWN_ORDER, 0),
        (me.ST_CANCELED, 0, 5), (me.ST_REJECTED, me.RJ_UNKNOWN_ORDER, 0), (me.ST_REJECTED, me.RJ_UNKNOWN_ORDER, 0),
        (me.ST_FILLED, 0, 0)]
    assert ob.resting() == 2
    # no OID is 0 (the reference's counter starts at 1); every other u64 seq is accepted
    r, _ = ob.submit(_batch(me, [(0, B, L, 0, 1000, 1)], start_seq=0))
    assert (r["status"][0], r["reason"][0]) == (me.ST_REJECTED, me.RJ_BAD_SEQ)


def test_semantics_unbounded_prices_and_seqs(me, orc):
    """The reference accepts any LIMIT with a positive raw price at any int64 Q4
    (matching_engine_service.cpp:78-83, price.hpp:15-29) and OIDs are an unbounded u64 (:29-32):
    no admission rule beyond the domain's, prices sort as int64, cancels find seqs above 2^33."""
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    I64 = (1 << 63) - 1
    ob = orc.OracleBook(1)
    start = (1 << 33) + 17
    rows = [
        (0, S, L, 0, I64, 2),          # ask at the top of the int64 range
        (0, S, L, 0, 10 ** 15, 3),     # ask far below it
        (0, B, L, 0, -(1 << 62), 4),   # bid deep in the negative range
        (0, B, L, 0, 5, 1),            # best bid
        (0, B, M, 0, 0, 4),            # market buy: 3 @1e15 then 1 @I64
        (0, S, L, 0, -(1 << 63), 6),   # sell at INT64_MIN: crosses both bids (1 @5, 4 @-2^62), rests 1
        (0, S, L, 1, start + 2, 0),    # cancel the -2^62 bid: already filled -> REJECTED
        (0, S, L, 1, start, 0),        # cancel the I64 ask: 1 left -> CANCELED 1
    ]
    r, f = ob.submit(_batch(me, rows, start_seq=start))
    got = [(int(x["taker_seq"]) - start, int(x["maker_seq"]) - start, int(x["price_q4"]), int(x["qty"])) for x in f]
    assert got == [(4, 1, 10 ** 15, 3), (4, 0, I64, 1), (5, 3, 5, 1), (5, 2, -(1 << 62), 4)]
    assert [int(x) for x in r["status"]] == [me.ST_NEW, me.ST_NEW, me.ST_NEW, me.ST_NEW, me.ST_FILLED,
                                             me.ST_PARTIALLY_FILLED, me.ST_REJECTED, me.ST_CANCELED]
    assert int(r["remaining_qty"][7]) == 1
    d = ob.dump(0)
    assert [(int(x["seq"]) - start, int(x["price_q4"]), int(x["qty"]), int(x["side"])) for x in d] == [
        (5, -(1 << 63), 1, S)]


def test_semantics_cancel_frees_level_and_best_moves(me, orc):
    B, S, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    ob = orc.OracleBook(1)
    rows = [(0, S, L, 0, 1010, 5), (0, S, L, 0, 1020, 5), (0, S, L, 1, 1, 0), (0, B, L, 0, 1015, 9)]
    r, f = ob.submit(_batch(me, rows))
    assert len(f) == 0 and r["status"][3] == me.ST_NEW  # 1010 cancelled: best ask is now 1020 > 1015
    r, f = ob.submit(_batch(me, [(0, B, L, 0, 1020, 7)], start_seq=5))
    assert [(int(x["maker_seq"]), int(x["qty"]), int(x["price_q4"])) for x in f] == [(2, 5, 1020)]
    assert r["status"][0] == me.ST_PARTIALLY_FILLED and r["remaining_qty"][0] == 2
