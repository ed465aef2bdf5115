"""Cancels inside the grouped walk (GPU): k_agg_gwalk_cx + k_agg_gres's cancel paths (me_agg.hip).

A cancel of order X at level l removes X's remaining quantity at that moment. The walk computes it from
level totals and fixed maker positions (what the takes consumed, where X starts once the group's earlier
cancels ahead of it are taken out) instead of handing the symbol to k_match_reg's continuation; the resolve
shortens each cancelled maker to its consumed part, and unlinks chunks a cancel of an older order left without
live orders (head, middle, tail). Semantics: CANCELED with the quantity removed, or REJECTED / UNKNOWN_ORDER
when the target is not a live resting order of the symbol (oracle/oracle_book.cpp submit_core, the CANCELED
status of /root/reference/proto/matching_engine.proto:83). Every batch, the books and the resting counters
must equal the oracle's."""
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


@pytest.fixture
def cx_env(monkeypatch):
    monkeypatch.setenv("ME_REG_AGG", "1")
    monkeypatch.setenv("ME_GW_CANCEL", "1")


def _rows(me, rows, seq0):
    """rows: (symbol, side, type, op, price_q4 / cancel target, qty)"""
    n = len(rows)
    return me.Batch(np.arange(seq0, seq0 + n, dtype=np.uint64), [r[4] for r in rows], [r[5] for r in rows],
                    [r[0] for r in rows], [me.kind(r[1], r[2], r[3]) for r in rows])


def _sync(eng, ob, batches, ctx, symbols):
    for k, b in enumerate(batches):
        r, f = eng.submit_batch(b)
        ro, fo = ob.submit(b)
        assert_results_equal(r, ro, f"{ctx} batch {k}")
        assert_fills_equal(f, fo, f"{ctx} batch {k}")
    assert_books_equal(eng, ob, symbols, ctx)
    assert eng.resting_count() == ob.resting() == eng.admission()["resting"], ctx


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
    for k, b in enumerate(batches):
        ro, fo = ob.submit(b)
        assert_results_equal(outs[k][0], ro, f"{ctx} batch {k}")
        assert_fills_equal(outs[k][1], fo, f"{ctx} batch {k}")
    assert_books_equal(eng, ob, range(eng.num_symbols), ctx)
    assert eng.resting_count() == ob.resting() == eng.admission()["resting"], ctx


@pytest.mark.parametrize("group,lag", [(1, 2), (8, 17), (32, 65)])
def test_cx_config5_stream_every_batch(me, orc, cx_env, group, lag):
    """Config 5's mix (60 % cancels, sweeping MARKETs) on 128 symbols (64 records per symbol and batch, as at
    config 5's shape): every batch of full and partial groups against the oracle, through the walk that covers
    cancels; hand-offs stay rare."""
    sc = me.preset(5, num_symbols=128, levels=128, batch=8192)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(48)]
    total = sum(len(b) for b in batches)
    ob = orc.OracleBook(sc.num_symbols)
    with me.Engine(sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=total + 1024, seq_ring=1 << 22,
                   batches_per_launch=group) as eng:
        p = eng.paths()
        assert p["grouped_agg"] and p["grouped_cancels"], p
        _check(eng, ob, batches, _pipelined(eng, batches, lag), f"cx config5 G={group}")
        launches = -(-len(batches) // group)
        assert eng.stats()["handoffs"] * 16 <= launches * sc.num_symbols, eng.stats()


def test_cx_targets_in_the_group(me, orc, cx_env):
    """One batch (one group): rests cancelled in the same block, a rest partially filled and then cancelled,
    a second cancel of the same order, cancels of a MARKET's seq, of a later seq, of another symbol's order and
    of a filled order, cancels that empty the best bid / ask (the next best level must be found), takes after
    cancels (they skip the cancelled quantity)."""
    B, S_, L, M, N, X = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET, me.OP_NEW, me.OP_CANCEL
    seq0 = 100
    rows = [
        (0, S_, L, N, 1010, 5),  # 100 best ask
        (0, S_, L, N, 1010, 7),  # 101
        (0, S_, L, N, 1012, 4),  # 102
        (0, B, L, N, 1005, 6),   # 103 best bid
        (0, B, L, N, 1003, 9),   # 104
        (1, S_, L, N, 1010, 3),  # 105 another symbol
        (0, B, L, X, 101, 0),    # 106 cancel 101 (untouched): 7
        (0, B, M, N, 0, 3),      # 107 MARKET takes 3 of 100
        (0, B, L, X, 100, 0),    # 108 cancel 100 (3 consumed): 2
        (0, B, L, X, 100, 0),    # 109 again: unknown
        (0, B, L, X, 107, 0),    # 110 a MARKET's seq: unknown
        (0, B, L, X, 115, 0),    # 111 a later seq: unknown
        (0, B, L, X, 105, 0),    # 112 symbol 1's order: unknown
        (0, B, L, N, 1012, 4),   # 113 takes all of 102 (level 1010 is empty now)
        (0, B, L, X, 102, 0),    # 114 filled: unknown
        (0, S_, L, X, 103, 0),   # 115 cancel the best bid 103 -> best bid 1003
        (0, S_, M, N, 0, 4),     # 116 takes 4 of 104
        (0, B, L, N, 1001, 2),   # 117
        (0, S_, L, N, 1020, 8),  # 118
        (0, S_, L, X, 104, 0),   # 119 cancel 104 (4 consumed): 5
        (0, B, L, X, 118, 0),    # 120 cancel the only ask: the ask side empties
        (0, S_, M, N, 0, 10),    # 121 takes 117's 2
        (1, B, L, X, 105, 0),    # 122 symbol 1 cancels its own: 3
    ]
    ob = orc.OracleBook(2)
    with me.Engine(2, 128, [1000, 1000], max_batch=64, max_resting=256, seq_ring=1 << 22) as eng:
        assert eng.paths()["grouped_cancels"]
        _sync(eng, ob, [_rows(me, rows, seq0)], "in-group", [0, 1])
        assert eng.stats()["handoffs"] == 0


@pytest.mark.parametrize("variant", range(4))
def test_cx_targets_before_the_group(me, orc, cx_env, variant):
    """Orders from earlier groups: 48 asks at one level (three chunks), then a group that takes from the
    head, cancels orders in the head, middle and tail chunks (whole chunks, so they must leave the FIFO),
    cancels a filled order and one twice, rests behind the old tail and takes again across the cancelled
    quantities; then a full sweep. Variants order the cancels differently and add rests."""
    B, S_, L, M, N, X = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET, me.OP_NEW, me.OP_CANCEL
    C = me._abi.CHUNK_SLOTS
    rng = np.random.default_rng(variant)
    ob = orc.OracleBook(1)
    seq = 1
    with me.Engine(1, 128, [1000], max_batch=256, max_resting=1024, seq_ring=1 << 22) as eng:
        batches = []
        adds = [(0, S_, L, N, 1010, int(q)) for q in rng.integers(1, 6, 3 * C)]
        batches.append(_rows(me, adds, seq))
        first = seq
        seq += len(adds)
        mid = [first + C + k for k in range(C)]  # the whole middle chunk
        tail = [first + 2 * C + k for k in range(C)]  # the whole tail chunk
        head_some = [first + 3, first + 5]
        order = mid + tail + head_some
        if variant % 2:
            order = order[::-1]
        if variant >= 2:
            rng.shuffle(order)
        g = [(0, B, M, N, 0, 4)]  # takes from the head
        g += [(0, B, L, X, t, 0) for t in order[: len(order) // 2]]
        g += [(0, B, L, X, first, 0)]  # the head order: filled (or partly) by the MARKET above
        g += [(0, S_, L, N, 1010, 3), (0, S_, L, N, 1010, 2)]  # rests behind the old tail
        g += [(0, B, L, X, t, 0) for t in order[len(order) // 2:]]
        g += [(0, B, L, X, order[0], 0)]  # twice
        g += [(0, B, M, N, 0, 9)]  # takes across the cancelled orders
        if variant >= 2:
            g += [(0, S_, L, N, 1011, 5), (0, B, L, X, seq + len(g), 0)]  # a rest cancelled in the same group
        batches.append(_rows(me, g, seq))
        seq += len(g)
        batches.append(_rows(me, [(0, B, M, N, 0, 1000)], seq))
        _sync(eng, ob, batches, f"pre-group variant {variant}", [0])
        assert eng.resting_count() == 0


def test_cx_tight_pool_chunks_unlinked(me, orc, cx_env):
    """The chunk-unlinking test of the register kernel on the walk with cancels: a level that never empties,
    chunk after chunk filled and then cancelled by later groups; a 4-chunk pool must suffice for 30 rounds."""
    B, S_, L, M = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET
    C = me._abi.CHUNK_SLOTS
    ob = orc.OracleBook(1)
    seq = 1
    with me.Engine(1, 128, [1000], max_batch=4 * C, max_resting=4 * C, max_chunks=4, seq_ring=1 << 22) as eng:
        _sync(eng, ob, [_rows(me, [(0, B, L, 0, 1050, 7)], seq)], "anchor", [0])
        seq += 1
        for rnd in range(30):
            adds = [(0, B, L, 0, 1050, 1 + k) for k in range(2 * C)]
            b = _rows(me, adds, seq)
            first = seq
            seq += len(adds)
            order = list(range(C // 2, C + C // 2)) + list(range(C + C // 2, 2 * C)) + list(range(C // 2))
            if rnd % 3 == 2:
                order = order[::-1]
            cancels = _rows(me, [(0, B, L, 1, first + k, 0) for k in order], seq)
            seq += len(order)
            _sync(eng, ob, [b, cancels], f"round {rnd}", [0])
        _sync(eng, ob, [_rows(me, [(0, S_, M, 0, 0, 5)], seq)], "final sweep", [0])
        assert eng.stats()["handoffs"] == 0


def test_cx_level_list_overflow_hands_off(me, orc, cx_env):
    """A level with more cancels in one group than the walk lists (GW_CXL = 20): cancels the bounds decide
    (nothing consumed up to the order, or all of it) still run in the walk; one that needs the exact start of
    a partly consumed order hands the symbol's rest of the group to the continuation. Every result is the
    oracle's."""
    B, S_, L, M, X = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET, me.OP_CANCEL
    ob = orc.OracleBook(1)
    rows = [(0, S_, L, 0, 1010, 2) for _ in range(40)]  # seqs 1..40, two lots each
    rows += [(0, B, L, X, k, 0) for k in range(18, 41)]  # 23 cancels behind the front: bounds suffice
    rows += [(0, B, M, 0, 0, 5)]  # takes #1, #2 and one lot of #3
    rows += [(0, B, L, X, 3, 0)]  # partly consumed, 23 cancels at the level: the continuation
    rows += [(0, S_, L, 0, 1011, 1), (0, B, L, X, 5, 0), (0, B, L, X, 5, 0), (0, B, M, 0, 0, 100)]
    with me.Engine(1, 128, [1000], max_batch=128, max_resting=256, seq_ring=1 << 22) as eng:
        _sync(eng, ob, [_rows(me, rows, 1)], "list overflow", [0])
        assert eng.stats()["handoffs"] == 1


@pytest.mark.parametrize("seed", range(int(os.environ.get("ME_FUZZ_SEEDS", "0")) or 12))
def test_cx_fuzz(me, orc, cx_env, seed):
    """Randomized shapes with cancels (10-60 %), sweeping MARKETs, a few far LIMITs and drifting mids (which
    still hand off), unknown symbols, device groups / host pipeline / synchronous batches."""
    rng = np.random.default_rng(9000 + seed)
    levels = int(rng.choice([64, 128]))
    S = int(rng.choice([1, 5, 64, 200]))
    batch = int(rng.choice([2048, 8192]))
    group = int(rng.choice([1, 4, 16, 32]))
    nb = int(rng.integers(6, 24))
    over = dict(num_symbols=S, levels=levels, batch=batch, cancel_pct=int(rng.choice([10, 40, 60])),
                market_pct=int(rng.choice([5, 20])), market_qty_mult=int(rng.choice([0, 3, 20])),
                far_pct=int(rng.choice([0, 0, 1])), drift_step=int(rng.choice([0, 0, 1])),
                drift_every=int(rng.choice([1, 3])), seq_start=int(rng.choice([1, (1 << 40) + 3])),
                zipf_s=float(rng.choice([0.0, 1.1])), spread_ticks=min(32, levels // 2 - 1))
    if over["drift_step"] == 0:
        over["drift_every"] = 0
    sc = me.preset(5, **over)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(batch) for _ in range(nb)]
    if rng.random() < 0.3:
        for b in batches:
            b.symbol[:: max(1, len(b) // 5)] = S + 7
    path = str(rng.choice(["device", "host", "sync"]))
    total = sum(len(b) for b in batches)
    ctx = f"cx seed {seed}: L={levels} S={S} batch={batch} G={group} path={path} {over}"
    ob = orc.OracleBook(S)
    with me.Engine(S, levels, base, max_batch=batch, max_resting=total + 1024, seq_ring=1 << 20,
                   batches_per_launch=group) as eng:
        assert eng.paths()["grouped_cancels"], ctx
        outs = [None] * nb
        if path == "device":
            for g0 in range(0, nb, group):
                grp = batches[g0:g0 + group]
                dbs = [eng.upload(b) for b in grp]
                for db in dbs:
                    eng.submit_device(db)
                eng.sync()
                for k in range(len(grp)):
                    outs[g0 + k] = eng.fetch_group_outputs(k, len(grp[k]))
                for db in dbs:
                    db.free()
        elif path == "host":
            outs = _pipelined(eng, batches, int(rng.integers(1, 2 * group + 2)))
        else:
            outs = [eng.submit_batch(b) for b in batches]
        _check(eng, ob, batches, outs, ctx)
