"""Two independent CPU restatements of the matching semantics must agree (no GPU).

The reference has no matcher, so fills are pinned by the build's own golden model
(`oracle/oracle_book.cpp`, an unbounded std::map book). `oracle/pybook.py` restates the semantics a
second time (sorted containers, written from DESIGN.md §2): it must reproduce every committed
fixture (results, tapes, final books) and agree with the C++ oracle on random streams with rejects,
cancels of live / dead / foreign orders and int64-extreme prices.
"""
import numpy as np
import pytest

from tests._parity import load_fixture

@pytest.fixture(scope="module")
def orc(built):
    from oracle import oracle

    return oracle


FIELDS_RES = ("filled_qty", "remaining_qty", "fill_count", "tape_offset", "status", "reason")
FIELDS_FILL = ("taker_seq", "maker_seq", "price_q4", "qty", "symbol")
FIELDS_BOOK = ("seq", "price_q4", "qty", "side")


def same(a, b, fields, ctx):
    assert len(a) == len(b), f"{ctx}: {len(a)} vs {len(b)} entries"
    for f in fields:
        if not np.array_equal(np.asarray(a[f]), np.asarray(b[f])):
            i = int(np.nonzero(np.asarray(a[f]) != np.asarray(b[f]))[0][0])
            raise AssertionError(f"{ctx}: field {f} differs first at {i}: {a[i]} vs {b[i]}")


@pytest.mark.parametrize("cid", [1, 2, 3, 4, 5, 6])
def test_pybook_reproduces_golden_fixture(built, cid):
    from oracle.pybook import PyBook

    meta, batches, res, fills, book = load_fixture(cid)
    pb = PyBook(meta["num_symbols"])
    for k, b in enumerate(batches):
        r, f = pb.submit(b)
        same(r, res[k], FIELDS_RES, f"c{cid} batch {k} results")
        same(f, fills[k], FIELDS_FILL, f"c{cid} batch {k} tape")
    dumps = np.concatenate([pb.dump(s) for s in range(meta["num_symbols"])])
    same(dumps, book, FIELDS_BOOK, f"c{cid} final book")


def random_stream(rng, S, n, seq0):
    from matching_engine_amd import Batch, kind

    seq = np.arange(seq0, seq0 + n, dtype=np.uint64)
    sym = np.where(rng.random(n) < 0.05, S, rng.integers(0, S, n)).astype(np.uint32)  # S: out of range
    side = np.where(rng.random(n) < 0.05, rng.choice([0, 3], n), rng.choice([1, 2], n))
    typ = (rng.random(n) < 0.2).astype(np.int64)
    op = (rng.random(n) < 0.25).astype(np.int64)
    qty = rng.integers(-2, 60, n).astype(np.int32)
    px = (1_000_000 + rng.integers(-12, 13, n)).astype(np.int64)
    ext = rng.random(n) < 0.02
    px[ext] = rng.choice(np.array([np.iinfo(np.int64).max, np.iinfo(np.int64).min, 1, -5], dtype=np.int64), int(ext.sum()))
    # cancel targets: mostly earlier seqs of the stream (live, filled, cancelled or another symbol's)
    earlier = seq0 + np.floor(rng.random(n) * np.arange(n)).astype(np.int64)  # this batch, before it
    tgt = np.where(rng.random(n) < 0.6, earlier, rng.integers(max(1, seq0 - n), seq0 + n, n)).astype(np.int64)
    px = np.where(op == 1, tgt, px)
    kd = np.array([kind(int(a), int(b), int(c)) for a, b, c in zip(side, typ, op)], dtype=np.uint8)
    seq[rng.integers(0, n, 2)] = 0  # records without an OID
    return Batch(seq, px, qty, sym, kd)


@pytest.mark.parametrize("seed", range(6))
def test_pybook_agrees_with_cpp_oracle_random(orc, seed):
    from oracle.pybook import PyBook

    rng = np.random.default_rng(1000 + seed)
    S = 3
    ob, pb = orc.OracleBook(S), PyBook(S)
    seq0 = 1 + (seed % 2) * (1 << 40)
    for k in range(5):
        b = random_stream(rng, S, 600, seq0)
        seq0 += 600
        r1, f1 = ob.submit(b)
        r2, f2 = pb.submit(b)
        same(r2, r1, FIELDS_RES, f"seed {seed} batch {k} results")
        same(f2, f1, FIELDS_FILL, f"seed {seed} batch {k} tape")
        for s in range(S):
            same(pb.dump(s), ob.dump(s), FIELDS_BOOK, f"seed {seed} batch {k} book {s}")
    assert sum(len(pb.dump(s)) for s in range(S)) == ob.resting()
