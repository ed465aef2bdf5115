"""The FIFO chunk pool at its default size (GPU): liquidity that moves between symbols.

Chunks freed by one symbol's levels stay parked with that symbol (its free list, its fcache row) for fast
reuse; k_seq_sweep's reclamation returns every symbol's free chunks to the shared pool ahead of a launch
group that could otherwise run out (me_kernels.hip chunk_reclaim). Without it the chunks
drawn were the sum of every symbol's peak rather than the peak of the sum, and a stream that the reference
accepts order by order (src/server/matching_engine_service.cpp:66-104) and the oracle runs fine failed the
engine stickily with ERR_CHUNK_OOM. Every test here runs at the default max_chunks (0 = max_resting +
32 S + 64) with max_resting at the stream's own peak, on the three paths that allocate chunks: the
register-window kernel (L = 128), the grouped aggregate path (L = 128, ME_REG_AGG=1) and a deep window's
hot aggregate path, and compares every batch and the final books with the oracle."""
import numpy as np
import pytest

from tests._parity import assert_books_equal, assert_fills_equal, assert_results_equal

pytestmark = pytest.mark.gpu

PATHS = [("reg", 128), ("agg", 128), ("deep", 1024)]


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


@pytest.fixture(scope="module")
def orc(built):
    from oracle import oracle

    return oracle


def _batch(me, rows, seq0):
    """rows: (symbol, side, type, op, price_q4, qty); seqs seq0, seq0 + 1, ..."""
    n = len(rows)
    return me.Batch(np.arange(seq0, seq0 + n, dtype=np.uint64), [r[4] for r in rows], [r[5] for r in rows],
                    [r[0] for r in rows], [me.kind(r[1], r[2], r[3]) for r in rows])


def _limits(b):
    """LIMIT NEW records of a batch (the ones that may rest)."""
    k = b.kind
    return int(np.sum((((k >> 3) & 1) == 0) & (((k >> 2) & 1) == 0)))


def _max_resting(orc, S, batches):
    ob = orc.OracleBook(S)
    need = 0
    for b in batches:
        need = max(need, ob.resting() + _limits(b))
        ob.submit(b)
    ob.close()
    return need


def _run(me, orc, S, L, path, batches, monkeypatch, ctx, max_batch, expect_reclaims=True):
    monkeypatch.setenv("ME_REG_AGG", "1" if path == "agg" else "0")
    R = _max_resting(orc, S, batches)
    ob = orc.OracleBook(S)
    base = [1000] * S
    with me.Engine(S, L, base, max_batch=max_batch, max_resting=R, seq_ring=1 << 22, batches_per_launch=4) as eng:
        assert eng.paths()["grouped_agg"] == (path == "agg")
        cs = eng.chunk_stats()
        assert cs["pool"] == R + 32 * S + 64, cs  # the default size
        for k, b in enumerate(batches):
            r, f = eng.submit_batch(b)
            ro, fo = ob.submit(b)
            assert_results_equal(r, ro, f"{ctx} batch {k}")
            assert_fills_equal(f, fo, f"{ctx} batch {k}")
        assert_books_equal(eng, ob, range(S), ctx)
        assert eng.resting_count() == ob.resting() == eng.admission()["resting"]
        cs = eng.chunk_stats()
        assert cs["high_water"] <= cs["pool"], cs
        if expect_reclaims:
            assert cs["reclaims"] > 0, cs
        return cs


@pytest.mark.parametrize("path,levels", PATHS)
def test_liquidity_migrates_between_symbols(me, orc, monkeypatch, path, levels):
    """The review's stream: symbol s rests R orders at R distinct prices (one chunk each), a MARKET sweeps
    them, then the next symbol does the same — six times over two symbols. Resting orders never exceed R,
    so admission lets every batch in; the chunks drawn over the stream are 6 R against a pool of R + 128."""
    B, Sd, LIM, MKT, NEW = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET, me.OP_NEW
    S = 2
    R = 900 if path == "deep" else 300  # L = 128: 128 window levels + far asks above the window
    batches, seq = [], 1
    for cyc in range(6):
        s = cyc % S
        rows = [(s, Sd, LIM, NEW, 1000 + k, 1 + k % 3) for k in range(R)]
        batches.append(_batch(me, rows, seq))
        seq += len(rows)
        batches.append(_batch(me, [(s, B, MKT, NEW, 0, 10 * R)], seq))
        seq += 1
    _run(me, orc, S, levels, path, batches, monkeypatch, f"migrate {path}", max_batch=1024)


def _fuzz_stream(me, seed, S, nphase, per_phase, n, spread):
    """A randomized stream whose hot symbol moves: in phase p symbol p % S takes ~85 % of the records
    (LIMITs at scattered prices, MARKETs, cancels of its own earlier orders); each phase ends with MARKETs
    on both sides of the symbol that was hot, so its liquidity — and its chunks — go away."""
    rng = np.random.default_rng(seed)
    B, Sd, LIM, MKT, NEW, CAN = me.SIDE_BUY, me.SIDE_SELL, me.TYPE_LIMIT, me.TYPE_MARKET, me.OP_NEW, me.OP_CANCEL
    mid = 1000 + spread
    placed = [[] for _ in range(S)]
    batches, seq = [], 1
    for p in range(nphase):
        hot = p % S
        for _ in range(per_phase):
            rows = []
            for _ in range(n):
                s = hot if rng.random() < 0.85 else int(rng.integers(0, S))
                u = rng.random()
                side = B if rng.random() < 0.5 else Sd
                if u < 0.58:
                    # buys below the mid, sells above it, with some crossing
                    off = int(rng.integers(-spread // 8, spread))
                    px = mid - off if side == B else mid + off
                    rows.append((s, side, LIM, NEW, px, int(rng.integers(1, 20))))
                    placed[s].append(seq + len(rows) - 1)
                elif u < 0.76:
                    rows.append((s, side, MKT, NEW, 0, int(rng.integers(1, 60))))
                else:
                    tgt = placed[s][int(rng.integers(0, len(placed[s])))] if placed[s] else 1
                    rows.append((s, side, LIM, CAN, tgt, 0))
            batches.append(_batch(me, rows, seq))
            seq += len(rows)
        rows = [(hot, B, MKT, NEW, 0, 1 << 30), (hot, Sd, MKT, NEW, 0, 1 << 30)]
        batches.append(_batch(me, rows, seq))
        seq += len(rows)
    return batches


@pytest.mark.parametrize("seed", [3, 17])
@pytest.mark.parametrize("path,levels", PATHS)
def test_fuzz_hot_symbol_migrates(me, orc, monkeypatch, path, levels, seed):
    """Randomized: the hot symbol changes every phase, max_resting is the stream's own peak and the pool
    its default; every batch, the books and the device resting counter equal the oracle's."""
    S = 6
    if path == "deep":
        n, spread = 2048, 400  # the hot symbol's ~1,740 records per batch take the hot aggregate path
    else:
        n, spread = 1024, 56
    batches = _fuzz_stream(me, seed, S, nphase=8, per_phase=3, n=n, spread=spread)
    _run(me, orc, S, levels, path, batches, monkeypatch, f"fuzz {path} seed {seed}", max_batch=n,
         expect_reclaims=False)
