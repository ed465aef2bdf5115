"""Randomised engine configurations against the oracle (GPU): window size (register kernel at 64 /
128 levels, deep-window kernel at 256 / 1,024 / 4,096), group size, symbols, batch size, the
stream's mix (cancels, sweeping MARKETs, far LIMITs, drifting mids, Zipf symbols, unknown symbols)
and the submission path (device groups, host pipeline with a collect lag, synchronous batches) are
drawn per case from a seeded generator; every batch's results and tape and the final books must
equal the oracle's. Cheap cases, many shapes: the kind of test that found the group-count bug."""
import os

import numpy as np
import pytest

from tests._parity import assert_books_equal, assert_fills_equal, assert_results_equal

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def me(built):
    import matching_engine_amd

    return matching_engine_amd


def _case(me, seed, agg=False):
    rng = np.random.default_rng((5000 if agg else 1000) + seed)
    if agg:  # the grouped aggregate path's shapes: register windows, batches of >= 8,192 records
        levels = int(rng.choice([64, 128]))
        S = int(rng.choice([1, 17, 64, 256]))
        batch = int(rng.choice([8192, 16384]))
        group = int(rng.choice([1, 4, 16, 32]))
        nb = int(rng.integers(4, 24))
    else:
        levels = int(rng.choice([64, 128, 128, 256, 1024, 4096]))
        S = int(rng.choice([1, 3, 17, 64, 300]))
        batch = int(rng.choice([64, 500, 2048, 6000]))
        group = int(rng.choice([1, 2, 7, 16, 32]))
        nb = int(rng.integers(6, 40))
    cancel = int(rng.choice([0, 10, 40]))
    market = int(rng.choice([5, 20]))
    over = dict(num_symbols=S, levels=levels, batch=batch, cancel_pct=cancel, market_pct=market,
                market_qty_mult=int(rng.choice([0, 3, 20])), far_pct=int(rng.choice([0, 1, 5])),
                drift_step=int(rng.choice([0, 1, 4])), drift_every=int(rng.choice([1, 3, 9])),
                seq_start=int(rng.choice([1, (1 << 40) + 3])), zipf_s=float(rng.choice([0.0, 1.1])))
    if over["drift_step"] == 0:
        over["drift_every"] = 0
    spread = min(32, levels // 2 - 1)
    sc = me.preset(5, spread_ticks=spread, **over)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(batch) for _ in range(nb)]
    if rng.random() < 0.3:  # a few unknown symbol ids
        for b in batches:
            b.symbol[:: max(1, len(b) // 5)] = S + 7
    path = str(rng.choice(["device", "host", "sync"]))
    lag = int(rng.integers(1, 3 * group + 2))
    return sc, base, batches, group, path, lag


# ME_FUZZ_SEEDS=N widens both draws to N seeds for soak runs (profiles/r4/soak); the suite's default stays cheap
_SEEDS = int(os.environ.get("ME_FUZZ_SEEDS", "0"))


@pytest.mark.parametrize("seed", range(_SEEDS or 24))
def test_fuzz_case(me, seed):
    _run_case(me, seed, False)


@pytest.mark.parametrize("seed", range(_SEEDS or 10))
def test_fuzz_agg_case(me, seed, monkeypatch):
    """ME_REG_AGG=1: every launch group through k_agg_gwalk (cancels, far prices and overfull buckets hand
    symbols to k_match_reg's continuation mid-group), chunk pool max_resting + 2S."""
    monkeypatch.setenv("ME_REG_AGG", "1")
    _run_case(me, seed, True)


def test_fuzz_agg_seed55_default_far_levels(me, monkeypatch):
    """The soak draw that once failed the engine (profiles/r4/soak/fuzz80.log: agg seed 55, one symbol,
    180k records, 5 % far LIMITs up to 64 windows out): more distinct far levels per side than the inline
    region holds. At the DEFAULT far_levels the sides move into the far arena and every batch, the
    final book and the resting counts equal the oracle's (no sticky failure)."""
    monkeypatch.setenv("ME_REG_AGG", "1")
    st = _run_case(me, 55, True)
    assert st["moves"] > 0, st


def _run_case(me, seed, agg):
    from oracle.oracle import OracleBook

    sc, base, batches, group, path, lag = _case(me, seed, agg)
    total = sum(len(b) for b in batches)
    ctx = (f"{'agg ' if agg else ''}seed {seed}: L={sc.levels} S={sc.num_symbols} batch={sc.batch} G={group} path={path} "
           f"lag={lag} cancel={sc.cancel_pct} far={sc.far_pct} drift={sc.drift_step}/{sc.drift_every}")
    ob = OracleBook(sc.num_symbols)
    with me.Engine(sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=total + 1024,
                   max_chunks=total + 1024 + 2 * sc.num_symbols, seq_ring=1 << 20, batches_per_launch=group) as eng:
        if agg:
            assert eng.paths()["grouped_agg"], ctx
        outs = [None] * len(batches)
        if path == "device":
            group = eng.config()["batches_per_launch"]  # deep windows: one batch per launch
            for g0 in range(0, len(batches), group):
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
            lag = min(lag, eng.config()["host_slots"] - 1)  # deep windows run one batch per launch
            pend = []
            for k, b in enumerate(batches):
                pend.append((k, eng.submit_host(b)))
                while len(pend) > lag:
                    j, t = pend.pop(0)
                    outs[j] = eng.collect(t)
            for j, t in pend:
                outs[j] = eng.collect(t)
        else:
            outs = [eng.submit_batch(b) for b in batches]
        for k, b in enumerate(batches):
            ro, fo = ob.submit(b)
            assert_results_equal(outs[k][0], ro, f"{ctx} batch {k}")
            assert_fills_equal(outs[k][1], fo, f"{ctx} batch {k}")
        assert_books_equal(eng, ob, range(sc.num_symbols), ctx)
        assert eng.resting_count() == ob.resting() == eng.admission()["resting"], ctx
        return eng.far_stats()
