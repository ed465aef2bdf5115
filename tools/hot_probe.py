"""Diagnostic: the aggregate hot walk's cycles by part (k_agg_walk, configs 1 and 4) from the -DME_STAMPS
build's s_memtime stamps (never the product): set-up (ladder load / list rebuild), block set-up, record loop
and end, per record walked, for the busiest symbols.

    ME_ENGINE_LIB=matching_engine_amd/build/libme_engine_stamps.so python tools/hot_probe.py --config 4
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import matching_engine_amd as me  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=4)
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--skip", type=int, default=2)
    ap.add_argument("--seed-top", type=int, default=1000)
    ap.add_argument("--per-side", type=int, default=10_000)
    ap.add_argument("--top", type=int, default=4)
    a = ap.parse_args()
    assert "stamps" in me._abi.LIB_PATH, "set ME_ENGINE_LIB to the stamps build"
    sc = me.preset(a.config)
    st = me.Stream(sc)
    base = st.base_prices()
    lib = me._abi.load()
    lib.me_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    seeds = st.seed_books(range(a.seed_top), a.per_side) if (a.config == 4 and a.seed_top) else None
    nseed = len(seeds) if seeds is not None else 0
    eng = me.Engine(sc.num_symbols, sc.levels, base, max_batch=max(sc.batch, min(nseed, 1 << 20)),
                    max_resting=(1 << 23) + nseed)
    for i in range(0, nseed, 1 << 20):
        eng.submit_batch(seeds.take(slice(i, i + (1 << 20))), want_fills=False)
    buf = np.zeros(sc.num_symbols * 24, dtype=np.uint64)
    for k in range(a.skip):
        eng.submit_batch(st.next(sc.batch), want_fills=False)
    lib.me_debug_stamps(eng.h, buf.ctypes.data, buf.size)
    before = buf.reshape(-1, 24)[:, :5].astype(np.float64).copy()
    for k in range(a.batches):
        eng.submit_batch(st.next(sc.batch), want_fills=False)
    lib.me_debug_stamps(eng.h, buf.ctypes.data, buf.size)
    d = buf.reshape(-1, 24)[:, :5].astype(np.float64) - before
    order = np.argsort(-d[:, 3])[: a.top]
    print(f"config {a.config}: {a.batches} batches; cycles per record walked (and per batch) by part")
    for s in order:
        r = max(d[s, 3], 1)
        print(f"  symbol {s}: {int(d[s, 3] / a.batches)} records/batch; set-up {d[s, 0] / r:7.1f} ({d[s, 0] / a.batches:9.0f}), "
              f"block set-up {d[s, 1] / r:6.1f}, record loop {d[s, 2] / r:7.1f}, end {d[s, 4] / r:6.1f} ({d[s, 4] / a.batches:8.0f})")
    eng.close()


if __name__ == "__main__":
    main()
