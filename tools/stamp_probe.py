"""Diagnostic: phase cycle shares of k_match from the -DME_STAMPS build (never the product).

    ME_ENGINE_LIB=matching_engine_amd/build/libme_engine_stamps.so python tools/stamp_probe.py [--config 2]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import matching_engine_amd as me  # noqa: E402

PH = ["prologue", "fetch", "sweep", "walk", "rest", "cancel", "result", "epilogue", "sw_window", "sw_update",
      "sw_jump", "sw_best"]
WK = ["wk_get", "wk_scan", "wk_emit", "wk_tail"]
CT = ["cache_miss", "walks", "evictions", "fast_path"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batches", type=int, default=30)
    ap.add_argument("--skip", type=int, default=5, help="warm batches not measured")
    ap.add_argument("--symbols", type=int, default=0)
    ap.add_argument("--seed-top", type=int, default=0, help="config 4: pre-seed the K most popular books")
    ap.add_argument("--per-side", type=int, default=10_000)
    a = ap.parse_args()
    assert "stamps" in me._abi.LIB_PATH, "set ME_ENGINE_LIB to the stamps build"
    over = {"num_symbols": a.symbols} if a.symbols else {}
    sc = me.preset(a.config, **over)
    st = me.Stream(sc)
    base = st.base_prices()
    lib = me._abi.load()
    lib.me_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    seeds = st.seed_books(range(a.seed_top), a.per_side) if a.seed_top else None
    nseed = len(seeds) if seeds is not None else 0
    eng = me.Engine(sc.num_symbols, sc.levels, base, max_batch=max(sc.batch, min(nseed, 1 << 20)),
                    max_resting=(1 << 23) + nseed)
    for i in range(0, nseed, 1 << 20):
        eng.submit_batch(seeds.take(slice(i, i + (1 << 20))), want_fills=False)
    hot = np.zeros(24, dtype=np.float64)
    buf = np.zeros(sc.num_symbols * 24, dtype=np.uint64)
    tot = np.zeros(24, dtype=np.float64)
    maxwave = []
    norders = 0
    for k in range(a.batches):
        b = st.next(sc.batch)
        eng.submit_batch(b, want_fills=False)
        if k < a.skip:
            continue  # warm
        lib.me_debug_stamps(eng.h, buf.ctypes.data, buf.size)
        m = buf.reshape(-1, 24).astype(np.float64)
        tot += m.sum(0)
        wsum = m[:, :12].sum(1) + m[:, 16:20].sum(1)
        maxwave.append(wsum.max())
        hot += m[int(np.argmax(wsum))]
        norders += len(b)
    cyc = np.concatenate([tot[:12], tot[16:20]])
    share = cyc / cyc.sum()
    per_order = cyc / norders
    print(f"config {a.config}: {norders} orders, {sc.num_symbols} symbols")
    for p, s_, c in zip(PH + WK, share, per_order):
        print(f"  {p:9s} {100 * s_:6.2f}%  {c:9.1f} cycles/order")
    for name, v in zip(CT, tot[12:16]):
        print(f"  {name:10s} {v / norders:.3f} per order")
    print(f"  total {cyc.sum() / norders:.1f} cycles/order/wave; slowest wave {np.mean(maxwave):.0f} cycles/batch")
    hc = np.concatenate([hot[:12], hot[16:20]]) / len(maxwave)
    print("  slowest wave per batch, cycles:", ", ".join(f"{p} {c:.0f}" for p, c in zip(PH + WK, hc) if c),
          "| counts:", ", ".join(f"{n} {v / len(maxwave):.0f}" for n, v in zip(CT, hot[12:16] )))


if __name__ == "__main__":
    main()
