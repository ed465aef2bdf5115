"""Diagnostic: per-symbol timeline of a grouped aggregate launch (k_agg_gwalk, then k_agg_gres's phases) from
the -DME_STAMPS build's absolute s_memtime stamps (never the product).

    ME_ENGINE_LIB=matching_engine_amd/build/libme_engine_stamps.so python tools/gres_probe.py [--batches 20]
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import matching_engine_amd as me  # noqa: E402


def pct(v):
    return " ".join(f"{q}%={np.percentile(v, q):9.0f}" for q in (0, 50, 90, 100))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--warm", type=int, default=5)
    a = ap.parse_args()
    assert "stamps" in me._abi.LIB_PATH, "set ME_ENGINE_LIB to the stamps build"
    sc = me.preset(a.config)
    st = me.Stream(sc)
    base = st.base_prices()
    lib = me._abi.load()
    lib.me_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    eng = me.Engine(sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=1 << 24)
    warm = [eng.upload(st.next(sc.batch)) for _ in range(a.warm)]
    timed = [eng.upload(st.next(sc.batch)) for _ in range(a.batches)]
    for db in warm:
        eng.submit_device(db)
    eng.sync()
    for db in timed:
        eng.submit_device(db)
    eng.sync()
    buf = np.zeros(sc.num_symbols * 24, dtype=np.uint64)
    lib.me_debug_stamps(eng.h, buf.ctypes.data, buf.size)
    gw = buf.reshape(-1, 24)[:, 0:4].astype(np.float64)  # the walk's parts (cycles) and records, per symbol
    m = buf.reshape(-1, 24)[:, 16:24].astype(np.float64)
    t0 = m[:, 0].min()
    m -= t0
    print(f"config {a.config}: {sc.num_symbols} symbols, group of {a.batches} batches; cycles from the first walk start")
    print("walk start      ", pct(m[:, 0]))
    print("walk duration   ", pct(m[:, 1] - m[:, 0]))
    print("walk end        ", pct(m[:, 1]))
    rec = np.maximum(gw[:, 3], 1)
    for i, n in enumerate(["batch set-up", "block set-up", "record loop"]):
        print(f"walk {n:13s}   ", pct(gw[:, i]), f"  per record (median) {np.median(gw[:, i] / rec):7.1f}")
    print("walk records    ", pct(gw[:, 3]))
    print("gres start      ", pct(m[:, 2]))
    names = ["A sort", "B levels", "C scan+results", "D1 alloc+fills", "D2 place"]
    for i, n in enumerate(names):
        print(f"gres {n:15s}", pct(m[:, 3 + i] - m[:, 2 + i]))
    print("gres duration   ", pct(m[:, 7] - m[:, 2]))
    print("gres end        ", pct(m[:, 7]))
    # occupancy rounds: symbols whose gres started after the earliest gres ended
    first_end = m[:, 7].min()
    print(f"symbols whose gres started after the first gres ended: {(m[:, 2] > first_end).sum()}")
    for db in warm + timed:
        db.free()
    eng.close()


if __name__ == "__main__":
    main()
