"""Diagnostic: where the grouped walk with cancels (k_agg_gwalk_cx) spends its cycles on config 5, from the
-DME_STAMPS build (never the product): the walker's barrier waits (the helper not done), its block set-up and
results, its record loop, and the helper's batch preparation.

    ME_ENGINE_LIB=matching_engine_amd/build/libme_engine_stamps.so ME_GW_CANCEL=1 python tools/cx_probe.py [--config 5]
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
    ap.add_argument("--config", type=int, default=5)
    ap.add_argument("--batches", type=int, default=20)
    ap.add_argument("--warm", type=int, default=5)
    a = ap.parse_args()
    assert "stamps" in me._abi.LIB_PATH, "set ME_ENGINE_LIB to the stamps build"
    sc = me.preset(a.config)
    st = me.Stream(sc)
    lib = me._abi.load()
    lib.me_debug_stamps.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t]
    eng = me.Engine(sc.num_symbols, sc.levels, st.base_prices(), max_batch=sc.batch, max_resting=1 << 24)
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
    d = buf.reshape(-1, 24).astype(np.float64)
    rec = np.maximum(d[:, 3], 1)
    print(f"config {a.config}: group of {a.batches} batches, paths {eng.paths()}, handoffs {eng.stats()['handoffs']}")
    print(f"walk duration (cycles) median {np.median(d[:, 17] - d[:, 16]):.0f}, records walked median {np.median(rec):.0f}")
    for i, n in enumerate(["barrier waits", "set-up+results", "record loop"]):
        print(f"walker {n:15s} median {np.median(d[:, i]):10.0f}  per record {np.median(d[:, i] / rec):7.1f}")
    print(f"helper prepare         median {np.median(d[:, 5]):10.0f}  per record {np.median(d[:, 5] / rec):7.1f}")
    # the record loop by record kind (k_agg_gwalk_cx only: dbg[s * 24 + 6..15])
    if d[:, 10:14].sum() > 0:
        for i, n in enumerate(["cancel (bounds)", "LIMIT", "MARKET", "cancel (list)"]):
            cyc, cnt = d[:, 6 + i].sum(), d[:, 10 + i].sum()
            print(f"record kind {n:15s} count {cnt:10.0f}  cycles per record {cyc / max(cnt, 1):7.1f}")
        print(f"cancels that emptied a best level {d[:, 14].sum():.0f}, removing from orders before the group {d[:, 15].sum():.0f}")

if __name__ == "__main__":
    main()
