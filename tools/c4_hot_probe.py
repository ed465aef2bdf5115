#!/usr/bin/env python3
"""Config 4's hot symbol alone: symbol 0 of the c4 stream (Zipf(1.1) over 100k symbols, ~13.7 % of
every batch) with its book seeded to 10,000 levels per side at L = 32,768, fed only its own records
in stream order. Prints the kernel time per hot record — the figure that bounds config 4 on one GPU
— and, run under rocprofv3 --pmc, gives the SQ counters per hot record.

    python tools/c4_hot_probe.py [--batches 24] [--lib path/to/libme_engine.so]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=24)
    ap.add_argument("--warmup", type=int, default=4)
    a = ap.parse_args()
    import matching_engine_amd as me

    sc = me.preset(4, batch=65536)
    st = me.Stream(sc)
    base = st.base_prices()
    seeds = st.seed_books([0], 10_000)
    hot = []
    for _ in range(a.batches):
        b = st.next(sc.batch)
        sel = np.nonzero(b.symbol == 0)[0]
        hb = b.take(sel)
        hb.symbol = np.zeros(len(hb), dtype=np.uint32)
        hot.append(hb)
    n_all = sum(len(h) for h in hot) + len(seeds)
    eng = me.Engine(1, sc.levels, base[:1], max_batch=max(len(seeds), max(len(h) for h in hot)) + 1,
                    max_resting=n_all + 1024, max_chunks=n_all + 64, seq_ring=1 << 26)
    eng.submit_batch(seeds, want_fills=False)
    dbs = [eng.upload(h) for h in hot]
    for db in dbs[: a.warmup]:
        eng.submit_device(db)
    eng.sync()
    eng.timing_enable(1)
    t0 = time.perf_counter()
    for db in dbs[a.warmup:]:
        eng.submit_device(db)
    eng.sync()
    dt = time.perf_counter() - t0
    tm = eng.timing_read()
    n = sum(db.n for db in dbs[a.warmup:])
    print(json.dumps({"hot_records": n, "records_per_batch": n / max(len(dbs) - a.warmup, 1),
                      "kernel_us_per_record": tm["match_ms"] * 1e3 / max(tm["orders"], 1),
                      "wall_us_per_record": dt * 1e6 / n, "fills_per_record": tm["fills"] / n,
                      "config4_bound_orders_per_s": 1.0 / (0.137 * tm["match_ms"] * 1e-3 / max(tm["orders"], 1)),
                      "handoffs": eng.stats()["handoffs"]}), flush=True)
    for db in dbs:
        db.free()
    eng.close()


if __name__ == "__main__":
    main()
