#!/usr/bin/env python3
"""Where the pipelined host path's time goes (config 2 batches through me_submit_host / me_collect):
host time inside submit_host (staging copy + H2D enqueue + launches) and collect (waits), per group
size. Diagnostic only."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import matching_engine_amd as me  # noqa: E402


def run(group, nb=288, slots=0):
    sc = me.preset(2, batch=65536)
    st = me.Stream(sc)
    base = st.base_prices()
    batches = [st.next(sc.batch) for _ in range(nb)]
    eng = me.Engine(sc.num_symbols, sc.levels, base, max_batch=65537, max_resting=int(os.environ.get('E2E_REST_MULT', '1')) * (nb * 65536 // 3) + 65536,
                    seq_ring=1 << 28, batches_per_launch=group, host_slots=slots)
    H = eng.config()["host_slots"]
    eng.host_reserve()
    warm = H + 8
    for b in batches[:warm]:
        eng.collect(eng.submit_host(b), copy=False)
    t_sub = t_col = 0.0
    pend = []
    t0 = time.perf_counter()
    for b in batches[warm:]:
        if len(pend) == H:
            a = time.perf_counter()
            eng.collect(pend.pop(0), copy=False)
            t_col += time.perf_counter() - a
        a = time.perf_counter()
        pend.append(eng.submit_host(b))
        t_sub += time.perf_counter() - a
    a = time.perf_counter()
    for t in pend:
        eng.collect(t, copy=False)
    t_col += time.perf_counter() - a
    dt = time.perf_counter() - t0
    n = sum(len(b) for b in batches[warm:])
    adm = eng.admission()
    eng.close()
    return {"group": group, "slots": H, "orders_per_s": n / dt, "submit_ms_per_batch": t_sub / (nb - warm) * 1e3,
            "collect_ms_per_batch": t_col / (nb - warm) * 1e3, "total_ms_per_batch": dt / (nb - warm) * 1e3,
            "admission_exact_counts": adm["exact_counts"], "resting": adm["resting"]}


if __name__ == "__main__":
    # args: GROUP[:SLOTS[:BATCHES]] ... (SLOTS 0 = the engine's default, 3G + 1; BATCHES 288)
    for a in sys.argv[1:] or ["8", "16", "32"]:
        g, h, nb = (a.split(":") + ["0", "288"])[:3] if ":" in a else (a, "0", "288")
        print(json.dumps(run(int(g), nb=int(nb or 288), slots=int(h or 0))), flush=True)
