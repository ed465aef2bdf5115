"""Debug: L=64 register-kernel stream variants; prints which raise. args: none"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import matching_engine_amd as me
from oracle.oracle import OracleBook
from tests._parity import assert_results_equal, assert_fills_equal

def run(L, nb=6, **over):
    kw = dict(num_symbols=64, levels=L, batch=500, cancel_pct=40, market_pct=20, market_qty_mult=3, far_pct=1,
              drift_step=4, drift_every=9, spread_ticks=min(32, L // 2 - 1))
    kw.update(over)
    sc = me.preset(5, **kw)
    st = me.Stream(sc)
    base = st.base_prices()
    bs = [st.next(sc.batch) for _ in range(nb)]
    ob = OracleBook(sc.num_symbols)
    eng = me.Engine(sc.num_symbols, L, base, max_batch=sc.batch, max_resting=100000, max_chunks=100000,
                    seq_ring=1 << 20, batches_per_launch=1)
    for k, b in enumerate(bs):
        try:
            r, f = eng.submit_batch(b)
        except Exception as e:
            return f"batch {k} raised {str(e)[:80]}"
        ro, fo = ob.submit(b)
        try:
            assert_results_equal(r, ro, "")
            assert_fills_equal(f, fo, "")
        except AssertionError as e:
            return f"batch {k} differs {str(e)[:120]}"
    return "ok"

for name, L, over in [("base", 64, {}), ("far0", 64, dict(far_pct=0)), ("drift0", 64, dict(drift_step=0, drift_every=0)),
                      ("far0drift0", 64, dict(far_pct=0, drift_step=0, drift_every=0)), ("cancel0", 64, dict(cancel_pct=0)),
                      ("L128", 128, {}), ("far5_L64", 64, dict(far_pct=5, drift_step=0, drift_every=0)),
                      ("S1", 64, dict(num_symbols=1))]:
    print(name, run(L, **over), flush=True)
