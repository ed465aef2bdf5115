"""Debug: the long drift stream through device groups (G per launch), every batch against the
oracle; prints the first mismatch. args: G NBATCHES [sync_every]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import matching_engine_amd as me
from oracle.oracle import OracleBook
from tests._parity import assert_results_equal, assert_fills_equal

G, NB = int(sys.argv[1]), int(sys.argv[2])
sc = me.preset(5, num_symbols=256, levels=128, batch=8192, cancel_pct=10, market_pct=15, market_qty_mult=3,
               drift_step=1, drift_every=5, far_pct=1, seq_start=(1 << 33) + 777)
st = me.Stream(sc)
base = st.base_prices()
batches = [st.next(8192) for _ in range(NB)]
ob = OracleBook(256)
eng = me.Engine(256, 128, base, max_batch=8192, max_resting=1 << 22, seq_ring=1 << 22, batches_per_launch=G)
bad = None
for g0 in range(0, NB, G):
    grp = batches[g0:g0 + G]
    dbs = [eng.upload(b) for b in grp]
    for db in dbs:
        eng.submit_device(db)
    eng.sync()
    for k, b in enumerate(grp):
        r, f = eng.fetch_group_outputs(k, len(b))
        ro, fo = ob.submit(b)
        try:
            assert_results_equal(r, ro, "")
            assert_fills_equal(f, fo, "")
        except AssertionError as e:
            bad = (g0 + k, str(e)[:300])
            break
    for db in dbs:
        db.free()
    if bad:
        break
print("G", G, "first mismatch", bad, "handoffs", eng.stats()["handoffs"], flush=True)
