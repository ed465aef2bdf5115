"""Debug: one fuzz case (tests/test_gpu_fuzz.py) through a chosen path, reporting the first batch
that raises or differs. args: SEED [path] [G]"""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import matching_engine_amd as me
from oracle.oracle import OracleBook
from tests._parity import assert_results_equal, assert_fills_equal
from tests.test_gpu_fuzz import _case

seed = int(sys.argv[1])
sc, base, batches, group, path, lag = _case(me, seed)
if len(sys.argv) > 2: path = sys.argv[2]
if len(sys.argv) > 3: group = int(sys.argv[3])
print("case", dict(L=sc.levels, S=sc.num_symbols, batch=sc.batch, G=group, path=path, cancel=sc.cancel_pct,
                   market=sc.market_pct, mqm=sc.market_qty_mult, far=sc.far_pct, drift=(sc.drift_step, sc.drift_every),
                   seq0=sc.seq_start, zipf=sc.zipf_s, nb=len(batches)), flush=True)
total = sum(len(b) for b in batches)
ob = OracleBook(sc.num_symbols)
eng = me.Engine(sc.num_symbols, sc.levels, base, max_batch=sc.batch, max_resting=total + 1024,
                max_chunks=total + 2 * sc.num_symbols + 64, seq_ring=1 << 20, batches_per_launch=group)
for k, b in enumerate(batches):
    try:
        r, f = eng.submit_batch(b)
    except Exception as e:
        print("batch", k, "raised", e, flush=True)
        break
    ro, fo = ob.submit(b)
    try:
        assert_results_equal(r, ro, "")
        assert_fills_equal(f, fo, "")
    except AssertionError as e:
        print("batch", k, "differs", str(e)[:300], flush=True)
        break
else:
    print("all", len(batches), "batches equal", flush=True)
print("handoffs", eng.stats()["handoffs"] if not eng_failed(eng) else None) if False else None
