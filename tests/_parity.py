"""Helpers shared by the parity tests: run the same batches through the GPU engine and the CPU
oracle and require bit-exact equality of per-record results, trade tapes and resting books."""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from matching_engine_amd import BOOK_ENTRY_DTYPE, FILL_DTYPE, RESULT_DTYPE  # noqa: E402

RES_FIELDS = ("filled_qty", "remaining_qty", "fill_count", "tape_offset", "status", "reason")


def assert_results_equal(got, exp, ctx=""):
    assert len(got) == len(exp), f"{ctx}: result count {len(got)} != {len(exp)}"
    for f in RES_FIELDS:
        bad = np.nonzero(got[f] != exp[f])[0]
        if len(bad):
            i = bad[0]
            raise AssertionError(f"{ctx}: field {f} differs at record {i} ({len(bad)} records): "
                                 f"got {got[i]} expected {exp[i]}")


def assert_fills_equal(got, exp, ctx=""):
    if len(got) != len(exp):
        n = min(len(got), len(exp))
        d = np.nonzero(got[:n] != exp[:n])[0]
        first = d[0] if len(d) else n
        raise AssertionError(f"{ctx}: tape length {len(got)} != {len(exp)}; first difference at {first}: "
                             f"got {got[first] if first < len(got) else None} "
                             f"expected {exp[first] if first < len(exp) else None}")
    bad = np.nonzero(got != exp)[0]
    if len(bad):
        i = bad[0]
        raise AssertionError(f"{ctx}: tape differs at {i} ({len(bad)} fills): got {got[i]} expected {exp[i]}")


def assert_books_equal(eng, orc, symbols, ctx=""):
    for s in symbols:
        g = eng.dump(int(s))
        e = orc.dump(int(s))
        if len(g) != len(e) or np.any(g != e):
            n = min(len(g), len(e))
            d = np.nonzero(g[:n] != e[:n])[0]
            first = d[0] if len(d) else n
            raise AssertionError(f"{ctx}: book of symbol {s} differs (gpu {len(g)} orders, oracle {len(e)}); "
                                 f"first at {first}: gpu {g[first] if first < len(g) else None} "
                                 f"oracle {e[first] if first < len(e) else None}")


def run_both(eng, orc, batches, check_books=True, book_symbols=None, ctx=""):
    """Submit every batch to both; compare after each batch. Returns total fills."""
    total = 0
    for k, b in enumerate(batches):
        rg, fg = eng.submit_batch(b)
        ro, fo = orc.submit(b)
        assert_results_equal(rg, ro, f"{ctx} batch {k}")
        assert_fills_equal(fg, fo, f"{ctx} batch {k}")
        total += len(fo)
    if check_books:
        syms = range(eng.num_symbols) if book_symbols is None else book_symbols
        assert_books_equal(eng, orc, syms, ctx)
        assert eng.resting_count() == orc.resting(), f"{ctx}: resting count"
        if hasattr(eng, "admission"):  # the device-wide counter admission control reads
            assert eng.admission()["resting"] == orc.resting(), f"{ctx}: ST_RESTING counter"
    return total


def load_fixture(cid):
    z = np.load(os.path.join(HERE, "golden", f"match_c{cid}.npz"))
    from matching_engine_amd import Batch

    batches, res, fills = [], [], []
    for k in range(int(z["nbatches"][0])):
        batches.append(Batch(*[z[f"b{k}_{f}"] for f in ("seq", "price_q4", "qty", "symbol", "kind")]))
        res.append(np.ascontiguousarray(z[f"b{k}_res"]).view(RESULT_DTYPE).reshape(-1))
        fills.append(np.ascontiguousarray(z[f"b{k}_fills"]).view(FILL_DTYPE).reshape(-1))
    book = np.ascontiguousarray(z["book"]).view(BOOK_ENTRY_DTYPE).reshape(-1)
    meta = dict(num_symbols=int(z["num_symbols"][0]), levels=int(z["levels"][0]), base=z["base"],
                book_counts=z["book_counts"])
    return meta, batches, res, fills, book


def side_levels(dump, side, depth):
    """Oracle resting orders of one side (dump order: priority) restricted to its first `depth`
    distinct prices."""
    d = dump[dump["side"] == side]
    prices = []
    keep = np.zeros(len(d), dtype=bool)
    for i, p in enumerate(d["price_q4"]):
        if not prices or prices[-1] != p:
            prices.append(p)
        keep[i] = len(prices) <= depth
    return d[keep]
