"""Regenerate the committed golden fixtures under tests/golden/ (run in the build container).

1. price_q4.json — outputs of the REFERENCE's own normalize_to_q4, compiled from
   /root/reference/include/domain/price.hpp by oracle/Makefile into oracle/_ref/ref_price.
   Pins the oracle restatement and the product's me_normalize_to_q4.
2. submit_contract.json — SubmitOrder request -> response/persisted-row cases. The reference
   server cannot be built here (gRPC/protobuf/SQLiteCpp absent), so expected
   values are restated from its source (cited per case); the Q4 prices inside come from (1).
3. match_c{1..6}.npz — small seeded streams of the five configurations, plus (6) a drifting,
   cancel-heavy stream with far-away LIMITs and OIDs above 2^33, run through the CPU oracle (an
   unbounded price-time book): per-batch results + tapes + final resting books. The reference has
   no matcher, so these are "parity unpinned" w.r.t. the reference: they pin the oracle against
   regressions and are the GPU engine's bit-exact target (its 128-level windows must re-centre and
   spill to far levels to reproduce them).

usage: python tests/golden/make_golden.py [--only price|contract|match]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

I64_MAX = (1 << 63) - 1
I64_MIN = -(1 << 63)


def price_pairs():
    pairs = [(10050, s) for s in range(0, 19)]  # test_price.cpp:8-13 and the full scale sweep
    pairs += [(10050, -1), (10050, 19), (10050, 100), (0, 0), (0, 18), (-10059, 5), (-10050, 8), (-1, 5),
              (1, 0), (-1, 0), (10 ** 15, 0), (-(10 ** 15), 0), (922337203685477, 0), (922337203685478, 0),
              (-922337203685477, 0), (-922337203685478, 0), (I64_MAX, 4), (I64_MIN, 4), (I64_MAX, 18),
              (I64_MIN, 18), (I64_MAX, 3), (I64_MIN, 3), (I64_MAX // 10, 3), (I64_MIN // 10, 3),
              (I64_MAX // 10 + 1, 3), (I64_MIN // 10 - 1, 3), (123456789, 2), (123456789, 8), (987654321, 12),
              (1000000, 4), (10000, 2), (100000000, 8)]
    rng = np.random.default_rng(20250905)
    for _ in range(200):
        p = int(rng.integers(-(10 ** 12), 10 ** 12))
        pairs.append((p, int(rng.integers(0, 19))))
    return pairs


def make_price():
    from oracle.oracle import ref_normalize_many

    pairs = price_pairs()
    outs = ref_normalize_many(pairs)
    rows = []
    for (p, s), o in zip(pairs, outs):
        rows.append({"price": p, "scale": s, "q4": o if isinstance(o, int) else None,
                     "exception": None if isinstance(o, int) else [o[1], o[2]]})
    meta = {"source": "oracle/_ref/ref_price built from /root/reference/include/domain/price.hpp:15-29",
            "cases": rows}
    with open(os.path.join(HERE, "price_q4.json"), "w") as f:
        json.dump(meta, f, indent=0)
    print(f"price_q4.json: {len(rows)} cases")


def make_contract():
    """SubmitOrder cases restated from src/server/matching_engine_service.cpp:41-121 and
    src/storage/storage.cpp:78-123 (fresh DB: load_next_oid_seq -> 1, storage.cpp:254-267)."""
    from oracle.oracle import ref_normalize_many

    L, M = 0, 1
    B, S_, U = 1, 2, 0
    reqs = [
        # tests/test_submit_order.cpp:57-79: LIMIT BUY 10050@8 qty 10 -> success, OID-1, price 1
        dict(symbol="SYM", order_type=L, side=B, price=10050, scale=8, quantity=10, cite="tests/test_submit_order.cpp:56-79"),
        # scripts/smoke.ps1:24-27 — four LIMIT BUY at scales 8, 9, 2, 0
        dict(symbol="SYM", order_type=L, side=B, price=10050, scale=9, quantity=5, cite="scripts/smoke.ps1:24-27"),
        dict(symbol="SYM", order_type=L, side=B, price=10050, scale=2, quantity=5, cite="scripts/smoke.ps1:24-27"),
        dict(symbol="SYM", order_type=L, side=B, price=10050, scale=0, quantity=5, cite="scripts/smoke.ps1:24-27"),
        # validation :66-83 (no OID consumed)
        dict(symbol="", order_type=L, side=B, price=100, scale=4, quantity=1, cite="matching_engine_service.cpp:66-71"),
        dict(symbol="SYM", order_type=L, side=B, price=100, scale=4, quantity=0, cite="matching_engine_service.cpp:72-77"),
        dict(symbol="SYM", order_type=L, side=B, price=100, scale=4, quantity=-5, cite="matching_engine_service.cpp:72-77"),
        dict(symbol="SYM", order_type=L, side=S_, price=0, scale=4, quantity=3, cite="matching_engine_service.cpp:78-83"),
        dict(symbol="SYM", order_type=L, side=S_, price=-7, scale=4, quantity=3, cite="matching_engine_service.cpp:78-83"),
        dict(symbol="", order_type=L, side=B, price=0, scale=4, quantity=0, cite="first failing check wins :66"),
        # MARKET: price not checked (:78), normalized anyway (:89-97); persisted with order_type=1
        dict(symbol="SYM", order_type=M, side=S_, price=0, scale=4, quantity=7, cite="matching_engine_service.cpp:78,89-97"),
        dict(symbol="SYM", order_type=M, side=B, price=-3, scale=4, quantity=7, cite="matching_engine_service.cpp:78"),
        dict(symbol="SYM", order_type=5, side=B, price=0, scale=4, quantity=7, cite="unknown type treated as MARKET :50,78"),
        # normalization throws after the OID was consumed (:85 before :89) -> gap, UNKNOWN
        dict(symbol="SYM", order_type=L, side=B, price=10050, scale=19, quantity=1, cite="price.hpp:16 + service :85"),
        dict(symbol="SYM", order_type=L, side=B, price=10 ** 15, scale=0, quantity=1, cite="price.hpp:23"),
        dict(symbol="SYM", order_type=M, side=B, price=-(10 ** 15), scale=0, quantity=1, cite="price.hpp:24"),
        # side not in (1,2): OID allocated, CHECK fails -> success=false "DB insert failed", order_id set
        dict(symbol="SYM", order_type=L, side=U, price=100, scale=4, quantity=1, cite="storage.cpp:32 CHECK + service :107-111"),
        dict(symbol="SYM", order_type=L, side=3, price=100, scale=4, quantity=1, cite="storage.cpp:32 CHECK"),
        # plain accepts after the gaps
        dict(symbol="ABC", order_type=L, side=S_, price=1005000, scale=4, quantity=2147483647, cite="service :41-121"),
        dict(symbol="ABC", order_type=L, side=S_, price=-10059, scale=5, quantity=1, cite="price <= 0 only checked raw"),
        dict(symbol="ABC", order_type=L, side=B, price=1, scale=8, quantity=1, cite="normalizes to 0, still persisted"),
    ]
    nexp = ref_normalize_many([(r["price"], r["scale"]) for r in reqs])
    cases = []
    next_id = 1
    for r, q in zip(reqs, nexp):
        exp = {"order_id": "", "success": False, "error_message": "", "grpc_status": 0, "row": None}
        if not r["symbol"]:
            exp["error_message"] = "symbol is required"
        elif r["quantity"] <= 0:
            exp["error_message"] = "quantity must be > 0"
        elif r["order_type"] == L and r["price"] <= 0:
            exp["error_message"] = "price must be > 0 for LIMIT"
        else:
            oid = f"OID-{next_id}"
            next_id += 1
            if not isinstance(q, int):
                exp["grpc_status"] = 2  # escaping exception -> grpc UNKNOWN
                exp["error_message"] = q[2]
            else:
                exp["order_id"] = oid
                if r["side"] in (1, 2):
                    exp["success"] = True
                    exp["row"] = {"price": q, "order_type": 1, "status": 0, "remaining_quantity": r["quantity"],
                                  "side": r["side"], "quantity": r["quantity"]}
                else:
                    exp["error_message"] = "DB insert failed"
        cases.append({"request": {k: v for k, v in r.items() if k != "cite"}, "cite": r["cite"], "expect": exp})
    with open(os.path.join(HERE, "submit_contract.json"), "w") as f:
        json.dump({"source": "restated from reference source (server not buildable here); Q4 values from "
                             "oracle/_ref/ref_price", "cases": cases}, f, indent=1)
    print(f"submit_contract.json: {len(cases)} cases")


# Small versions of the five configurations; shared with tests/test_gpu_parity.py.
FIXTURES = {
    1: dict(preset=1, over=dict(batch=2048), batches=4),
    2: dict(preset=2, over=dict(num_symbols=64, batch=4096), batches=4),
    3: dict(preset=3, over=dict(num_symbols=5000, batch=8192), batches=3),
    4: dict(preset=4, over=dict(num_symbols=40, levels=1024, spread_ticks=250, seed_levels_per_side=300,
                                batch=4096), batches=3),
    5: dict(preset=5, over=dict(num_symbols=64, batch=4096), batches=4),
    # mids trend 3 ticks every 4 records of a symbol (~3 windows over the stream), 2 % of LIMITs
    # priced L..64L away, 20 % cancels, sweeping MARKETs, OIDs from 2^33 + 12345
    6: dict(preset=5, over=dict(num_symbols=32, batch=2048, cancel_pct=20, market_pct=15, market_qty_mult=4,
                                drift_step=3, drift_every=4, far_pct=2, seq_start=(1 << 33) + 12345),
            batches=8),
}


def fixture_stream(cfg_id):
    """(stream config, list of batches) of one fixture, deterministic."""
    import matching_engine_amd as me

    fx = FIXTURES[cfg_id]
    sc = me.preset(fx["preset"], **fx["over"])
    st = me.Stream(sc)
    batches = []
    if sc.seed_levels_per_side:
        batches.append(st.seed_books(range(sc.num_symbols), sc.seed_levels_per_side))
    for _ in range(fx["batches"]):
        batches.append(st.next(sc.batch))
    return sc, st.base_prices(), batches


def make_match():
    from oracle.oracle import OracleBook

    for cid, fx in FIXTURES.items():
        sc, base, batches = fixture_stream(cid)
        ob = OracleBook(sc.num_symbols)
        out = {"base": base, "levels": np.array([sc.levels]), "num_symbols": np.array([sc.num_symbols]),
               "nbatches": np.array([len(batches)])}
        for k, b in enumerate(batches):
            res, fills = ob.submit(b)
            for f in ("seq", "price_q4", "qty", "symbol", "kind"):
                out[f"b{k}_{f}"] = getattr(b, f)
            out[f"b{k}_res"] = res.view(np.uint8).reshape(len(res), 20)
            out[f"b{k}_fills"] = fills.view(np.uint8).reshape(len(fills), 32)
        dumps = [ob.dump(s) for s in range(sc.num_symbols)]
        out["book_counts"] = np.array([len(d) for d in dumps], dtype=np.int64)
        out["book"] = np.concatenate(dumps).view(np.uint8).reshape(-1, 24) if sum(len(d) for d in dumps) else \
            np.zeros((0, 24), dtype=np.uint8)
        path = os.path.join(HERE, f"match_c{cid}.npz")
        np.savez_compressed(path, **out)
        nf = sum(len(out[f"b{k}_fills"]) for k in range(len(batches)))
        print(f"match_c{cid}.npz: {sum(len(b) for b in batches)} records, {nf} fills, "
              f"{int(out['book_counts'].sum())} resting, {os.path.getsize(path)} B")


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["price", "contract", "match"])
    a = ap.parse_args()
    if a.only in (None, "price"):
        make_price()
    if a.only in (None, "contract"):
        make_contract()
    if a.only in (None, "match"):
        make_match()
