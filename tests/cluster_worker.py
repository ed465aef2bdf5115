"""One rank of the sharded-service check (launched by tests/test_multirank.py).

Rank 0 hosts a MatchingEngineService over a cluster.ShardedMatcher (the shards: this rank's and
the other ranks' books, symbols splitmix64-hashed); the other ranks serve its commands. Rank 0 also
runs the same request stream through a second service whose matcher spans rank 0 alone (one book
holding every symbol) and compares the two SQLite databases row by row, the per-order books
(GetOrderBook) and the gathered level snapshot.

env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT; argv: BOOK(oracle|gpu|oracle_refuse) TMPDIR OUT_JSON
  oracle: every shard book is the CPU oracle (the host protocol under gloo, CPU tensors)
  gpu:    every shard book is the HIP engine on cuda:0 (ranks share the box's one GPU; gloo)
  oracle_refuse: oracle shards, and the last rank's admission control refuses its part of the
          second slice once: no shard may apply anything of it, the service keeps it queued, the
          next flush matches it (all-or-none admission, cluster.ShardedMatcher._match)
"""
import json
import os
import sqlite3
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class OracleShard:
    """The oracle with the Engine methods the matcher uses (test infrastructure)."""

    def __init__(self, ids, refuse_calls=()):
        from oracle.oracle import OracleBook

        self.ids = np.asarray(ids, dtype=np.uint32)
        self.ob = OracleBook(max(len(ids), 1), symbol_ids=self.ids if len(ids) else None)
        self.refuse_calls, self.calls = set(refuse_calls), 0

    def admits(self, b):
        self.calls += 1
        return self.calls not in self.refuse_calls

    def submit_batch(self, b):
        return self.ob.submit(b)

    def book_orders(self, s, depth):
        from tests._parity import side_levels

        d = self.ob.dump(s)
        lb, la = self.ob.snapshot(s, depth)
        return side_levels(d, 1, depth), side_levels(d, 2, depth), lb, la

    def levels_all(self, depth):
        from matching_engine_amd import LEVEL_DTYPE

        n = len(self.ids)
        lv = np.zeros((n, 2, depth), dtype=LEVEL_DTYPE)
        cnt = np.zeros((n, 2), dtype=np.uint32)
        for s in range(n):
            b, a = self.ob.snapshot(s, depth)
            lv[s, 0, : len(b)] = b
            lv[s, 1, : len(a)] = a
            cnt[s] = (len(b), len(a))
        return lv, cnt


def rows(db):
    con = sqlite3.connect(db)
    o = con.execute("SELECT order_id, client_id, symbol, side, order_type, price, quantity, status, "
                    "remaining_quantity FROM orders ORDER BY order_id").fetchall()
    f = con.execute("SELECT id, order_id, symbol, fill_price, fill_quantity FROM fills ORDER BY id").fetchall()
    con.close()
    return o, f


def main():
    kind, tmp, out_path = sys.argv[1], sys.argv[2], sys.argv[3]
    import torch.distributed as dist

    import matching_engine_amd as me
    from matching_engine_amd.cluster import ShardedMatcher

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    solo = dist.new_group([0])  # rank 0 alone: the single-engine run
    S, L, MB, MR = 40, 128, 4096, 1 << 16
    syms = [f"S{i:02d}" for i in range(S)]
    mids = {s: 1_000_000 + 1000 * i for i, s in enumerate(syms)}
    base = np.array([mids[s] - 64 for s in syms], dtype=np.int64)

    refuse = kind == "oracle_refuse"

    def shard(ids, last=False):
        if kind in ("oracle", "oracle_refuse"):
            return OracleShard(ids, refuse_calls=(2,) if (refuse and last) else ())
        return None

    from matching_engine_amd.sharding import ShardPlan

    plan = ShardPlan(S, world)
    m = ShardedMatcher(S, L, base, MB, MR, shard_book=shard(plan.members[rank], last=rank == world - 1), device=0)
    if rank != 0:
        m.serve()
        dist.barrier()
        dist.destroy_process_group()
        return
    m1 = ShardedMatcher(S, L, base, MB, MR, shard_book=shard(np.arange(S, dtype=np.uint32)), device=0, group=solo)
    dbs = [os.path.join(tmp, "sharded.sqlite"), os.path.join(tmp, "single.sqlite")]
    svcs = [me.MatchingEngineService(None, syms[:5], db_path=dbs[0], matcher=m),
            me.MatchingEngineService(None, syms[:5], db_path=dbs[1], matcher=m1)]
    rng = np.random.default_rng(17)
    owner = {}
    live = []
    outs = [[], []]
    refused = 0
    msg = ""
    ok = True
    for slice_no in range(5):
        for _ in range(1500):
            if live and rng.random() < 0.15:
                oid = live[int(rng.integers(len(live)))]
                s = owner[oid][1]
                for v in svcs:
                    v.cancel_order(owner[oid][0], s, f"OID-{oid}")
                continue
            s = syms[int(rng.integers(S))]
            otype = 1 if rng.random() < 0.2 else 0
            side = int(rng.choice([1, 2]))
            px = mids[s] + int(rng.integers(-40, 41)) + (int(rng.integers(-900, 900)) if rng.random() < 0.02 else 0)
            qn = int(rng.integers(1, 80))
            client = f"C{int(rng.integers(3))}"
            r = [v.submit_order(client, s, otype, side, 0 if otype else px, 4, qn) for v in svcs]
            assert r[0] == r[1], r
            oid = int(r[0]["order_id"][4:])
            owner[oid] = (client, s)
            if otype == 0:
                live.append(oid)
        for k, v in enumerate(svcs):
            try:
                outs[k].append(v.flush())
            except me.ServiceError as e:
                if not (refuse and k == 0 and refused == 0):
                    raise
                refused += 1  # the sharded service: nothing matched, the slice is still pending
                if v.pending == 0 or "refused" not in str(e):
                    ok, msg = False, f"refused flush: pending {v.pending}, error {e}"
                outs[k].append(v.flush())
    for k in range(5):
        for a, b, what in zip(outs[0][k], outs[1][k], ("seq", "results", "tape")):
            if len(a) != len(b) or not np.array_equal(a, b):
                ok, msg = False, f"slice {k}: {what} differs"
    ra, rb = rows(dbs[0]), rows(dbs[1])
    if ra != rb:
        ok, msg = False, f"DB rows differ: orders {len(ra[0])} vs {len(rb[0])}, fills {len(ra[1])} vs {len(rb[1])}"
    for s in syms[::7]:
        if svcs[0].order_book(s) != svcs[1].order_book(s):
            ok, msg = False, f"order book of {s} differs"
        if svcs[0].market_data(s) != svcs[1].market_data(s):
            ok, msg = False, f"market data of {s} differs"
    lv, cnt = m.snapshot(5)
    lv1, cnt1 = m1.snapshot(5)
    if not (np.array_equal(cnt, cnt1) and np.array_equal(lv, lv1)):
        ok, msg = False, "level snapshots differ"
    nrows, nfills = len(ra[0]), len(ra[1])
    for v in svcs:
        v.close()
    m.stop()
    dist.barrier()
    if refuse and refused != 1:
        ok, msg = False, f"expected one refused flush, saw {refused}"
    json.dump({"ok": ok, "msg": msg, "orders": nrows, "fill_rows": nfills, "world": world, "refused": refused},
              open(out_path, "w"))
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
