"""One rank of the sharded-deployment checks (launched by tests/test_multirank.py), through the C++
cluster (include/me_cluster.h, csrc/me_cluster.cpp) — no torch.distributed anywhere.

Rank 0 drives the cluster: (1) direct slices through me_cluster_submit / collect (two in flight) against
ONE oracle book over the whole stream, out-of-range symbol ids included; (2) a SubmitOrder service over
me_cluster_matcher next to a service over a single oracle book fed the same requests: every flush's
outputs, all SQLite rows, the per-order books, market data and the gathered level snapshot must be
equal. The other ranks sit in me_cluster_serve.

env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT; argv: KIND TMPDIR OUT_JSON
  oracle:        oracle shards (me_shard_ops over the CPU oracle), TCP transport
  oracle_refuse: oracle shards; the last rank's admission refuses its 2nd part once: nothing of that slice
                 may apply anywhere, the service splits it and matches the halves
  gpu:           HIP engine shards on cuda:0 (ranks share the box's one GPU), TCP transport
  rccl:          HIP engine shard over RCCL (world size 1 on a one-GPU box: every RCCL call of the protocol,
                 the self send / recv included)
"""
import json
import os
import sqlite3
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class OracleShard:
    """The oracle behind me_shard_ops (test infrastructure)."""

    def __init__(self, ids, refuse_calls=()):
        from oracle.oracle import OracleBook

        self.ids = np.asarray(ids, dtype=np.uint32)
        self.ob = OracleBook(max(len(ids), 1), symbol_ids=self.ids if len(ids) else None)
        self.refuse_calls, self.calls, self.refused = set(refuse_calls), 0, 0

    def admit(self, n_rest):
        self.calls += 1
        if self.calls in self.refuse_calls:
            self.refused += 1
            return False
        return True

    def match(self, b):
        return self.ob.submit(b)

    def book_orders(self, s, depth):
        from tests._parity import side_levels

        depth = depth or (1 << 20)  # 0: the whole book
        d = self.ob.dump(s)
        lb, la = self.ob.snapshot(s, depth)
        return side_levels(d, 1, depth), side_levels(d, 2, depth), lb, la

    def levels_all(self, depth):
        from matching_engine_amd import LEVEL_DTYPE

        n = max(len(self.ids), 1)
        lv = np.zeros((n, 2, depth), dtype=LEVEL_DTYPE)
        cnt = np.zeros((n, 2), dtype=np.uint32)
        for s in range(len(self.ids)):
            b, a = self.ob.snapshot(s, depth)
            lv[s, 0, : len(b)] = b
            lv[s, 1, : len(a)] = a
            cnt[s] = (len(b), len(a))
        return lv, cnt


class SingleBook:
    """One oracle book holding every symbol, as a me_matcher (cluster.python_matcher)."""

    def __init__(self, S, max_batch, max_resting):
        self.shard = OracleShard(np.arange(S, dtype=np.uint32))
        self.num_symbols, self.max_batch, self.max_resting = S, max_batch, max_resting

    def match(self, b):
        return self.shard.match(b)

    def book_orders(self, s, depth):
        return self.shard.book_orders(s, depth)

    def c_matcher(self):
        from matching_engine_amd.cluster import python_matcher

        return python_matcher(self)


def rows(db):
    con = sqlite3.connect(db)
    o = con.execute("SELECT order_id, client_id, symbol, side, order_type, price, quantity, status, "
                    "remaining_quantity FROM orders ORDER BY order_id").fetchall()
    f = con.execute("SELECT id, order_id, symbol, fill_price, fill_quantity FROM fills ORDER BY id").fetchall()
    con.close()
    return o, f


def direct_batch(st, sc, S, k):
    """Direct slices use the upper half of the symbol ids (the service below uses the lower half, so
    its orders never meet these books' resting orders, which have no DB rows)."""
    b = st.next(sc.batch)
    b.symbol = (S // 2 + b.symbol % (S // 2)).astype(np.uint32)
    if k == 1:
        b.symbol[::997] = S + 5  # unknown ids: BAD_SYMBOL, like one engine
    return b


def direct_slices(me, cl, S, world):
    """Slices straight through me_cluster_submit / collect, two in flight, against one oracle book."""
    from oracle.oracle import OracleBook

    sc = me.preset(5, num_symbols=S, batch=3000)
    st = me.Stream(sc)
    ref = OracleBook(S)
    batches = [direct_batch(st, sc, S, k) for k in range(6)]
    fills = 0
    pend = []
    for k, b in enumerate(batches):
        pend.append((cl.submit(b), b))
        if len(pend) == 2 or k == len(batches) - 1:
            while pend:
                t, bb = pend.pop(0)
                res, tape = cl.collect(t, len(bb))
                ro, fo = ref.submit(bb)
                fills += len(fo)
                if not (len(tape) == len(fo) and np.array_equal(tape, fo)):
                    return False, f"direct slice {k}: tape differs ({len(tape)} vs {len(fo)})", fills
                for x in ("filled_qty", "remaining_qty", "fill_count", "tape_offset", "status", "reason"):
                    if not np.array_equal(res[x], ro[x]):
                        return False, f"direct slice {k}: results.{x} differs", fills
    return True, "", fills


def main():
    kind, tmp, out_path = sys.argv[1], sys.argv[2], sys.argv[3]
    import matching_engine_amd as me
    from matching_engine_amd.cluster import Cluster, ShardOps, shard_symbols

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    port = int(os.environ["MASTER_PORT"])
    S, L, MR = 40, 128, 1 << 16
    MB = int(os.environ.get("ME_TEST_MAX_BATCH", "4096"))  # (a large one: the cluster reserves few slots)
    syms = [f"S{i:02d}" for i in range(S)]
    mids = {s: 1_000_000 + 1000 * i for i, s in enumerate(syms)}
    base = np.array([mids[s] - 64 for s in syms], dtype=np.int64)
    refuse = kind == "oracle_refuse"
    gpu = kind in ("gpu", "rccl")
    ops = None
    if not gpu:
        shard = OracleShard(shard_symbols(S, world, rank), refuse_calls=(2,) if (refuse and rank == world - 1) else ())
        ops = ShardOps(shard, MR)
    cl = Cluster(rank, world, S, MB, transport="rccl" if kind == "rccl" else "tcp", port=port, device=0, levels=L,
                 base_prices=base, max_resting=MR, shard_ops=ops, timeout_ms=120000)
    if rank != 0:
        cl.serve()
        res = {"refused": shard.refused if ops is not None else 0, "stats": cl.stats()}
        tmp = out_path + f".r{rank}.tmp"
        with open(tmp, "w") as f:
            json.dump(res, f)
        os.replace(tmp, out_path + f".r{rank}")  # rank 0 polls for the file: it appears complete
        cl.close()
        return
    ok, msg, direct_fills = (True, "", 0) if refuse else direct_slices(me, cl, S, world)
    # fresh books for the service comparison: a second cluster would need a second port; instead the
    # single-book side replays the direct slices first, so both sides start from the same books
    single = SingleBook(S, MB, world * MR)
    if not refuse:
        sc = me.preset(5, num_symbols=S, batch=3000)
        st = me.Stream(sc)
        for k in range(6):
            single.match(direct_batch(st, sc, S, k))
    first_oid = 6 * 3000 + 1 if not refuse else 1
    dbs = [os.path.join(tmp, "sharded.sqlite"), os.path.join(tmp, "single.sqlite")]
    svcs = [me.MatchingEngineService(None, syms[:5], db_path=dbs[0], matcher=cl),
            me.MatchingEngineService(None, syms[:5], db_path=dbs[1], matcher=single)]
    rng = np.random.default_rng(17)
    owner, live = {}, []
    outs = [[], []]
    # the services start at OID 1 while the books already hold the direct slices' seqs (up to 18,000):
    # burn OIDs below first_oid with requests the service rejects after allocating an OID (side 0)
    for _ in range(first_oid - 1):
        for v in svcs:
            v.submit_order("C", "S00", 0, 0, 100, 4, 1)
    for slice_no in range(5):
        for _ in range(1500):
            if live and rng.random() < 0.15:
                oid = live[int(rng.integers(len(live)))]
                for v in svcs:
                    v.cancel_order(owner[oid][0], owner[oid][1], f"OID-{oid}")
                continue
            s = syms[int(rng.integers(S // 2))]
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
            outs[k].append(v.flush())
    for k in range(5):
        for a, b, what in zip(outs[0][k], outs[1][k], ("seq", "results", "tape")):
            if ok and (len(a) != len(b) or not np.array_equal(a, b)):
                ok, msg = False, f"service slice {k}: {what} differs"
    ra, rb = rows(dbs[0]), rows(dbs[1])
    if ok and ra != rb:
        ok, msg = False, f"DB rows differ: orders {len(ra[0])} vs {len(rb[0])}, fills {len(ra[1])} vs {len(rb[1])}"
    for s in syms[::7]:
        if ok and svcs[0].order_book(s) != svcs[1].order_book(s):
            ok, msg = False, f"order book of {s} differs"
        if ok and svcs[0].market_data(s) != svcs[1].market_data(s):
            ok, msg = False, f"market data of {s} differs"
        if ok and [x.tolist() for x in svcs[0].get_order_book(s, 5)] != [x.tolist() for x in svcs[1].get_order_book(s, 5)]:
            ok, msg = False, f"level view of {s} differs"
    lv, cnt = cl.snapshot(5)
    lv1 = np.zeros_like(lv)
    cnt1 = np.zeros_like(cnt)
    for s in range(S):
        b, a = single.shard.ob.snapshot(s, 5)
        lv1[s, 0, : len(b)] = b
        lv1[s, 1, : len(a)] = a
        cnt1[s] = (len(b), len(a))
    if ok and not (np.array_equal(cnt, cnt1) and np.array_equal(lv, lv1)):
        ok, msg = False, "level snapshots differ"
    nrows, nfills = len(ra[0]), len(ra[1])
    errs = [v.last_error() for v in svcs]
    for v in svcs:
        v.close()
    st0 = cl.stats()
    cl.stop()
    cl.close()
    refused = 0
    if refuse:
        import time

        path = out_path + f".r{world - 1}"
        for _ in range(400):
            if os.path.exists(path):
                break
            time.sleep(0.05)
        if world > 1:
            with open(path) as f:
                refused = json.load(f)["refused"]
        else:
            refused = shard.refused
        if refused != 1:
            ok, msg = False, f"expected one refusal, saw {refused}"
    json.dump({"ok": ok, "msg": msg, "orders": nrows, "fill_rows": nfills, "world": world, "refused": refused,
               "direct_fills": direct_fills, "errors": errs, "slices": st0["slices"], "bytes": st0["bytes"]},
              open(out_path, "w"))


if __name__ == "__main__":
    main()
