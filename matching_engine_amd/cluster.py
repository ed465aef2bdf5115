"""Sharded deployment: one rank per GPU behind ONE SubmitOrder service.

Rank 0 hosts the service (include/me_service.h: SubmitOrder, time slices, SQLite); every rank owns
the books of the symbols splitmix64(symbol) % world == rank on its own GPU. The service reaches the
shards through a matcher (me_service_create_matcher) whose calls rank 0 turns into commands that
every rank runs together (the other ranks sit in ``serve()``):

  MATCH     rank 0 broadcasts the slice; each rank matches its part on its engine
            (me_submit_host / me_collect); tapes and results are gathered to rank 0 and merged by
            taker seq (gather.py) — the exact single-engine output, which the service then persists
            in one transaction per slice.
  BOOK      GetOrderBook of one symbol: its owner runs the device snapshot kernel
            (me_book_orders), the entries are gathered to rank 0.
  SNAPSHOT  the periodic book snapshot: every rank's top-N levels of all its symbols
            (me_book_levels_all, one launch), gathered to rank 0 (``levels`` on rank 0).
  STOP      the serve loops return.

Collectives run on torch.distributed: "nccl" (RCCL over xGMI) moves the merged payloads between GPUs;
"gloo" runs the same protocol with CPU tensors (the tests). The only data exchanged is the slice
going out and each shard's outputs coming back — matching itself never crosses GPUs.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import BOOK_ENTRY_DTYPE, FILL_DTYPE, LEVEL_DTYPE, RESULT_DTYPE
from .engine import Batch, Engine
from .gather import gather_batch
from .sharding import ShardPlan

CMD_MATCH, CMD_BOOK, CMD_SNAPSHOT, CMD_STOP = 1, 2, 3, 4
_REC = 8 + 8 + 4 + 4 + 1  # packed slice record: seq, price_q4, qty, symbol, kind


class SliceRefused(RuntimeError):
    """A shard's admission control refused its part of a slice; no shard applied anything."""


class ShardedMatcher:
    """The matcher of a sharded deployment (one instance per rank).

    shard_book: this rank's book object with the Engine interface used here (submit_batch,
    book_orders, levels_all); None = an Engine on `device` holding this rank's symbols.
    """

    def __init__(self, num_symbols: int, levels: int, base_prices, max_batch: int, max_resting: int,
                 shard_book=None, device: int = 0, group=None, snapshot_depth: int = 10, **engine_kw):
        import torch
        import torch.distributed as dist

        self.dist, self.torch = dist, torch
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.num_symbols, self.max_batch, self.max_resting = num_symbols, max_batch, max_resting
        self.plan = ShardPlan(num_symbols, self.world)
        self.ids = self.plan.members[self.rank]
        base = np.ascontiguousarray(base_prices, dtype=np.int64)
        self.book = shard_book if shard_book is not None else Engine(
            max(len(self.ids), 1), levels, base[self.ids] if len(self.ids) else base[:1], max_batch=max_batch,
            max_resting=max_resting, device=device, symbol_ids=self.ids if len(self.ids) else None, **engine_kw)
        self.dev = torch.device("cuda", device) if dist.get_backend(group) == "nccl" else torch.device("cpu")
        self.snapshot_depth = snapshot_depth
        self.levels = None   # rank 0: last SNAPSHOT, [num_symbols, 2, depth] LEVEL_DTYPE
        self.counts = None
        self._keep = None    # rank 0: outputs of the last MATCH (the service reads them until the next)
        self._cmatcher = None

    # ---------------------------------------------------------------- the command channel
    def _bcast_header(self, cmd=0, a=0, b=0):
        t = self.torch.tensor([cmd, a, b], dtype=self.torch.int64, device=self.dev)
        self.dist.broadcast(t, src=0, group=self.group)
        return [int(x) for x in t.cpu()]

    def serve(self):
        """Ranks != 0: run the commands rank 0 issues until STOP."""
        while True:
            cmd, a, b = self._bcast_header()
            if cmd == CMD_STOP:
                return
            if cmd == CMD_MATCH:
                self._match(None, a)
            elif cmd == CMD_BOOK:
                self._book(a, b)
            elif cmd == CMD_SNAPSHOT:
                self._snapshot(a)

    def stop(self):
        if self.rank == 0:
            self._bcast_header(CMD_STOP)

    # ---------------------------------------------------------------- commands (all ranks)
    def _match(self, batch, n):
        torch = self.torch
        buf = torch.empty(max(n * _REC, 1), dtype=torch.uint8, device=self.dev)
        if self.rank == 0:
            host = np.empty(n * _REC, dtype=np.uint8)
            o = 0
            for a in (batch.seq, batch.price_q4, batch.qty, batch.symbol, batch.kind):
                host[o:o + a.nbytes] = a.view(np.uint8)
                o += a.nbytes
            buf[: n * _REC].copy_(torch.from_numpy(host))
        self.dist.broadcast(buf, src=0, group=self.group)
        raw = buf[: n * _REC].cpu().numpy()
        cols, o = [], 0
        for t, w in ((np.uint64, 8), (np.int64, 8), (np.int32, 4), (np.uint32, 4), (np.uint8, 1)):
            cols.append(raw[o:o + n * w].view(t))
            o += n * w
        b = Batch(*cols)
        lb, pos = self.plan.split(b)[self.rank]
        # all-or-none: every shard's admission control must take its part before any shard applies
        # its part (a refused slice stays queued in the service, no book changed)
        ok = torch.tensor([1 if (not len(lb) or not hasattr(self.book, "admits") or self.book.admits(lb)) else 0],
                          dtype=torch.int64, device=self.dev)
        self.dist.all_reduce(ok, op=self.dist.ReduceOp.MIN, group=self.group)
        if int(ok.item()) == 0:
            return None
        if len(lb):
            r, f = self.book.submit_batch(lb)
        else:
            r, f = np.zeros(0, dtype=RESULT_DTYPE), np.zeros(0, dtype=FILL_DTYPE)
        tape = torch.from_numpy(f.view(np.uint8).copy()).to(self.dev)
        res = torch.from_numpy(r.view(np.uint8).copy()).to(self.dev)
        post = torch.from_numpy(pos.astype(np.int64)).to(self.dev)
        return gather_batch(tape, len(f), res, post, len(lb), n, 0, self.group)

    def _book(self, symbol, depth):
        owner = int(self.plan.shard[symbol]) if symbol < self.num_symbols else -1
        mine = None
        if owner == self.rank:
            if depth == 0:  # the whole book
                cfg = self.book.config() if hasattr(self.book, "config") else {"levels": 1 << 20, "far_levels": 0}
                depth = cfg["levels"] + cfg["far_levels"]
            mine = self.book.book_orders(int(self.plan.local[symbol]), depth)
        got = [None] * self.world if self.rank == 0 else None
        self.dist.gather_object(mine, got, dst=0, group=self.group)
        return None if got is None or owner < 0 else got[owner]

    def _snapshot(self, depth):
        lv, cnt = self.book.levels_all(depth) if len(self.ids) else (None, None)
        got = [None] * self.world if self.rank == 0 else None
        self.dist.gather_object((self.ids, lv, cnt), got, dst=0, group=self.group)
        if self.rank != 0:
            return
        levels = np.zeros((self.num_symbols, 2, depth), dtype=LEVEL_DTYPE)
        counts = np.zeros((self.num_symbols, 2), dtype=np.uint32)
        for ids, l, c in got:
            if l is not None and len(ids):
                levels[ids] = l[: len(ids)]
                counts[ids] = c[: len(ids)]
        self.levels, self.counts = levels, counts

    # ---------------------------------------------------------------- rank 0 API
    def match(self, batch: Batch):
        """One slice through every shard -> (results, tape) merged on rank 0. Raises SliceRefused
        when a shard's admission control refused its part: then no shard applied anything."""
        self._bcast_header(CMD_MATCH, len(batch))
        got = self._match(batch, len(batch))
        if got is None:
            raise SliceRefused("a shard's max_resting refused the slice; no book changed")
        tape, res = got
        return res, tape

    def book_orders(self, symbol: int, depth: int):
        self._bcast_header(CMD_BOOK, symbol, depth)
        return self._book(symbol, depth)

    def snapshot(self, depth: int | None = None):
        """The periodic book snapshot: top-`depth` levels of every symbol of every shard on rank 0."""
        d = depth or self.snapshot_depth
        self._bcast_header(CMD_SNAPSHOT, d)
        self._snapshot(d)
        return self.levels, self.counts

    # ---------------------------------------------------------------- the C-ABI matcher (rank 0)
    def c_matcher(self) -> "_abi.MeMatcher":
        """me_matcher for me_service_create_matcher; callbacks run on the thread that flushes."""
        if self._cmatcher is not None:
            return self._cmatcher

        def match_cb(ctx, soa, n, fills, nf, results):
            try:
                s = soa.contents
                cols = [np.ctypeslib.as_array(C.cast(getattr(s, f), C.POINTER(t)), shape=(n,)).copy()
                        for f, t in (("seq", C.c_uint64), ("price_q4", C.c_int64), ("qty", C.c_int32),
                                     ("symbol", C.c_uint32), ("kind", C.c_uint8))]
                res, tape = self.match(Batch(*cols))
                res = np.ascontiguousarray(res)
                tape = np.ascontiguousarray(tape)
                self._keep = (res, tape)
                fills[0] = tape.ctypes.data if len(tape) else None
                nf[0] = len(tape)
                results[0] = res.ctypes.data
                return 0
            except SliceRefused:  # nothing applied: the service keeps the slice queued
                return _abi.ME_E_CAPACITY
            except Exception:  # a lost slice: the service fails loudly
                return _abi.ME_E_STATE

        def book_cb(ctx, symbol, depth, bids, bcap, nb, asks, acap, na, bl, al, nbl, nal):
            try:
                got = self.book_orders(symbol, depth)
                eb, ea, lb, la = got if got is not None else (np.zeros(0, BOOK_ENTRY_DTYPE),) * 2 + (
                    np.zeros(0, LEVEL_DTYPE),) * 2
                for arr, ptr_, cap, cnt in ((eb, bids, bcap, nb), (ea, asks, acap, na)):
                    if cnt:
                        cnt[0] = len(arr)
                    if ptr_ and cap:
                        k = min(cap, len(arr))
                        C.memmove(ptr_, arr.ctypes.data, k * arr.itemsize)
                for arr, ptr_, cnt in ((lb, bl, nbl), (la, al, nal)):
                    if cnt:
                        cnt[0] = len(arr)
                    if ptr_ and len(arr):
                        C.memmove(ptr_, arr.ctypes.data, len(arr) * arr.itemsize)
                return 0
            except Exception:
                return _abi.ME_E_STATE

        m = _abi.MeMatcher()
        m.ctx = None
        m.num_symbols = self.num_symbols
        m.max_batch = self.max_batch
        m.max_resting = self.max_resting
        m.match = _abi.MATCH_FN(match_cb)
        m.book = _abi.BOOK_FN(book_cb)
        self._cmatcher = m  # keeps the callbacks alive
        return m
