"""Sharded deployment — the Python view of include/me_cluster.h.

The cluster itself is C++ (csrc/me_cluster.cpp): one process per GPU, symbols hash-partitioned
(me_shard_of), RCCL over xGMI (or a TCP star: the CPU tests) only to scatter each slice's parts and to
bring tapes, results, books and level snapshots back to rank 0, where the SubmitOrder service runs
over ``Cluster.c_matcher()`` (me_cluster_matcher). This module creates it and exposes its entry points;
it moves no data itself.

``ShardOps`` adapts a Python book object to me_shard_ops (the CPU tests put the oracle behind it), and
``python_matcher`` a Python object to me_matcher (the single-book services the tests compare with).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import (BOOK_ENTRY_DTYPE, FILL_DTYPE, LEVEL_DTYPE, RESULT_DTYPE, MeClusterConfig, MeConfig, MeMatcher,
                   MeOrderSoa, MeShardOps, ptr)
from .engine import Batch, _view

TRANSPORTS = {"rccl": _abi.TRANSPORT_RCCL, "tcp": _abi.TRANSPORT_TCP}


class ClusterError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"cluster error {code}: {msg}")
        self.code = code


class SliceRefused(ClusterError):
    """A shard's admission control refused its part of a slice; no shard applied anything."""


def _batch_of(soa, n: int) -> Batch:
    s = soa.contents
    cols = [np.ctypeslib.as_array(C.cast(getattr(s, f), C.POINTER(t)), shape=(n,)).copy()
            for f, t in (("seq", C.c_uint64), ("price_q4", C.c_int64), ("qty", C.c_int32), ("symbol", C.c_uint32),
                         ("kind", C.c_uint8))]
    return Batch(*cols)


def _book_out(got, bids, bcap, nb, asks, acap, na, bl, al, nbl, nal):
    """me_book_orders' output contract from (bid entries, ask entries, bid levels, ask levels)."""
    eb, ea, lb, la = got
    for arr, p, cap, cnt in ((eb, bids, bcap, nb), (ea, asks, acap, na)):
        if cnt:
            cnt[0] = len(arr)
        if p and cap and len(arr):
            C.memmove(p, arr.ctypes.data, min(cap, len(arr)) * arr.itemsize)
    for arr, p, cnt in ((lb, bl, nbl), (la, al, nal)):
        if cnt:
            cnt[0] = len(arr)
        if p and len(arr):
            C.memmove(p, arr.ctypes.data, len(arr) * arr.itemsize)


def python_matcher(obj) -> MeMatcher:
    """me_matcher over a Python object with match(batch) -> (results, tape), book_orders(symbol, depth)
    -> (bid entries, ask entries, bid levels, ask levels), num_symbols, max_batch, max_resting. Test
    infrastructure (a single book standing in for a backend); the callbacks run on the flushing thread."""
    keep = {}

    def match_cb(ctx, soa, n, fills, nf, results):
        try:
            res, tape = obj.match(_batch_of(soa, n))
            res, tape = np.ascontiguousarray(res), np.ascontiguousarray(tape)
            keep["out"] = (res, tape)
            fills[0] = tape.ctypes.data if len(tape) else None
            nf[0] = len(tape)
            results[0] = res.ctypes.data
            return 0
        except SliceRefused:
            return _abi.ME_E_CAPACITY
        except Exception:
            return _abi.ME_E_STATE

    def book_cb(ctx, symbol, depth, *out):
        try:
            _book_out(obj.book_orders(symbol, depth), *out)
            return 0
        except Exception:
            return _abi.ME_E_STATE

    m = MeMatcher()
    m.ctx = None
    m.num_symbols, m.max_batch, m.max_resting = obj.num_symbols, obj.max_batch, obj.max_resting
    m.match = _abi.MATCH_FN(match_cb)
    m.book = _abi.BOOK_FN(book_cb)
    m._keep = (m.match, m.book, keep)  # the callbacks live as long as the struct
    return m


class ShardOps:
    """me_shard_ops over a Python book: admit(n_rest) -> bool (optional), match(batch) -> (results,
    tape), book_orders(local symbol, depth) -> (bid entries, ask entries, bid levels, ask levels),
    levels_all(depth) -> (levels [n, 2, depth], counts [n, 2])."""

    def __init__(self, book, max_resting: int):
        self.book = book
        self._out = None

        def admit_cb(ctx, n_rest, ok):
            try:
                ok[0] = 1 if (not hasattr(book, "admit") or book.admit(int(n_rest))) else 0
                return 0
            except Exception:
                return _abi.ME_E_STATE

        def match_cb(ctx, soa, n, fills, nf, results):
            try:
                res, tape = book.match(_batch_of(soa, n))
                self._out = (np.ascontiguousarray(res), np.ascontiguousarray(tape))
                fills[0] = self._out[1].ctypes.data if len(tape) else None
                nf[0] = len(tape)
                results[0] = self._out[0].ctypes.data
                return 0
            except Exception:
                return _abi.ME_E_STATE

        def book_cb(ctx, symbol, depth, *out):
            try:
                _book_out(book.book_orders(int(symbol), int(depth)), *out)
                return 0
            except Exception:
                return _abi.ME_E_STATE

        def levels_cb(ctx, depth, levels, counts):
            try:
                lv, cnt = book.levels_all(int(depth))
                lv, cnt = np.ascontiguousarray(lv, dtype=LEVEL_DTYPE), np.ascontiguousarray(cnt, dtype=np.uint32)
                C.memmove(levels, lv.ctypes.data, lv.nbytes)
                C.memmove(counts, cnt.ctypes.data, cnt.nbytes)
                return 0
            except Exception:
                return _abi.ME_E_STATE

        self.struct = MeShardOps(None, int(max_resting), _abi.ADMIT_FN(admit_cb), _abi.MATCH_FN(match_cb),
                                 _abi.BOOK_FN(book_cb), _abi.LEVELS_FN(levels_cb))


def shard_symbols(num_symbols: int, world: int, rank: int) -> np.ndarray:
    """Global symbol ids of rank's shard (local id = position), me_cluster_shard_symbols."""
    lib = _abi.load()
    n = lib.me_cluster_shard_symbols(num_symbols, world, rank, None, 0)
    out = np.zeros(max(n, 1), dtype=np.uint32)
    lib.me_cluster_shard_symbols(num_symbols, world, rank, ptr(out), n)
    return out[:n]


class Cluster:
    """One rank of the sharded deployment (me_cluster_create is collective: every rank constructs it).

    The shard is an engine built from (levels, base_prices[num_symbols global], max_resting, engine
    options) — or, with ``shard_ops``, a ShardOps. Rank 0 issues submit / collect / match / book_orders
    / snapshot / stop; the other ranks call serve()."""

    def __init__(self, rank: int, world: int, num_symbols: int, max_batch: int, transport: str = "rccl",
                 addr: str = "127.0.0.1", port: int = 29610, device: int = 0, levels: int = 128, base_prices=None,
                 max_resting: int = 1 << 20, shard_ops: ShardOps | None = None, timeout_ms: int = 60000,
                 seq_ring: int = 0, batches_per_launch: int = 0, far_levels: int = 0):
        self.lib = _abi.load()
        self.rank, self.world, self.num_symbols, self.max_batch = rank, world, num_symbols, max_batch
        self._addr = addr.encode()
        cfg = MeClusterConfig(rank, world, num_symbols, max_batch, TRANSPORTS[transport], device, self._addr, port,
                              timeout_ms)
        self._ops = shard_ops
        ecfg = None
        if shard_ops is None:
            self._base = np.ascontiguousarray(base_prices, dtype=np.int64)
            assert len(self._base) == num_symbols
            ecfg = MeConfig(device, num_symbols, levels, max_batch, max_resting, 0, seq_ring,
                            self._base.ctypes.data_as(C.POINTER(C.c_int64)), None, batches_per_launch, far_levels,
                            0, 0)
        self.h = self.lib.me_cluster_create(C.byref(cfg), C.byref(ecfg) if ecfg is not None else None,
                                            C.byref(shard_ops.struct) if shard_ops is not None else None)
        if not self.h:
            raise ClusterError(_abi.ME_E_STATE, self._err(None))
        self._cm = None

    def _err(self, h) -> str:
        buf = C.create_string_buffer(1024)
        self.lib.me_cluster_last_error(h, buf, 1024)
        return buf.value.decode(errors="replace")

    def _check(self, rc: int):
        if rc == _abi.ME_E_CAPACITY:
            raise SliceRefused(rc, self._err(self.h))
        if rc != _abi.ME_OK:
            raise ClusterError(rc, self._err(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.lib.me_cluster_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- ranks != 0
    def serve(self):
        self._check(self.lib.me_cluster_serve(self.h))

    # -- rank 0
    def stop(self):
        self._check(self.lib.me_cluster_stop(self.h))

    def submit(self, b: Batch) -> int:
        t = C.c_uint64(0)
        soa = b.soa()
        self._check(self.lib.me_cluster_submit(self.h, C.byref(soa), len(b), C.byref(t)))
        return t.value

    def collect(self, ticket: int, n: int, copy: bool = True):
        """(results[n], tape) of the oldest ticket: copies, or (copy=False) views valid until the next call."""
        f, r, nf = C.c_void_p(), C.c_void_p(), C.c_size_t(0)
        self._check(self.lib.me_cluster_collect(self.h, ticket, C.byref(f), C.byref(nf), C.byref(r)))
        res, tape = _view(r.value, n, RESULT_DTYPE), _view(f.value, nf.value, FILL_DTYPE)
        return (res.copy(), tape.copy()) if copy else (res, tape)

    def match(self, b: Batch):
        return self.collect(self.submit(b), len(b))

    def book_orders(self, symbol: int, depth: int):
        nb, na, nbl, nal = C.c_size_t(0), C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
        self._check(self.lib.me_cluster_book(self.h, symbol, depth, None, 0, C.byref(nb), None, 0, C.byref(na), None,
                                             None, C.byref(nbl), C.byref(nal)))
        eb, ea = np.zeros(max(nb.value, 1), BOOK_ENTRY_DTYPE), np.zeros(max(na.value, 1), BOOK_ENTRY_DTYPE)
        lb = np.zeros(max(depth, nbl.value, 1), LEVEL_DTYPE)
        la = np.zeros(max(depth, nal.value, 1), LEVEL_DTYPE)
        self._check(self.lib.me_cluster_book(self.h, symbol, depth, ptr(eb), len(eb), C.byref(nb), ptr(ea), len(ea),
                                             C.byref(na), ptr(lb), ptr(la), C.byref(nbl), C.byref(nal)))
        return eb[:nb.value], ea[:na.value], lb[:nbl.value if depth else 0], la[:nal.value if depth else 0]

    def snapshot(self, depth: int):
        """Top-`depth` levels of every global symbol: (levels [S, 2, depth], counts [S, 2])."""
        lv = np.zeros((self.num_symbols, 2, depth), dtype=LEVEL_DTYPE)
        cnt = np.zeros((self.num_symbols, 2), dtype=np.uint32)
        self._check(self.lib.me_cluster_snapshot(self.h, depth, ptr(lv), ptr(cnt)))
        return lv, cnt

    def c_matcher(self) -> MeMatcher:
        """me_cluster_matcher: the service on rank 0 is created over it (two slices in flight)."""
        if self._cm is None:
            m = MeMatcher()
            self._check(self.lib.me_cluster_matcher(self.h, C.byref(m)))
            self._cm = m
        return self._cm

    def stats(self) -> dict:
        s, b = C.c_uint64(0), C.c_uint64(0)
        self.lib.me_cluster_stats(self.h, C.byref(s), C.byref(b))
        return {"slices": s.value, "bytes": b.value}

    PHASES = ("split", "control", "scatter", "vote", "match", "collect", "gather", "merge", "split_count", "split_slot")

    def phases(self) -> dict:
        """Rank 0's seconds per protocol phase since create (me_cluster_phases)."""
        v = (C.c_double * len(self.PHASES))()
        self.lib.me_cluster_phases(self.h, v, len(self.PHASES))
        return dict(zip(self.PHASES, list(v)))
