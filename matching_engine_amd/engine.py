"""Host-side mirror of the batched matching core (C-ABI include/me_engine.h).

``Engine`` is one shard (one GPU): HBM-resident books for ``num_symbols`` local symbols, driven
batch by batch. Every call goes through libme_engine.so; nothing here computes a match.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi
from ._abi import BOOK_ENTRY_DTYPE, FILL_DTYPE, LEVEL_DTYPE, RESULT_DTYPE, MeConfig, MeGenParams, MeOrderSoa, ptr


class EngineError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"me error {code}: {msg}")
        self.code = code


def _check(lib, handle, rc: int) -> None:
    if rc != _abi.ME_OK:
        buf = C.create_string_buffer(1024)
        lib.me_last_error(handle, buf, 1024)
        raise EngineError(rc, buf.value.decode(errors="replace"))


def _view(addr, n: int, dtype) -> np.ndarray:
    """numpy view of n records at a C address (no copy)."""
    if not n:
        return np.zeros(0, dtype=dtype)
    buf = (C.c_char * (n * dtype.itemsize)).from_address(addr)
    return np.frombuffer(buf, dtype=dtype, count=n)


def normalize_to_q4(price: int, scale: int) -> int:
    """include/domain/price.hpp:15-29 through the product library; raises like the reference."""
    lib = _abi.load()
    out = C.c_int64(0)
    rc = lib.me_normalize_to_q4(int(price), int(scale), C.byref(out))
    if rc == 1:
        raise ValueError("scale out of range")
    if rc == 2:
        raise OverflowError("overflow")
    if rc == 3:
        raise OverflowError("underflow")
    return out.value


@dataclass
class Batch:
    """One batch in SoA form (host numpy arrays), ascending seq."""

    seq: np.ndarray
    price_q4: np.ndarray
    qty: np.ndarray
    symbol: np.ndarray
    kind: np.ndarray

    def __post_init__(self):
        self.seq = np.ascontiguousarray(self.seq, dtype=np.uint64)
        self.price_q4 = np.ascontiguousarray(self.price_q4, dtype=np.int64)
        self.qty = np.ascontiguousarray(self.qty, dtype=np.int32)
        self.symbol = np.ascontiguousarray(self.symbol, dtype=np.uint32)
        self.kind = np.ascontiguousarray(self.kind, dtype=np.uint8)
        n = len(self.seq)
        assert all(len(a) == n for a in (self.price_q4, self.qty, self.symbol, self.kind))

    def __len__(self) -> int:
        return len(self.seq)

    def take(self, idx) -> "Batch":
        return Batch(self.seq[idx], self.price_q4[idx], self.qty[idx], self.symbol[idx], self.kind[idx])

    def soa(self) -> MeOrderSoa:
        return MeOrderSoa(ptr(self.seq), ptr(self.price_q4), ptr(self.qty), ptr(self.symbol), ptr(self.kind))


class DeviceBatch:
    """A batch copied once into HBM (me_device_alloc), for device-resident submission."""

    def __init__(self, engine: "Engine", b: Batch):
        self.engine = engine
        self.n = len(b)
        self.ptrs = []
        for a in (b.seq, b.price_q4, b.qty, b.symbol, b.kind):
            p = C.c_void_p()
            _check(engine.lib, engine.h, engine.lib.me_device_alloc(engine.h, max(a.nbytes, 1), C.byref(p)))
            if a.nbytes:
                _check(engine.lib, engine.h, engine.lib.me_memcpy_h2d(engine.h, p, ptr(a), a.nbytes))
            self.ptrs.append(p.value)
        self._soa = MeOrderSoa(*self.ptrs)

    def free(self):
        for p in self.ptrs:
            self.engine.lib.me_device_free(self.engine.h, p)
        self.ptrs = []


class Engine:
    """One shard of HBM-resident books (include/me_engine.h me_create ... me_destroy).

    `levels` is the depth of each symbol's on-chip window; `base_prices` only its initial position:
    any int64 price is accepted (far levels + re-centring) and any u64 seq (the seq ring, `seq_ring`
    entries, 0 = 2^28)."""

    def __init__(
        self,
        num_symbols: int,
        levels: int,
        base_prices,
        max_batch: int,
        max_resting: int,
        seq_ring: int = 0,
        max_chunks: int = 0,
        device: int = 0,
        symbol_ids=None,
        batches_per_launch: int = 0,
        far_levels: int = 0,
        host_slots: int = 0,
        host_tape_cap: int = 0,
    ):
        self.lib = _abi.load()
        self.num_symbols = int(num_symbols)
        self.levels = int(levels)
        self._base = np.ascontiguousarray(base_prices, dtype=np.int64)
        assert len(self._base) == num_symbols
        self._ids = None if symbol_ids is None else np.ascontiguousarray(symbol_ids, dtype=np.uint32)
        cfg = MeConfig(
            device,
            num_symbols,
            levels,
            max_batch,
            max_resting,
            max_chunks,
            seq_ring,
            self._base.ctypes.data_as(C.POINTER(C.c_int64)),
            None if self._ids is None else self._ids.ctypes.data_as(C.POINTER(C.c_uint32)),
            batches_per_launch,
            far_levels,
            host_slots,
            host_tape_cap,
        )
        self.max_batch = int(max_batch)
        h = self.lib.me_create(C.byref(cfg))
        if not h:
            buf = C.create_string_buffer(1024)
            self.lib.me_last_error(None, buf, 1024)
            raise EngineError(_abi.ME_E_HIP, buf.value.decode(errors="replace"))
        self.h = h

    # -- lifecycle
    def close(self):
        if getattr(self, "h", None):
            self.lib.me_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # -- batches
    def fill_bound(self, n: int) -> int:
        return int(self.lib.me_fill_bound(self.h, n))

    def submit_batch(self, b: Batch, want_fills: bool = True):
        """Host batch -> (results[n] RESULT_DTYPE, fills[k] FILL_DTYPE), synchronous."""
        n = len(b)
        res = np.zeros(n, dtype=RESULT_DTYPE)
        cap = self.fill_bound(n) if want_fills else 0
        fills = np.zeros(cap, dtype=FILL_DTYPE) if want_fills else None
        nf = C.c_size_t(0)
        soa = b.soa()
        rc = self.lib.me_submit_batch(
            self.h, C.byref(soa), n, ptr(fills) if want_fills else None, cap, C.byref(nf), ptr(res)
        )
        _check(self.lib, self.h, rc)
        return res, (fills[: nf.value].copy() if want_fills else nf.value)

    # -- pipelined host batches (me_submit_host / me_collect)
    def submit_host(self, b: Batch) -> int:
        """Enqueue a host batch (staged into the next pinned slot unless it already lives there, see
        host_inputs); returns its ticket at once."""
        t = C.c_uint64(0)
        soa = b.soa()
        _check(self.lib, self.h, self.lib.me_submit_host(self.h, C.byref(soa), len(b), C.byref(t)))
        return t.value

    def collect(self, ticket: int, copy: bool = True):
        """(results[n], fills[k]) of a ticket. copy=False returns views of the slot's pinned memory, valid
        until the next collect, or until a submit_host / host_inputs call that finds every other slot busy
        and takes the held slot back (me_collect's contract, include/me_engine.h)."""
        fp, rp = C.c_void_p(), C.c_void_p()
        nf, nr = C.c_size_t(0), C.c_size_t(0)
        _check(self.lib, self.h,
               self.lib.me_collect(self.h, ticket, C.byref(fp), C.byref(nf), C.byref(rp), C.byref(nr)))
        res = _view(rp.value, nr.value, RESULT_DTYPE)
        fills = _view(fp.value, nf.value, FILL_DTYPE)
        return (res.copy(), fills.copy()) if copy else (res, fills)

    def host_inputs(self, n: int) -> Batch:
        """Writable numpy views of the pinned arrays the next submit_host takes for an n-record batch
        (fill them in place, then submit_host the returned Batch: no staging copy)."""
        w = _abi.MeOrderSoaW()
        _check(self.lib, self.h, self.lib.me_host_inputs(self.h, n, C.byref(w)))
        arrs = [_view(getattr(w, f), n, np.dtype(t)) for f, t in
                (("seq", "<u8"), ("price_q4", "<i8"), ("qty", "<i4"), ("symbol", "<u4"), ("kind", "u1"))]
        return Batch(*arrs)

    def host_reserve(self, nslots: int = 0):
        """Allocate host slots now (0 = all) rather than on first use."""
        _check(self.lib, self.h, self.lib.me_host_reserve(self.h, nslots))

    def config(self) -> dict:
        cfg = MeConfig()
        _check(self.lib, self.h, self.lib.me_get_config(self.h, C.byref(cfg)))
        return {f: getattr(cfg, f) for f, _ in MeConfig._fields_ if f not in ("base_price", "symbol_ids")}

    def upload(self, b: Batch) -> DeviceBatch:
        return DeviceBatch(self, b)

    def submit_device(self, db: DeviceBatch):
        _check(self.lib, self.h, self.lib.me_submit_batch_device(self.h, C.byref(db._soa), db.n))

    def sync(self):
        _check(self.lib, self.h, self.lib.me_sync(self.h))

    def fetch_outputs(self, n: int):
        res = np.zeros(n, dtype=RESULT_DTYPE)
        nf = C.c_size_t(0)
        _check(self.lib, self.h, self.lib.me_fetch_outputs(self.h, None, 0, C.byref(nf), ptr(res), n))
        fills = np.zeros(nf.value, dtype=FILL_DTYPE)
        _check(self.lib, self.h, self.lib.me_fetch_outputs(self.h, ptr(fills), nf.value, C.byref(nf), None, 0))
        return res, fills

    def last_group_size(self) -> int:
        return int(self.lib.me_last_group_size(self.h))

    def fetch_group_outputs(self, k: int, n: int):
        """Outputs of the k-th batch (n records) of the most recent launch group."""
        res = np.zeros(n, dtype=RESULT_DTYPE)
        nf = C.c_size_t(0)
        _check(self.lib, self.h, self.lib.me_fetch_group_outputs(self.h, k, None, 0, C.byref(nf), ptr(res), n))
        fills = np.zeros(nf.value, dtype=FILL_DTYPE)
        _check(self.lib, self.h, self.lib.me_fetch_group_outputs(self.h, k, ptr(fills), nf.value, C.byref(nf),
                                                                 None, 0))
        return res, fills

    def copy_tape_device(self, dst_ptr: int, cap_fills: int) -> int:
        """Last batch's tape -> device buffer at dst_ptr (engine stream); returns its length."""
        nf = C.c_size_t(0)
        _check(self.lib, self.h, self.lib.me_copy_tape_device(self.h, dst_ptr, cap_fills, C.byref(nf)))
        return nf.value

    def copy_results_device(self, dst_ptr: int, n: int):
        """Last batch's n per-record results -> device buffer at dst_ptr (engine stream)."""
        _check(self.lib, self.h, self.lib.me_copy_results_device(self.h, dst_ptr, n))

    def set_stream(self, stream_handle: int | None):
        _check(self.lib, self.h, self.lib.me_set_stream(self.h, stream_handle))

    # -- book inspection
    def snapshot(self, symbol: int, depth: int = 10):
        bids = np.zeros(depth, dtype=LEVEL_DTYPE)
        asks = np.zeros(depth, dtype=LEVEL_DTYPE)
        nb, na = C.c_size_t(0), C.c_size_t(0)
        rc = self.lib.me_book_snapshot(self.h, symbol, ptr(bids), ptr(asks), depth, C.byref(nb), C.byref(na))
        _check(self.lib, self.h, rc)
        return bids[: nb.value], asks[: na.value]

    def book_orders(self, symbol: int, depth: int):
        """GetOrderBook per order from one device snapshot launch: (bids, asks) BOOK_ENTRY_DTYPE in
        priority order over the top `depth` levels per side, and (bid_levels, ask_levels)."""
        nb, na, nlb, nla = C.c_size_t(0), C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
        lb = np.zeros(max(depth, 1), dtype=LEVEL_DTYPE)
        la = np.zeros(max(depth, 1), dtype=LEVEL_DTYPE)
        _check(self.lib, self.h, self.lib.me_book_orders(self.h, symbol, depth, None, 0, C.byref(nb), None, 0,
                                                         C.byref(na), ptr(lb), ptr(la), C.byref(nlb), C.byref(nla)))
        bids = np.zeros(nb.value, dtype=BOOK_ENTRY_DTYPE)
        asks = np.zeros(na.value, dtype=BOOK_ENTRY_DTYPE)
        _check(self.lib, self.h, self.lib.me_book_orders(self.h, symbol, depth, ptr(bids), len(bids), C.byref(nb),
                                                         ptr(asks), len(asks), C.byref(na), None, None, None, None))
        return bids, asks, lb[: nlb.value], la[: nla.value]

    def levels_all(self, depth: int):
        """Top `depth` levels per side of every symbol (one launch): (levels[S, 2, depth], counts[S, 2])."""
        lv = np.zeros(self.num_symbols * 2 * depth, dtype=LEVEL_DTYPE)
        cnt = np.zeros(self.num_symbols * 2, dtype=np.uint32)
        _check(self.lib, self.h, self.lib.me_book_levels_all(self.h, depth, ptr(lv), ptr(cnt)))
        return lv.reshape(self.num_symbols, 2, depth), cnt.reshape(self.num_symbols, 2)

    def dump(self, symbol: int) -> np.ndarray:
        n = C.c_size_t(0)
        _check(self.lib, self.h, self.lib.me_book_dump(self.h, symbol, None, 0, C.byref(n)))
        out = np.zeros(n.value, dtype=BOOK_ENTRY_DTYPE)
        _check(self.lib, self.h, self.lib.me_book_dump(self.h, symbol, ptr(out), n.value, C.byref(n)))
        return out

    def resting_count(self) -> int:
        v = C.c_uint64(0)
        _check(self.lib, self.h, self.lib.me_resting_count(self.h, C.byref(v)))
        return v.value

    def stats(self) -> dict:
        """Device event counters since creation (me_stats_read)."""
        h = C.c_uint64(0)
        _check(self.lib, self.h, self.lib.me_stats_read(self.h, C.byref(h)))
        return {"handoffs": h.value}

    def far_stats(self) -> dict:
        """The far arena (me_far_stats): sides moved to a larger region, collections, entries in use."""
        m, g, u = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        _check(self.lib, self.h, self.lib.me_far_stats(self.h, C.byref(m), C.byref(g), C.byref(u)))
        return {"moves": m.value, "collections": g.value, "arena_used": u.value}

    def chunk_stats(self) -> dict:
        """The FIFO chunk pool (me_chunk_stats): reclamations, chunk ids ever handed out, pool size."""
        r, h, p = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        _check(self.lib, self.h, self.lib.me_chunk_stats(self.h, C.byref(r), C.byref(h), C.byref(p)))
        return {"reclaims": r.value, "high_water": h.value, "pool": p.value}

    def paths(self) -> dict:
        """The matching paths running now (me_paths_read): grouped launches / hot symbols through the
        aggregate path (me_agg.hip)."""
        f = C.c_uint32(0)
        _check(self.lib, self.h, self.lib.me_paths_read(self.h, C.byref(f)))
        return {"grouped_agg": bool(f.value & 1), "hot_agg": bool(f.value & 2), "grouped_cancels": bool(f.value & 4)}

    def admits(self, b: Batch) -> bool:
        """Would submit_batch(b) be admitted now (me_admission_check)? Nothing is enqueued."""
        n_rest = int(np.count_nonzero((b.kind & 0x0C) == 0))
        ok = C.c_int(0)
        _check(self.lib, self.h, self.lib.me_admission_check(self.h, n_rest, C.byref(ok)))
        return bool(ok.value)

    def admission(self) -> dict:
        """Admission control (me_admission_read): device resting count after all enqueued work, the
        host's current bound, and how many submits had to take an exact count."""
        r, b, x = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        _check(self.lib, self.h, self.lib.me_admission_read(self.h, C.byref(r), C.byref(b), C.byref(x)))
        return {"resting": r.value, "bound": b.value, "exact_counts": x.value}

    # -- timing
    def timing_enable(self, period: int = 1):
        """HIP events on every `period`-th match launch (True = every launch, 0/False = off)."""
        _check(self.lib, self.h, self.lib.me_timing_enable(self.h, int(period)))

    def timing_read(self):
        m, p = C.c_double(0), C.c_double(0)
        k, f, o = C.c_uint64(0), C.c_uint64(0), C.c_uint64(0)
        rc = self.lib.me_timing_read(self.h, C.byref(m), C.byref(p), C.byref(k), C.byref(f), C.byref(o))
        _check(self.lib, self.h, rc)
        return {"match_ms": m.value, "pipeline_ms": p.value, "launches": k.value, "fills": f.value,
                "orders": o.value}


# ---------------------------------------------------------------------------------------------
# Synthetic streams (SURVEY.md §8(d) configurations)
@dataclass
class StreamConfig:
    config: int
    seed: int
    num_symbols: int
    levels: int
    spread_ticks: int = 32
    max_qty: int = 100
    market_pct: int = 20
    cancel_pct: int = 0
    zipf_s: float = 0.0
    market_qty_mult: int = 0
    batch: int = 65536
    batches: int = 1024
    seed_levels_per_side: int = 0
    seq_start: int = 0       # first seq (0 = 1); > 2^33 exercises OIDs far beyond any fixed table
    drift_step: int = 0      # > 0: each symbol's mid trends drift_step ticks every drift_every records
    drift_every: int = 0
    far_pct: int = 0         # % of LIMITs priced U[L, 64L] ticks away from the mid (outside the window)


def preset(config: int, **over) -> StreamConfig:
    """The five benchmark configurations of SURVEY.md §8(d) (override any field for small tests)."""
    base = {
        1: dict(config=1, seed=1, num_symbols=1, levels=128, batch=62500, batches=16),  # 1M orders on "SYM"
        2: dict(config=2, seed=2, num_symbols=1024, levels=128, batch=65536, batches=1024),
        3: dict(config=3, seed=3, num_symbols=100_000, levels=128, batch=1 << 20, batches=128),
        4: dict(config=4, seed=4, num_symbols=100_000, levels=32768, spread_ticks=5000, zipf_s=1.1,
                seed_levels_per_side=10_000, batch=65536, batches=256),
        5: dict(config=5, seed=5, num_symbols=1024, levels=128, cancel_pct=60, market_pct=15,
                market_qty_mult=20, batch=65536, batches=1024),
    }[config]
    base.update(over)
    return StreamConfig(**base)


class Stream:
    """Deterministic global order stream (me_gen_*), seq = 1, 2, ... across batches."""

    def __init__(self, sc: StreamConfig):
        self.lib = _abi.load()
        self.sc = sc
        p = MeGenParams(sc.config, sc.seed, sc.num_symbols, sc.levels, sc.spread_ticks, sc.max_qty,
                        sc.market_pct, sc.cancel_pct, float(sc.zipf_s), sc.market_qty_mult, sc.seq_start,
                        sc.drift_step, sc.drift_every, sc.far_pct)
        self.g = self.lib.me_gen_create(C.byref(p))
        if not self.g:
            raise ValueError(f"invalid stream config {sc}")

    def close(self):
        if self.g:
            self.lib.me_gen_destroy(self.g)
            self.g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def base_prices(self) -> np.ndarray:
        out = np.zeros(self.sc.num_symbols, dtype=np.int64)
        self.lib.me_gen_base_prices(self.g, ptr(out))
        return out

    def next(self, n: int) -> Batch:
        a = [np.zeros(n, dtype=t) for t in (np.uint64, np.int64, np.int32, np.uint32, np.uint8)]
        self.lib.me_gen_next(self.g, n, *[ptr(x) for x in a])
        return Batch(*a)

    def seed_books(self, symbols, per_side: int) -> Batch:
        """Config 4 pre-seed: per_side resting orders per side for every symbol in `symbols`."""
        parts = []
        for s in symbols:
            m = 2 * per_side
            a = [np.zeros(m, dtype=t) for t in (np.uint64, np.int64, np.int32, np.uint8)]
            rc = self.lib.me_gen_seed_book(self.g, int(s), per_side, *[ptr(x) for x in a])
            if rc:
                raise ValueError("seed_book failed")
            parts.append(Batch(a[0], a[1], a[2], np.full(m, s, dtype=np.uint32), a[3]))
        return Batch(*[np.concatenate([getattr(p, f) for p in parts]) for f in
                       ("seq", "price_q4", "qty", "symbol", "kind")])


def shard_of(symbol: int, shards: int) -> int:
    return int(_abi.load().me_shard_of(symbol, shards))


def shard_table(num_symbols: int, shards: int):
    """global symbol -> (shard, local id); per shard the global ids in local-id order."""
    lib = _abi.load()
    shard = np.array([lib.me_shard_of(s, shards) for s in range(num_symbols)], dtype=np.uint32)
    local = np.zeros(num_symbols, dtype=np.uint32)
    members = []
    for r in range(shards):
        ids = np.nonzero(shard == r)[0].astype(np.uint32)
        local[ids] = np.arange(len(ids), dtype=np.uint32)
        members.append(ids)
    return shard, local, members
