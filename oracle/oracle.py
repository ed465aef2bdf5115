"""CPU ORACLE — TEST INFRASTRUCTURE ONLY.

ctypes view of oracle/build/liboracle.so (oracle_book.cpp). Only tests/, __graft_entry__.smoke()
and bench.py's cpu_baseline leg may import this module, and only as the checker / CPU baseline.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

from matching_engine_amd._abi import BOOK_ENTRY_DTYPE, FILL_DTYPE, LEVEL_DTYPE, RESULT_DTYPE

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(_HERE, "build", "liboracle.so")
REF_PRICE = os.path.join(_HERE, "_ref", "ref_price")
_lib = None


def build(target="lib"):
    """`lib` = the oracle library; `ref` = oracle/_ref (container only: needs /root/reference)."""
    subprocess.run(["make", "-C", _HERE, target], check=True, stdout=subprocess.DEVNULL)


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        P, SZ = C.c_void_p, C.c_size_t
        lib.orc_create.restype = P
        lib.orc_create.argtypes = [C.c_uint32]
        lib.orc_destroy.argtypes = [P]
        lib.orc_resting.restype = C.c_uint64
        lib.orc_resting.argtypes = [P]
        lib.orc_submit.restype = C.c_int
        lib.orc_submit.argtypes = [P, SZ, P, P, P, P, P, P, P, P, SZ, C.POINTER(SZ)]
        lib.orc_dump.restype = SZ
        lib.orc_dump.argtypes = [P, C.c_uint32, P, SZ]
        lib.orc_snapshot.restype = C.c_int
        lib.orc_snapshot.argtypes = [P, C.c_uint32, P, P, SZ, C.POINTER(SZ), C.POINTER(SZ)]
        lib.orc_service_create.restype = P
        lib.orc_service_create.argtypes = [C.c_uint64]
        lib.orc_service_destroy.argtypes = [P]
        lib.orc_service_submit.restype = C.c_int
        lib.orc_service_submit.argtypes = [P, C.c_char_p, C.c_int32, C.c_int32, C.c_int64, C.c_int32, C.c_int32,
                                           C.c_char_p, SZ, C.POINTER(C.c_int), C.c_char_p, SZ,
                                           C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int64),
                                           C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int64),
                                           C.POINTER(C.c_int32)]
        lib.orc_run_sharded.restype = C.c_double
        lib.orc_run_sharded.argtypes = [C.c_uint32, C.c_uint32, P, P, P, P, P, P, P, P, P]
        lib.ref_submit_run.restype = C.c_longlong
        lib.ref_submit_run.argtypes = [C.c_char_p, C.c_char_p, C.c_char_p, SZ, P, P, P, P, P, C.c_int, P]
        _lib = lib
    return _lib


def _p(a):
    return None if a is None else a.ctypes.data


class OracleBook:
    """Unbounded scalar price-time books for num_symbols symbols: no price window, no seq cap (the
    engine's fixed-depth windows and seq ring are implementation details it must hide)."""

    def __init__(self, num_symbols, symbol_ids=None):
        self.lib = load()
        self.ids = None if symbol_ids is None else np.ascontiguousarray(symbol_ids, dtype=np.uint32)
        self.h = self.lib.orc_create(num_symbols)

    def close(self):
        if self.h:
            self.lib.orc_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def submit(self, b, fills_cap=None):
        """Process a batch; returns (results, fills)."""
        n = len(b)
        res = np.zeros(n, dtype=RESULT_DTYPE)
        # fills of one batch <= resting makers + 2n, so this never truncates
        cap = fills_cap if fills_cap is not None else self.resting() + 2 * n + 16
        fills = np.zeros(cap, dtype=FILL_DTYPE)
        nf = C.c_size_t(0)
        rc = self.lib.orc_submit(self.h, n, _p(b.seq), _p(b.price_q4), _p(b.qty), _p(b.symbol), _p(b.kind),
                                 _p(self.ids), _p(res), _p(fills), cap, C.byref(nf))
        if rc != 0:
            raise RuntimeError("oracle tape capacity too small; pass fills_cap >= resting + 2n")
        return res, fills[: nf.value].copy()

    def resting(self):
        return int(self.lib.orc_resting(self.h))

    def dump(self, symbol):
        n = self.lib.orc_dump(self.h, symbol, None, 0)
        out = np.zeros(n, dtype=BOOK_ENTRY_DTYPE)
        self.lib.orc_dump(self.h, symbol, _p(out), n)
        return out

    def snapshot(self, symbol, depth=10):
        bids = np.zeros(depth, dtype=LEVEL_DTYPE)
        asks = np.zeros(depth, dtype=LEVEL_DTYPE)
        nb, na = C.c_size_t(0), C.c_size_t(0)
        self.lib.orc_snapshot(self.h, symbol, _p(bids), _p(asks), depth, C.byref(nb), C.byref(na))
        return bids[: nb.value], asks[: na.value]


def run_sharded(books, parts, nwarm=0):
    """The native CPU baseline (orc_run_sharded): books[r] (OracleBook) runs the batches parts[r] on its
    own std::thread, no Python inside the timed region; each thread's first nwarm batches run untimed
    before the clock starts. Returns (wall seconds of the rest, their fills)."""
    T = len(books)
    lib = load()
    cols = {f: [] for f in ("seq", "price_q4", "qty", "symbol", "kind")}
    nb = np.array([len(p) for p in parts], dtype=np.uint32)
    offs = []
    for p in parts:
        assert p, "every thread needs its list of batches (empty batches allowed)"
        o = np.zeros(len(p) + 1, dtype=np.uint64)
        o[1:] = np.cumsum([len(b) for b in p])
        offs.append(o)
        for f in cols:  # (+ one pad element: an empty part still has a valid pointer)
            a = np.concatenate([getattr(b, f) for b in p])
            cols[f].append(np.ascontiguousarray(np.concatenate([a, np.zeros(1, a.dtype)])))

    def ptrs(arrs):
        return (C.c_void_p * T)(*[a.ctypes.data for a in arrs])

    hb = (C.c_void_p * T)(*[b.h for b in books])
    fills = np.zeros(T, dtype=np.uint64)
    w = lib.orc_run_sharded(T, nwarm, hb, nb.ctypes.data, ptrs(offs), ptrs(cols["seq"]), ptrs(cols["price_q4"]),
                            ptrs(cols["qty"]), ptrs(cols["symbol"]), ptrs(cols["kind"]), fills.ctypes.data)
    return float(w), int(fills.sum())


class OracleService:
    """SubmitOrder restatement (src/server/matching_engine_service.cpp:41-121), no gRPC/SQLite."""

    def __init__(self, next_id=1):
        self.lib = load()
        self.h = self.lib.orc_service_create(next_id)

    def __del__(self):
        try:
            self.lib.orc_service_destroy(self.h)
        except Exception:
            pass

    def submit(self, symbol, order_type, side, price, scale, quantity):
        oid = C.create_string_buffer(64)
        err = C.create_string_buffer(128)
        ok, st, pers = C.c_int(0), C.c_int(0), C.c_int(0)
        rp, rot, rst, rrem, rsd = C.c_int64(0), C.c_int32(0), C.c_int32(0), C.c_int64(0), C.c_int32(0)
        self.lib.orc_service_submit(self.h, symbol.encode(), order_type, side, price, scale, quantity, oid, 64,
                                    C.byref(ok), err, 128, C.byref(st), C.byref(pers), C.byref(rp), C.byref(rot),
                                    C.byref(rst), C.byref(rrem), C.byref(rsd))
        row = None
        if pers.value:
            row = dict(price=rp.value, order_type=rot.value, status=rst.value, remaining_quantity=rrem.value,
                       side=rsd.value, quantity=quantity)
        return dict(order_id=oid.value.decode(), success=bool(ok.value), error_message=err.value.decode(),
                    grpc_status=st.value, row=row)


def ref_normalize_many(pairs):
    """Run the REFERENCE's normalize_to_q4 (oracle/_ref/ref_price, compiled from
    /root/reference/include/domain/price.hpp) on (price, scale) pairs. Container-only."""
    if not os.path.exists(REF_PRICE):
        build("ref")
    if not os.path.exists(REF_PRICE):
        raise FileNotFoundError("oracle/_ref/ref_price not built (reference tree absent)")
    inp = "".join(f"{p} {s}\n" for p, s in pairs)
    out = subprocess.run([REF_PRICE], input=inp, capture_output=True, text=True, check=True).stdout
    res = []
    for line in out.strip().splitlines():
        parts = line.split()
        if parts[2] == "EXC":
            res.append(("EXC", parts[3], " ".join(parts[4:])))
        else:
            res.append(int(parts[2]))
    return res


def ref_submit_run(db_path, client_id, symbol, order_type, side, price, scale, quantity, log_fd):
    """The reference's per-order SubmitOrder + insert_new_order path (oracle/ref_submit.cpp), one SQLite
    transaction per order, logs to log_fd. Returns (rows written, ok[n])."""
    n = len(order_type)
    arrs = [np.ascontiguousarray(a, dtype=t) for a, t in
            ((order_type, np.int32), (side, np.int32), (price, np.int64), (scale, np.int32), (quantity, np.int32))]
    ok = np.zeros(n, dtype=np.uint8)
    rows = load().ref_submit_run(db_path.encode(), client_id.encode(), symbol.encode(), n,
                                 *[a.ctypes.data for a in arrs], log_fd, ok.ctypes.data)
    if rows < 0:
        raise RuntimeError("ref_submit_run: SQLite unavailable")
    return rows, ok
