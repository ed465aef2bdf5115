"""MatchingEngineService — Python view of include/me_service.h, the SubmitOrder drop-in
(src/server/matching_engine_service.cpp:41-121 re-hosted on the batched GPU core)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import (FILL_DTYPE, LEVEL_DTYPE, RESULT_DTYPE, MeBookOrder, MeCancelRequest, MeOrderRequest,
                   MeOrderResponse, MeMarketData, MeOrderUpdate, ptr)


class ServiceError(RuntimeError):
    pass


class MatchingEngineService:
    """SubmitOrder / GetOrderBook over one engine shard; SQLite persistence when db_path is given."""

    def __init__(self, engine, symbols, db_path=None, matcher=None):
        """engine: the Engine the slices match on; or matcher: an object with c_matcher() -> MeMatcher —
        a cluster.Cluster (rank 0 of a sharded deployment, me_cluster_matcher) or a Python book behind
        cluster.python_matcher (tests) — for me_service_create_matcher."""
        self.lib = _abi.load()
        self.engine = engine
        self.matcher = matcher
        self.symbols = list(symbols)
        arr = (C.c_char_p * max(len(self.symbols), 1))(*[s.encode() for s in self.symbols])
        self._arr = arr
        if matcher is not None:
            self._cm = matcher.c_matcher()
            self.h = self.lib.me_service_create_matcher(C.byref(self._cm), arr, len(self.symbols),
                                                        db_path.encode() if db_path else None)
            if not self.h:
                raise ServiceError("me_service_create_matcher refused the matcher")
        else:
            self.h = self.lib.me_service_create(engine.h if engine is not None else None, arr, len(self.symbols),
                                                db_path.encode() if db_path else None)
        err = self.last_error()
        if db_path and err:
            raise ServiceError(err)

    def close(self):
        if getattr(self, "h", None):
            self.lib.me_service_destroy(self.h)
            self.h = None

    def start(self, interval_us: int = 1000, slice_orders: int = 0):
        """Background flusher: slices close at slice_orders records or interval_us age and are matched
        and persisted without a caller (errors: last_error())."""
        rc = self.lib.me_service_start(self.h, interval_us, slice_orders)
        if rc != 0:
            raise ServiceError(f"start failed ({rc}): {self.last_error()}")

    def stop(self):
        self.lib.me_service_stop(self.h)

    @property
    def unpersisted(self) -> int:
        """Matched records whose SQLite transaction has not committed yet."""
        return int(self.lib.me_service_unpersisted(self.h))

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def last_error(self) -> str:
        buf = C.create_string_buffer(1024)
        self.lib.me_service_last_error(self.h, buf, 1024)
        return buf.value.decode(errors="replace")

    def submit_order(self, client_id, symbol, order_type, side, price, scale, quantity) -> dict:
        """OrderRequest -> OrderResponse fields + grpc status (0 OK, 2 UNKNOWN)."""
        req = MeOrderRequest(client_id.encode(), symbol.encode(), order_type, side, price, scale, quantity)
        resp = MeOrderResponse()
        self.lib.me_service_submit_order(self.h, C.byref(req), C.byref(resp))
        return {"order_id": resp.order_id.decode(), "success": bool(resp.success),
                "error_message": resp.error_message.decode(), "grpc_status": resp.grpc_status}

    def cancel_order(self, client_id, symbol, order_id) -> dict:
        """CancelOrder (build extension, me_service.h): queue a cancel of a resting order; the outcome
        arrives as an OrderUpdate after the flush."""
        req = MeCancelRequest(client_id.encode(), symbol.encode(), order_id.encode())
        resp = MeOrderResponse()
        self.lib.me_service_cancel_order(self.h, C.byref(req), C.byref(resp))
        return {"order_id": resp.order_id.decode(), "success": bool(resp.success),
                "error_message": resp.error_message.decode(), "grpc_status": resp.grpc_status}

    def order_updates(self, client_id=None, cap=1 << 16) -> list:
        """StreamOrderUpdates (proto:34,71-91): drain the queued OrderUpdate events (one client, or all)."""
        out = []
        buf = (MeOrderUpdate * cap)()
        while True:
            n = C.c_size_t(0)
            self.lib.me_service_updates(self.h, client_id.encode() if client_id else None, buf, cap, C.byref(n))
            for u in buf[: n.value]:
                out.append({"order_id": u.order_id.decode(), "client_id": u.client_id.decode(),
                            "symbol": u.symbol.decode(), "status": u.status, "fill_price": u.fill_price,
                            "scale": u.scale, "fill_quantity": u.fill_quantity,
                            "remaining_quantity": u.remaining_quantity})
            if n.value < cap:
                return out

    @property
    def pending(self) -> int:
        return int(self.lib.me_service_pending(self.h))

    @property
    def next_oid(self) -> int:
        return int(self.lib.me_service_next_oid(self.h))

    def flush(self, outputs: bool = True):
        """Match + persist every slice submitted so far -> (seq[n], results[n], fills[k]) of the records
        this call matched (outputs=False: nothing copied out, returns None)."""
        if not outputs:
            rc = self.lib.me_service_flush(self.h, None, 0, None, None, None, 0, None)
            if rc != 0:
                raise ServiceError(f"flush failed ({rc}): {self.last_error()}")
            return None
        n = self.pending
        res = np.zeros(max(n, 1), dtype=RESULT_DTYPE)
        seq = np.zeros(max(n, 1), dtype=np.uint64)
        if self.engine is not None:
            cap = self.engine.fill_bound(n) + 1
        else:
            cap = (self._cm.max_resting + 2 * n + 1) if self.matcher is not None else 1
        fills = np.zeros(cap, dtype=FILL_DTYPE)
        nf, nr = C.c_size_t(0), C.c_size_t(0)
        rc = self.lib.me_service_flush(self.h, ptr(fills), cap, C.byref(nf), ptr(res), ptr(seq), len(res),
                                       C.byref(nr))
        if rc != 0:
            raise ServiceError(f"flush failed ({rc}): {self.last_error()}")
        return seq[: nr.value].copy(), res[: nr.value].copy(), fills[: nf.value].copy()

    @property
    def updates_dropped(self) -> int:
        return int(self.lib.me_service_updates_dropped(self.h))

    def stats(self) -> dict:
        """Books handed over from idle symbols, resting orders replayed from the DB at create."""
        a, b = C.c_uint64(0), C.c_uint64(0)
        self.lib.me_service_stats(self.h, C.byref(a), C.byref(b))
        return {"reclaimed_books": a.value, "recovered_orders": b.value}

    def market_data(self, symbol) -> dict:
        """MarketDataUpdate (proto:60-67) from the GPU book; a missing side has has_* False and 0s."""
        m = MeMarketData()
        rc = self.lib.me_service_market_data(self.h, symbol.encode(), C.byref(m))
        if rc != 0:
            raise ServiceError(self.last_error())
        return {"symbol": symbol, "best_bid": m.best_bid, "best_ask": m.best_ask, "scale": m.scale,
                "bid_size": m.bid_size, "ask_size": m.ask_size, "has_bid": bool(m.has_bid),
                "has_ask": bool(m.has_ask)}

    def get_order_book(self, symbol, depth=10):
        bids = np.zeros(depth, dtype=LEVEL_DTYPE)
        asks = np.zeros(depth, dtype=LEVEL_DTYPE)
        nb, na = C.c_size_t(0), C.c_size_t(0)
        rc = self.lib.me_service_book(self.h, symbol.encode(), ptr(bids), ptr(asks), depth, C.byref(nb),
                                      C.byref(na))
        if rc != 0:
            raise ServiceError(self.last_error())
        return bids[: nb.value], asks[: na.value]

    def order_book(self, symbol, depth=0):
        """GetOrderBook in the reference's shape (OrderBookResponse: repeated Order bids / asks, proto
        :16-23,57-60): lists of {order_id, client_id, price, scale, quantity, side} dicts, best price
        first, time order within a price; depth = price levels per side (0: the whole book)."""
        nb, na = C.c_size_t(0), C.c_size_t(0)
        rc = self.lib.me_service_order_book(self.h, symbol.encode(), depth, None, 0, C.byref(nb), None, 0, C.byref(na))
        if rc != 0:
            raise ServiceError(self.last_error())
        bids, asks = (MeBookOrder * max(nb.value, 1))(), (MeBookOrder * max(na.value, 1))()
        rc = self.lib.me_service_order_book(self.h, symbol.encode(), depth, bids, nb.value, C.byref(nb), asks,
                                            na.value, C.byref(na))
        if rc != 0:
            raise ServiceError(self.last_error())

        def conv(arr, n):
            return [{"order_id": o.order_id.decode(), "client_id": o.client_id.decode(), "price": o.price,
                     "scale": o.scale, "quantity": o.quantity, "side": o.side} for o in arr[:n]]

        return conv(bids, nb.value), conv(asks, na.value)
