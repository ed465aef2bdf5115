"""Second, independent restatement of the matching semantics — TEST INFRASTRUCTURE ONLY.

The reference has no matcher (`include/engine/model.hpp` is empty), so fills cannot be pinned against
it. `oracle/oracle_book.cpp` is the golden model the GPU is checked against; this module restates
the same semantics a second time, in plain Python over sorted containers, written from the spec in
DESIGN.md §2 rather than from the C++ code, so that two independent implementations must agree on
every committed fixture and on random streams (`tests/test_pybook_cross.py`). Only tests import it.

Semantics (reference citations where the reference defines them):
  * domain: Side BUY=1 / SELL=2 (`include/domain/side.hpp:8-9`); OrderType LIMIT=0, anything else is
    MARKET (`src/server/matching_engine_service.cpp:50,78`); integer Q4 prices
    (`include/domain/price.hpp:6-29`); OIDs are the numeric seq, ascending (`:29-32`).
  * priority: price, then seq (FIFO inside a level); trade price = the maker's level; trade qty =
    min(taker remaining, maker remaining); a LIMIT remainder rests, a MARKET remainder is discarded.
  * statuses (`proto/matching_engine.proto:79-85`): LIMIT NEW / PARTIALLY_FILLED / FILLED; MARKET
    FILLED / CANCELED; CANCEL records CANCELED (remaining = qty removed) or REJECTED.
  * reject order: symbol out of range; cancel of a non-live order; qty <= 0; side not BUY/SELL;
    seq 0.
"""
from __future__ import annotations

from collections import deque

import numpy as np
from sortedcontainers import SortedDict

BUY, SELL = 1, 2
ST_NEW, ST_PARTIAL, ST_FILLED, ST_CANCELED, ST_REJECTED = 0, 1, 2, 3, 4
RJ_NONE, RJ_BAD_QTY, RJ_BAD_SIDE, RJ_BAD_SYMBOL, RJ_UNKNOWN, RJ_BAD_SEQ = 0, 1, 2, 4, 5, 6

RESULT_DTYPE = np.dtype([("filled_qty", "<i4"), ("remaining_qty", "<i4"), ("fill_count", "<u4"),
                         ("tape_offset", "<u4"), ("status", "u1"), ("reason", "u1"), ("pad", "u1", (2,))])
FILL_DTYPE = np.dtype([("taker_seq", "<u8"), ("maker_seq", "<u8"), ("price_q4", "<i8"), ("qty", "<i4"),
                       ("symbol", "<u4")])
BOOK_DTYPE = np.dtype([("seq", "<u8"), ("price_q4", "<i8"), ("qty", "<i4"), ("side", "u1"), ("pad", "u1", (3,))])


class _Side:
    """One side of one symbol: price -> FIFO of [seq, qty] (qty 0 = gone), best price first."""

    def __init__(self, bids: bool):
        self.bids = bids
        self.levels = SortedDict()  # key: -price for bids, price for asks

    def key(self, price):
        return -price if self.bids else price

    def best(self):
        if not self.levels:
            return None
        k = self.levels.keys()[0]
        return -k if self.bids else k

    def fifo(self, price, create=False):
        k = self.key(price)
        q = self.levels.get(k)
        if q is None and create:
            q = self.levels[k] = deque()
        return q

    def drop_if_empty(self, price):
        q = self.levels.get(self.key(price))
        if q is not None and not any(e[1] > 0 for e in q):
            del self.levels[self.key(price)]


class PyBook:
    """All symbols of one engine; submit() takes a batch (seq-ordered records) like the C-ABI."""

    def __init__(self, num_symbols):
        self.S = num_symbols
        self.side = [(_Side(True), _Side(False)) for _ in range(num_symbols)]
        self.live = {}  # seq -> (symbol, side, price, entry)

    def submit(self, b):
        n = len(b.seq)
        res = np.zeros(n, dtype=RESULT_DTYPE)
        tape = []
        for i in range(n):
            seq, px, q = int(b.seq[i]), int(b.price_q4[i]), int(b.qty[i])
            s, kind = int(b.symbol[i]), int(b.kind[i])
            side, market, cancel = kind & 3, bool(kind & 4), bool(kind & 8)
            r = res[i]
            r["tape_offset"] = len(tape)
            if s >= self.S:
                r["status"], r["reason"] = ST_REJECTED, RJ_BAD_SYMBOL
                continue
            if cancel:
                hit = self.live.get(px)  # a cancel's price field carries its target seq
                if hit is None or hit[0] != s:
                    r["status"], r["reason"] = ST_REJECTED, RJ_UNKNOWN
                    continue
                _, tside, tprice, entry = hit
                got = entry[1]
                entry[1] = 0
                del self.live[px]
                book = self.side[s][0] if tside == BUY else self.side[s][1]
                book.drop_if_empty(tprice)
                r["status"], r["remaining_qty"] = ST_CANCELED, got
                continue
            if q <= 0:
                r["status"], r["reason"] = ST_REJECTED, RJ_BAD_QTY
                continue
            r["remaining_qty"] = q
            if side not in (BUY, SELL):
                r["status"], r["reason"] = ST_REJECTED, RJ_BAD_SIDE
                continue
            if seq == 0:
                r["status"], r["reason"] = ST_REJECTED, RJ_BAD_SEQ
                continue
            own, opp = (self.side[s][0], self.side[s][1]) if side == BUY else (self.side[s][1], self.side[s][0])
            rem, t0 = q, len(tape)
            while rem > 0:
                p = opp.best()
                if p is None or (not market and (p > px if side == BUY else p < px)):
                    break
                fifo = opp.fifo(p)
                while rem > 0 and fifo:
                    e = fifo[0]
                    if e[1] == 0:
                        fifo.popleft()
                        continue
                    t = min(rem, e[1])
                    tape.append((seq, e[0], p, t, s))
                    e[1] -= t
                    rem -= t
                    if e[1] == 0:
                        fifo.popleft()
                        del self.live[e[0]]
                opp.drop_if_empty(p)
            filled = q - rem
            r["filled_qty"], r["remaining_qty"], r["fill_count"] = filled, rem, len(tape) - t0
            if market:
                r["status"] = ST_FILLED if rem == 0 else ST_CANCELED
                continue
            if rem > 0:
                entry = [seq, rem]
                own.fifo(px, create=True).append(entry)
                self.live[seq] = (s, side, px, entry)
            r["status"] = ST_FILLED if rem == 0 else (ST_PARTIAL if filled else ST_NEW)
        fills = np.array(tape, dtype=FILL_DTYPE) if tape else np.zeros(0, dtype=FILL_DTYPE)
        return res, fills

    def dump(self, s):
        """Resting orders of symbol s: bids best first, then asks best first, FIFO inside a level."""
        out = []
        for side, book in ((BUY, self.side[s][0]), (SELL, self.side[s][1])):
            for k, fifo in book.levels.items():
                price = -k if book.bids else k
                out += [(e[0], price, e[1], side, (0, 0, 0)) for e in fifo if e[1] > 0]
        return np.array(out, dtype=BOOK_DTYPE) if out else np.zeros(0, dtype=BOOK_DTYPE)
