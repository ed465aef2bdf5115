"""Multi-GPU host logic: symbols are hash-sharded across GPUs with no cross-GPU matching
(SURVEY.md §8(e)). A global batch is split into per-shard batches (local symbol ids, global seq
kept); per-shard tapes and results merge back into exactly the single-engine output because
every taker's fills live on one shard and the tape order is (taker seq, fill#)."""
from __future__ import annotations

import numpy as np

from ._abi import FILL_DTYPE, RESULT_DTYPE
from .engine import Batch, shard_table


class ShardPlan:
    """global symbol -> (shard, local id) for `shards` GPUs over `num_symbols` symbols."""

    def __init__(self, num_symbols: int, shards: int):
        self.num_symbols = num_symbols
        self.shards = shards
        self.shard, self.local, self.members = shard_table(num_symbols, shards)

    def split(self, b: Batch):
        """-> list over shards of (batch with local ids, positions in the global batch)."""
        out = []
        sym = b.symbol
        ok = sym < self.num_symbols
        owner = np.where(ok, self.shard[np.minimum(sym, self.num_symbols - 1)], 0)
        for r in range(self.shards):
            pos = np.nonzero(owner == r)[0]
            lb = b.take(pos)
            s = lb.symbol
            inr = s < self.num_symbols
            # out-of-range ids stay out of range locally (the engine rejects them as BAD_SYMBOL)
            lb.symbol = np.where(inr, self.local[np.minimum(s, self.num_symbols - 1)],
                                 np.uint32(0xFFFFFFFF)).astype(np.uint32)
            out.append((lb, pos))
        return out


def merge_tapes(tapes) -> np.ndarray:
    """Per-shard tapes (each ordered by taker seq) -> the global tape, stable by taker seq."""
    tapes = [t for t in tapes if len(t)]
    if not tapes:
        return np.zeros(0, dtype=FILL_DTYPE)
    allf = np.concatenate(tapes)
    order = np.argsort(allf["taker_seq"], kind="stable")
    return allf[order]


def merge_results(n: int, parts) -> np.ndarray:
    """parts: (results of a shard, positions in the global batch) -> global results, with
    tape_offset recomputed against the merged tape."""
    res = np.zeros(n, dtype=RESULT_DTYPE)
    for r, pos in parts:
        res[pos] = r
    off = np.zeros(n, dtype=np.uint64)
    if n:
        off[1:] = np.cumsum(res["fill_count"].astype(np.uint64))[:-1]
    res["tape_offset"] = off.astype(np.uint32)
    return res
