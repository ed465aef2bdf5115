"""The symbol-hash partition as the bench's CPU baseline uses it: a global batch split
into per-shard batches (local symbol ids, global seq kept). The deployment's split, scatter, gather
and merge are C++ (csrc/me_cluster.cpp, include/me_cluster.h)."""
from __future__ import annotations

import numpy as np

from .engine import Batch, shard_table


class ShardPlan:
    """global symbol -> (shard, local id) for `shards` GPUs over `num_symbols` symbols."""

    def __init__(self, num_symbols: int, shards: int):
        self.num_symbols = num_symbols
        self.shards = shards
        self.shard, self.local, self.members = shard_table(num_symbols, shards)

    def split(self, b: Batch):
        """-> list over shards of (batch with local ids, positions in the global batch)."""
        sym = b.symbol
        ok = sym < self.num_symbols
        owner = np.where(ok, self.shard[np.minimum(sym, self.num_symbols - 1)], 0)
        # one stable sort by owner (batch order kept inside each shard), then a slice per shard
        order = np.argsort(owner, kind="stable")
        ends = np.cumsum(np.bincount(owner, minlength=self.shards))
        out = []
        for r in range(self.shards):
            pos = order[(ends[r - 1] if r else 0):ends[r]]
            lb = b.take(pos)
            s = lb.symbol
            inr = s < self.num_symbols
            # out-of-range ids stay out of range locally (the engine rejects them as BAD_SYMBOL)
            lb.symbol = np.where(inr, self.local[np.minimum(s, self.num_symbols - 1)],
                                 np.uint32(0xFFFFFFFF)).astype(np.uint32)
            out.append((lb, pos))
        return out
