"""RCCL gather of per-GPU trade tapes and per-record results to the persistence root.

SURVEY.md §8(e) and the north star: symbols are hash-sharded across the GPUs with no cross-GPU
matching; RCCL over xGMI is used only to bring every GPU's batch output to the host that persists
it (src/storage/storage.cpp:78-208 rewritten as a per-batch ingest, include/me_service.h). This is
the one collective of the design (torch.distributed backend "nccl" = RCCL on ROCm).

Per batch and rank the payload is the batch tape (32-B me_fill records, ordered by taker seq) and
the results of the rank's records (20-B me_order_result) with their positions in the global batch.
One all_gather exchanges the payload sizes; one gather per payload (padded to the largest rank's)
brings them to the root. The root merges the tapes by taker seq with a stable sort — every taker's
fills live on one shard, so this is exactly the single-engine tape — scatters the results back to
their global positions and recomputes tape offsets against the merged tape.

Backend-agnostic: RCCL with device tensors on the GPU box (the tape never leaves HBM before the
gather), gloo with CPU tensors in the CPU tests.
"""
from __future__ import annotations

import numpy as np

from ._abi import FILL_DTYPE, RESULT_DTYPE
from .sharding import merge_results

FILL_BYTES = FILL_DTYPE.itemsize      # 32
RESULT_BYTES = RESULT_DTYPE.itemsize  # 20
POS_BYTES = 8                         # int64 global position per local record


def _gather_padded(buf, nbytes: int, sizes, dst: int, group):
    """Gather the first nbytes of uint8 tensor buf from every rank (sizes[r] bytes from rank r) to
    dst. Returns the per-rank payloads (uint8 tensors) on dst, None elsewhere."""
    import torch
    import torch.distributed as dist

    pad = torch.zeros(max(max(sizes), 1), dtype=torch.uint8, device=buf.device)
    if nbytes:
        pad[:nbytes].copy_(buf.reshape(-1)[:nbytes])
    outs = [torch.empty_like(pad) for _ in sizes] if dist.get_rank(group) == dst else None
    dist.gather(pad, outs, dst=dst, group=group)
    return None if outs is None else [o[:s] for o, s in zip(outs, sizes)]


def merge_tape_tensors(parts) -> np.ndarray:
    """Per-shard tapes (uint8 tensors of 32-B fills, each ordered by taker seq) -> one tape ordered
    by taker seq (stable sort on the tensors' device), returned as host FILL_DTYPE records."""
    import torch

    parts = [p for p in parts if p.numel()]
    if not parts:
        return np.zeros(0, dtype=FILL_DTYPE)
    allf = torch.cat(parts).view(torch.int64).view(-1, FILL_BYTES // 8)
    order = torch.sort(allf[:, 0], stable=True).indices  # column 0 = taker_seq (< 2^63)
    merged = allf.index_select(0, order).contiguous().view(torch.uint8).reshape(-1).cpu().numpy()
    return merged.view(FILL_DTYPE)


def gather_batch(tape, n_fills: int, results, positions, n_local: int, n_global: int, dst: int = 0, group=None):
    """One batch's outputs of every rank -> (global tape, global results) on dst, (None, None)
    elsewhere.

    tape: uint8 tensor holding at least n_fills * 32 bytes (this rank's batch tape);
    results: uint8 tensor holding at least n_local * 20 bytes (this rank's per-record results);
    positions: int64 tensor [n_local], the global batch index of every local record.
    All three on the backend's device (HBM for RCCL, CPU for gloo)."""
    import torch
    import torch.distributed as dist

    if dist.get_backend(group) == "gloo" and tape.device.type != "cpu":
        # gloo (the CPU-test backend) moves host tensors; RCCL moves the device tensors directly
        tape, results, positions = tape.cpu(), results.cpu(), positions.cpu()
    dev = tape.device
    world = dist.get_world_size(group)
    mine = torch.tensor([n_fills * FILL_BYTES, n_local * (RESULT_BYTES + POS_BYTES)], dtype=torch.int64, device=dev)
    sizes = [torch.empty_like(mine) for _ in range(world)]
    dist.all_gather(sizes, mine, group=group)
    sz = torch.stack(sizes).cpu().numpy()
    tapes = _gather_padded(tape, n_fills * FILL_BYTES, [int(x) for x in sz[:, 0]], dst, group)
    rp = torch.empty(max(n_local * (RESULT_BYTES + POS_BYTES), 1), dtype=torch.uint8, device=dev)
    if n_local:
        rp[: n_local * RESULT_BYTES].copy_(results.reshape(-1)[: n_local * RESULT_BYTES])
        rp[n_local * RESULT_BYTES: n_local * (RESULT_BYTES + POS_BYTES)].copy_(
            positions[:n_local].to(torch.int64).contiguous().view(torch.uint8))
    res = _gather_padded(rp, n_local * (RESULT_BYTES + POS_BYTES), [int(x) for x in sz[:, 1]], dst, group)
    if tapes is None:
        return None, None
    parts = []
    for p in res:
        b = p.cpu().numpy()
        k = len(b) // (RESULT_BYTES + POS_BYTES)
        parts.append((b[: k * RESULT_BYTES].copy().view(RESULT_DTYPE),
                      b[k * RESULT_BYTES: k * (RESULT_BYTES + POS_BYTES)].copy().view(np.int64)))
    return merge_tape_tensors(tapes), merge_results(n_global, parts)


class EngineGather:
    """RCCL gather of one engine's batch outputs: device staging buffers sized for the engine, the
    engine's tape / results copied into them device-to-device, then gather_batch.

    With `stream` (a torch stream the engine runs on: engine.set_stream(stream.cuda_stream)) the
    gather of batch k overlaps the match of batch k+1:

        engine.submit_device(b[0])
        for k: nf = g.stage(n[k]); engine.submit_device(b[k + 1]); out = g.collect(nf, n[k], ...)

    stage() waits for batch k only and queues the staging copies on the engine stream; torch's
    current stream (where the collectives are ordered) waits for those copies through an event, not
    for the match launched after them. Without `stream`, stage() synchronises the engine."""

    def __init__(self, engine, device, max_batch: int, dst: int = 0, group=None, stream=None):
        import torch

        self.engine = engine
        self.dst = dst
        self.group = group
        self.stream = stream
        self.cap = engine.fill_bound(max_batch)
        self.tape = torch.empty(self.cap * FILL_BYTES, dtype=torch.uint8, device=device)
        self.res = torch.empty(max(max_batch, 1) * RESULT_BYTES, dtype=torch.uint8, device=device)

    def stage(self, n_local: int) -> int:
        """The most recent batch's tape and results into the staging buffers; returns its fills."""
        import torch

        nf = self.engine.copy_tape_device(self.tape.data_ptr(), self.cap)
        self.engine.copy_results_device(self.res.data_ptr(), n_local)
        if self.stream is not None:
            torch.cuda.current_stream(self.tape.device).wait_stream(self.stream)
        else:
            self.engine.sync()
        return nf

    def collect(self, nf: int, n_local: int, positions, n_global: int):
        """The staged batch of every rank -> (global tape, global results) on dst. Returns after the
        staging buffers were read, so the next stage() may overwrite them."""
        import torch

        out = gather_batch(self.tape, nf, self.res, positions, n_local, n_global, self.dst, self.group)
        # the payload copies out of the staging buffers were queued on torch's current stream (and
        # return at once off the root): the engine's next staging copies wait for them
        cur = torch.cuda.current_stream(self.tape.device)
        if self.stream is not None:
            self.stream.wait_stream(cur)
        else:
            cur.synchronize()
        return out

    def gather(self, n_local: int, positions, n_global: int):
        """After a batch of n_local records: -> (global tape, global results) on dst."""
        return self.collect(self.stage(n_local), n_local, positions, n_global)
