"""One rank of the multi-GPU sharding check (launched by tests/test_multirank.py).

Each rank owns the symbols splitmix64(symbol) % world == rank, runs its shard of the global
stream through a per-shard book, and the per-shard tapes/results are gathered to rank 0
(torch.distributed, gloo) and merged; rank 0 compares with ONE book over the whole stream.

env: RANK, WORLD_SIZE, MASTER_ADDR, MASTER_PORT; argv: ENGINE(oracle|gpu|gather|gpu_gather) OUT_JSON
  oracle:     the per-shard book is the CPU oracle (CPU test of the split/gather/merge host logic)
  gpu:        the per-shard book is the HIP engine on cuda:0 (all ranks share the box's one GPU)
  gather:     oracle shards, outputs moved by matching_engine_amd.gather.gather_batch (the RCCL
              tape/result gather) over gloo with CPU tensors
  gpu_gather: HIP engine shards, outputs staged device-to-device (EngineGather) and gathered with
              gather_batch (gloo stages the device tensors through the host; one GPU cannot host
              two RCCL ranks)
  rccl_gather: gpu_gather over the nccl (RCCL) backend with device tensors — world size 1 on the
              one-GPU box: the RCCL all_gather / gather calls and the overlapped staging run for real
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    engine_kind, out_path = sys.argv[1], sys.argv[2]
    import torch.distributed as dist

    import matching_engine_amd as me
    from matching_engine_amd.sharding import ShardPlan, merge_results, merge_tapes
    from oracle.oracle import OracleBook

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    if engine_kind == "rccl_gather":
        import torch

        torch.cuda.set_device(0)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        engine_kind = "gpu_gather"
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    S, nb = 300, 5
    sc = me.preset(5, num_symbols=S, batch=6000)
    st = me.Stream(sc)
    base = st.base_prices()
    plan = ShardPlan(S, world)
    ids = plan.members[rank]
    gath = None
    if engine_kind in ("gpu", "gpu_gather"):
        book = me.Engine(len(ids), sc.levels, base[ids], max_batch=sc.batch, max_resting=1 << 16,
                         symbol_ids=ids)
        submit = book.submit_batch
        if engine_kind == "gpu_gather":
            import torch

            from matching_engine_amd.gather import EngineGather

            ts = torch.cuda.Stream(device=torch.device("cuda", 0))
            book.set_stream(ts.cuda_stream)  # the gather of batch k overlaps the match of k + 1
            gath = EngineGather(book, torch.device("cuda", 0), sc.batch, stream=ts)
    else:
        book = OracleBook(len(ids), symbol_ids=ids)
        submit = book.submit
    ref = OracleBook(S) if rank == 0 else None
    ok, fills_total = True, 0
    msg = ""
    batches = []
    for k in range(nb):
        b = st.next(sc.batch)
        # a few out-of-range symbol ids too: rejected as BAD_SYMBOL on shard 0
        if k == 1:
            b.symbol[::997] = S + 5
        batches.append(b)
    splits = [plan.split(b)[rank] for b in batches]
    dbs = [book.upload(lb) for lb, _ in splits] if gath is not None else None
    if gath is not None:  # device-resident batches, the engine's outputs staged device to device
        book.submit_device(dbs[0])
    for k in range(nb):
        b = batches[k]
        lb, pos = splits[k]
        if gath is not None:
            nf = gath.stage(len(lb))
            if k + 1 < nb:
                book.submit_device(dbs[k + 1])  # matches while batch k is gathered
        else:
            r, f = submit(lb)
        if engine_kind in ("gather", "gpu_gather"):
            import torch

            from matching_engine_amd.gather import gather_batch

            post = torch.from_numpy(pos.astype(np.int64))
            if dist.get_backend() == "nccl":
                post = post.to("cuda:0")
            if gath is not None:
                tape, res = gath.collect(nf, len(lb), post, len(b))
            else:
                tape, res = gather_batch(torch.from_numpy(f.view(np.uint8).copy()), len(f),
                                         torch.from_numpy(r.view(np.uint8).copy()), post, len(lb), len(b))
        else:
            got = [None] * world
            dist.all_gather_object(got, (r, pos, f))
            if rank == 0:
                tape = merge_tapes([g[2] for g in got])
                res = merge_results(len(b), [(g[0], g[1]) for g in got])
        if rank == 0:
            ro, fo = ref.submit(b)
            fills_total += len(fo)
            same_t = len(tape) == len(fo) and bool(np.all(tape == fo))
            same_r = all(np.array_equal(res[x], ro[x]) for x in
                         ("filled_qty", "remaining_qty", "fill_count", "tape_offset", "status", "reason"))
            if ok and not (same_t and same_r):  # keep going: every rank must reach every collective
                ok = False
                msg = f"batch {k}: tape equal {same_t}, results equal {same_r}"
    if dbs is not None:
        book.sync()
        book.set_stream(None)
        for db in dbs:
            db.free()
    if rank == 0:
        json.dump({"ok": ok, "msg": msg, "fills": fills_total, "world": world}, open(out_path, "w"))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
