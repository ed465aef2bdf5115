"""The sharded deployment through the C++ cluster (include/me_cluster.h): ranks as processes, symbols
hash-partitioned, the protocol over TCP (CPU tests: oracle shards behind me_shard_ops) or RCCL (the GPU
box: world size 1, since one GPU cannot host two RCCL ranks). Every check compares against ONE book
holding every symbol: direct slices two in flight, then a SubmitOrder service over me_cluster_matcher
against a service over a single book — outputs, SQLite rows, books, market data, level snapshot."""
import json
import os
import socket
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(kind, world, tmp_path, timeout=240, env_extra=None):
    out = str(tmp_path / f"cl_{kind}_{world}.json")
    port = _free_port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **(env_extra or {}))
        # child processes (never exec over a GPU-initialised interpreter)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "cluster_worker.py"), kind, str(tmp_path),
                                       out], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    for p in procs:
        try:
            o, _ = p.communicate(timeout=timeout)
        except subprocess.TimeoutExpired:
            p.kill()
            o, _ = p.communicate()
        logs.append(o.decode(errors="replace")[-3000:])
    assert all(p.returncode == 0 for p in procs), "\n".join(logs)
    return json.load(open(out))


@pytest.mark.parametrize("world", [2, 3])
def test_cluster_tcp_oracle_shards(built, tmp_path, world):
    """the C++ cluster over a CPU transport (TCP star), oracle shards: direct slices
    and the sharded service's DB equal one book's."""
    r = _run("oracle", world, tmp_path)
    assert r["ok"], r["msg"]
    assert r["orders"] > 5000 and r["fill_rows"] > 1000 and r["direct_fills"] > 0
    assert r["errors"] == ["", ""], r["errors"]
    assert r["slices"] >= 6 + 5


def test_cluster_refused_slice_is_split_all_or_none(built, tmp_path):
    """One shard's admission control refuses its part of a slice once: no shard applies anything of it
    (all-or-none vote), the service splits the slice and matches the halves — the DB, outputs and books
    still equal the single book's, and the flush reports no error."""
    r = _run("oracle_refuse", 2, tmp_path)
    assert r["ok"], r["msg"]
    assert r["refused"] == 1
    assert r["errors"] == ["", ""], r["errors"]


@pytest.mark.gpu
def test_cluster_tcp_gpu_engines(built, tmp_path):
    """Two ranks, each with its own HIP engine on the box's GPU, protocol over TCP."""
    r = _run("gpu", 2, tmp_path)
    assert r["ok"], r["msg"]
    assert r["orders"] > 5000 and r["fill_rows"] > 1000


@pytest.mark.gpu
def test_cluster_rccl_single_rank(built, tmp_path):
    """The RCCL transport with an engine shard, world size 1, rank 0's part forced through the transport
    (ME_CLUSTER_DIRECT=0): ncclCommInitRank over the TCP bootstrap, and the grouped send / recv of parts,
    tapes and results (rank 0 sends to itself) — every RCCL call an 8-GPU node makes, minus the xGMI hops."""
    r = _run("rccl", 1, tmp_path, env_extra={"ME_CLUSTER_DIRECT": "0"})
    assert r["ok"], r["msg"]
    assert r["orders"] > 5000 and r["fill_rows"] > 1000 and r["bytes"] > 0


@pytest.mark.gpu
def test_cluster_rccl_single_rank_direct(built, tmp_path):
    """World size 1 as deployed: rank 0's part goes straight into its engine's pinned slots (no pack copy,
    scatter or gather) and collect hands out the slot's outputs in place; the same checks against one book."""
    r = _run("rccl", 1, tmp_path)
    assert r["ok"], r["msg"]
    assert r["orders"] > 5000 and r["fill_rows"] > 1000


@pytest.mark.gpu
def test_cluster_large_max_batch_reserves_protocol_slots(built, tmp_path):
    """me_cluster_create reserves only the host slots its protocol can use (two slices in flight
    plus the held one), not the engine's default 4 * 32 + 1. With a 4M-record max_batch each slot pins
    ~0.45 GB, so the default-config cluster here (batches_per_launch 32) would pin ~57 GB up front; it
    must come up and match the same direct slices and service traffic as the small one."""
    r = _run("rccl", 1, tmp_path, env_extra={"ME_TEST_MAX_BATCH": str(1 << 22)})
    assert r["ok"], r["msg"]
    assert r["orders"] > 5000 and r["fill_rows"] > 1000
