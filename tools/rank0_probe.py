"""Rank 0's host work per global slice at W shards, without a multi-GPU node:
me_cluster_host_probe runs the cluster's own split (owner counts + stable pack into per-rank parts) and
merge (results back to slice order, the merged tape by taker) code over config 3's global slice shape
(1,048,576 orders over 100,000 symbols) with synthetic shard outputs at config 3's fill rate, and reports
the per-slice times and the orders/s rank 0's host path alone could sustain.

    python tools/rank0_probe.py [--worlds 1,2,4,8] [--iters 8] [--fills-per-order 0.93] > out.json
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import matching_engine_amd as me  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--worlds", default="1,2,4,8")
    ap.add_argument("--iters", type=int, default=8)
    ap.add_argument("--fills-per-order", type=float, default=0.93)
    ap.add_argument("--slice", type=int, default=1 << 20)
    ap.add_argument("--symbols", type=int, default=100_000)
    a = ap.parse_args()
    lib = me._abi.load()
    sc = me.preset(3, num_symbols=a.symbols, batch=a.slice)
    b = me.Stream(sc).next(a.slice)
    soa = b.soa()
    rows = []
    for W in [int(x) for x in a.worlds.split(",")]:
        sec = (C.c_double * 4)()
        rc = lib.me_cluster_host_probe(W, a.symbols, C.byref(soa), len(b), a.fills_per_order, a.iters, sec)
        if rc:
            raise SystemExit(f"probe failed at W={W}: {rc}")
        tot = sec[0] + sec[1] + sec[2]
        rows.append({"world": W, "count_ms": round(sec[0] * 1e3, 3), "pack_ms": round(sec[1] * 1e3, 3),
                     "merge_ms": round(sec[2] * 1e3, 3), "split_plus_merge_ms": round(tot * 1e3, 3),
                     "tape_fills": int(sec[3]), "rank0_host_orders_per_s": len(b) / tot})
    host = {"nproc": os.cpu_count(), "cpus_allowed": len(os.sched_getaffinity(0))}
    try:
        host["cgroup_cpu_max"] = open("/sys/fs/cgroup/cpu.max").read().strip()
    except OSError:
        host["cgroup_cpu_max"] = None
    print(json.dumps({"what": "me_cluster_host_probe: rank 0's split + merge per global slice (config 3 shape), "
                              "synthetic shard outputs, no GPU or transport; one slice in flight at a time (the "
                              "deployment overlaps two)", "slice_orders": len(b), "symbols": a.symbols,
                      "fills_per_order": a.fills_per_order, "iters": a.iters, "host": host, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
