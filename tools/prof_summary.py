#!/usr/bin/env python3
"""Summaries of rocprofv3 output for tools/gpu/record.sh.

    prof_summary.py trace DIR [--steps K]        per-kernel count / avg / total (us) of a kernel trace, and
                                                 the timeline of the run's last launch group
    prof_summary.py dram DIR --bench LOG       byte-exact EA traffic per order from the 32-B-unit counters
    prof_summary.py traffic FETCH_DIR WRITE_DIR --bench LOG [--from-sweep K]
                                                 HBM bytes per order over every included dispatch of the run
                                                 (FETCH_SIZE x2, the gfx950 correction of MI355X_MICROARCH.md;
                                                 WRITE_SIZE x1; KB -> B), per kernel and in total, divided by
                                                 the orders the run pushed through (warmup + timed batches)
    prof_summary.py sq DIR [DIR ...]             SQ counters per kernel: median per dispatch, per wave
"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def kname(n):
    n = n.replace("me::(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", n)


def trace(d, steps=None):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), kname(r["Kernel_Name"])))
    rows.sort()
    agg = defaultdict(list)
    for s, e, n in rows:
        agg[n].append((e - s) / 1e3)
    print(f"{'kernel':44s} {'n':>5s} {'avg_us':>9s} {'max_us':>9s} {'total_us':>10s}")
    for n, v in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print(f"{n:44s} {len(v):5d} {sum(v) / len(v):9.1f} {max(v):9.1f} {sum(v):10.1f}")
    # the last launch group: everything after the largest idle gap among the last 60 dispatches
    tail = rows[-60:]
    if len(tail) > 2:
        cut, gap = 0, -1
        for i in range(1, len(tail)):
            g = tail[i][0] - max(e for _, e, _ in tail[:i])
            if g > gap:
                gap, cut = g, i
        grp = tail[cut:]
        t0 = grp[0][0]
        span = (max(e for _, e, _ in grp) - t0) / 1e3
        print(f"\nlast group: {len(grp)} dispatches over {span:.1f} us"
              + (f" ({span / steps:.2f} us per timed batch)" if steps else ""))
        for s, e, n in grp:
            print(f"  {n:44s} start {(s - t0) / 1e3:9.1f} end {(e - t0) / 1e3:9.1f} dur {(e - s) / 1e3:8.1f}")


def bench_orders(log):
    for line in open(log):
        if line.startswith('{"metric"'):
            d = json.loads(line)
            return d, (d["steps"] + d["warmup"]) * d["config"]["global_batch"]
    raise SystemExit(f"no bench line in {log}")


def counters(d, want=None, from_sweep=0):
    """{kernel: {counter: [value per dispatch]}} (values summed over the dispatch's rows); from_sweep = k:
    only the dispatches from the k-th k_seq_sweep on (the batches before it — config 4's seeding — dropped)."""
    out = defaultdict(lambda: defaultdict(dict))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        rows = list(csv.DictReader(open(f)))
        first = 0
        if from_sweep:
            sw = sorted({int(r.get("Dispatch_Id") or 0) for r in rows if "k_seq_sweep" in (r.get("Kernel_Name") or "")})
            first = sw[from_sweep] if from_sweep < len(sw) else 1 << 62
        for r in rows:
            if int(r.get("Dispatch_Id") or 0) < first:
                continue
            cn = r.get("Counter_Name") or r.get("Counter-Name")
            if want and cn != want:
                continue
            n = kname(r.get("Kernel_Name") or r.get("Kernel-Name") or "")
            did = int(r.get("Dispatch_Id") or r.get("Dispatch-Id") or 0)
            v = float(r.get("Counter_Value") or r.get("Counter-Value"))
            out[n][cn][did] = out[n][cn].get(did, 0.0) + v
    return {n: {c: [v[k] for k in sorted(v)] for c, v in cs.items()} for n, cs in out.items()}


def traffic(fdir, wdir, log, from_sweep=0):
    d, orders = bench_orders(log)
    f = counters(fdir, "FETCH_SIZE", from_sweep)
    w = counters(wdir, "WRITE_SIZE", from_sweep)
    per = {}
    tot_f = tot_w = 0.0
    for n in sorted(set(f) | set(w)):
        fb = 2.0 * 1024.0 * sum(f.get(n, {}).get("FETCH_SIZE", []))
        wb = 1024.0 * sum(w.get(n, {}).get("WRITE_SIZE", []))
        tot_f += fb
        tot_w += wb
        per[n] = {"dispatches": len(w.get(n, {}).get("WRITE_SIZE", [])), "fetch_bytes_per_order": fb / orders,
                  "write_bytes_per_order": wb / orders, "bytes_per_order": (fb + wb) / orders}
    out = {
        "bytes_per_order": (tot_f + tot_w) / orders,
        "fetch_bytes_per_order": tot_f / orders,
        "write_bytes_per_order": tot_w / orders,
        "orders": orders,
        "statistic": "sum over every dispatch of the match pipeline's kernels in the run (warmup + timed "
                     "batches, fill and drain launches included) / the orders of those batches",
        "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads, MI355X_MICROARCH.md), WRITE_SIZE x1, KB->B x1024",
        "from_sweep": from_sweep,
        "per_kernel": dict(sorted(per.items(), key=lambda x: -x[1]["bytes_per_order"])),
        "build": d.get("build"),
        "workload": d["config"].get("workload"),
        "steps": d["steps"], "warmup": d["warmup"],
    }
    print(json.dumps(out, indent=1))


DRAM = ("TCC_EA0_RDREQ_DRAM_32B", "TCC_EA0_WRREQ_WRITE_DRAM_32B", "TCC_EA0_WRREQ_WRITE_ATOMIC_32B", "TCC_EA0_RDREQ")


def dram(ddir, log):
    """Byte-exact EA traffic: the gfx950 32-byte-unit request counters (a 64-B request counts 2, a 128-B one
    4), so no request-size correction is needed — the cross-check of FETCH_SIZE x2 + WRITE_SIZE."""
    d, orders = bench_orders(log)
    c = counters(ddir)
    per = {}
    tot = defaultdict(float)
    for n, cs in c.items():
        v = {k: sum(cs.get(k, [])) for k in DRAM}
        rd, wr, at = 32.0 * v[DRAM[0]], 32.0 * v[DRAM[1]], 32.0 * v[DRAM[2]]
        for k, x in (("rd", rd), ("wr", wr), ("at", at), ("req", v[DRAM[3]])):
            tot[k] += x
        per[n] = {"dispatches": len(cs.get(DRAM[0], [])), "read_bytes_per_order": rd / orders,
                  "write_bytes_per_order": wr / orders, "atomic_bytes_per_order": at / orders,
                  "bytes_per_order": (rd + wr + at) / orders,
                  "mean_read_request_bytes": rd / v[DRAM[3]] if v[DRAM[3]] else None}
    out = {
        "bytes_per_order": (tot["rd"] + tot["wr"] + tot["at"]) / orders,
        "read_bytes_per_order": tot["rd"] / orders,
        "write_bytes_per_order": tot["wr"] / orders,
        "atomic_bytes_per_order": tot["at"] / orders,
        "orders": orders,
        "counters": "32 x (TCC_EA0_RDREQ_DRAM_32B + TCC_EA0_WRREQ_WRITE_DRAM_32B + TCC_EA0_WRREQ_WRITE_ATOMIC_32B), "
                    "one pass; TCC_EA0_RDREQ for the mean read request size",
        "statistic": "sum over every dispatch of the match pipeline's kernels in the run / the orders of those batches",
        "per_kernel": dict(sorted(per.items(), key=lambda x: -x[1]["bytes_per_order"])),
        "build": d.get("build"),
        "workload": d["config"].get("workload"),
        "steps": d["steps"], "warmup": d["warmup"],
    }
    print(json.dumps(out, indent=1))


def sq(dirs):
    allc = defaultdict(dict)
    for d in dirs:
        for n, cs in counters(d).items():
            allc[n].update(cs)
    for n, cs in sorted(allc.items()):
        print(f"== {n}")
        waves = cs.get("SQ_WAVES")
        for c, v in sorted(cs.items()):
            med = sorted(v)[len(v) // 2]
            extra = ""
            if waves and c != "SQ_WAVES":
                wm = sorted(waves)[len(waves) // 2]
                extra = f"  per wave {med / wm:.4g}" if wm else ""
            print(f"  {c:24s} n={len(v):4d} median/dispatch={med:.6g}{extra}")
        if "SQ_LDS_BANK_CONFLICT" in cs and "SQ_LDS_IDX_ACTIVE" in cs:
            bc, ia = sum(cs["SQ_LDS_BANK_CONFLICT"]), sum(cs["SQ_LDS_IDX_ACTIVE"])
            print(f"  LDS bank-conflict cycles / LDS-active cycles = {bc / ia if ia else 0:.4f}")
        if "SQ_WAIT_ANY" in cs and "SQ_WAVE_CYCLES" in cs:
            wa, wc = sum(cs["SQ_WAIT_ANY"]), sum(cs["SQ_WAVE_CYCLES"])
            print(f"  waiting share of wave cycles = {wa / wc if wc else 0:.3f}")


def main():
    a = sys.argv[1:]
    if a[0] == "trace":
        steps = int(a[a.index("--steps") + 1]) if "--steps" in a else None
        trace(a[1], steps)
    elif a[0] == "traffic":
        traffic(a[1], a[2], a[a.index("--bench") + 1], int(a[a.index("--from-sweep") + 1]) if "--from-sweep" in a else 0)
    elif a[0] == "dram":
        dram(a[1], a[a.index("--bench") + 1])
    elif a[0] == "sq":
        sq(a[1:])
    else:
        raise SystemExit(__doc__)


if __name__ == "__main__":
    main()
