"""HBM traffic per k_match launch from rocprofv3 PMC passes (one counter per pass).

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/fetch -o pmc -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/write -o pmc -- python3 bench.py ...
    python tools/pmc_traffic.py OUT/fetch OUT/write --kernel k_match > profiles/r1_pmc_traffic.json

FETCH_SIZE / WRITE_SIZE are kilobytes (derived from TCC_EA0_RDREQ / _WRREQ). gfx950 correction
(MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of wide coalesced reads, so it is
doubled; WRITE_SIZE is taken as is. Other access widths are uncalibrated (documented caveat).
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kernel, merge_next=None):
    """Counter per launch of `kernel`, in dispatch order. A continuation launch (the register kernel's
    `<true>` instance, which follows its common launch on the same stream) is added to the launch
    it continues: together they are one launch group's matching. Dispatches matching `merge_next`
    (k_match_hot: launched, on its own stream, just before the k_match of the same batch) are added
    to the next launch."""
    import re
    vals = []
    for f in glob.glob(os.path.join(d, "**", "*counter_collection*.csv"), recursive=True):
        acc = {}
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name") or r.get("Kernel-Name") or ""
            cn = r.get("Counter_Name") or r.get("Counter-Name") or ""
            if re.search(kernel, name) and cn == counter:
                did = int(r.get("Dispatch_Id") or r.get("Dispatch-Id") or len(acc))
                cont = "<true>" in name
                v = float(r.get("Counter_Value") or r.get("Counter-Value"))
                k = acc.setdefault(did, [cont, 0.0, name])
                k[1] += v
        merged = []
        carry = 0.0
        for did in sorted(acc):
            cont, v, name = acc[did]
            if merge_next and re.search(merge_next, name):
                carry += v
            elif cont and merged:
                merged[-1] += v
            elif not cont:
                merged.append(v + carry)
                carry = 0.0
        vals += merged
    return vals


def main():
    a = sys.argv[1:]
    kernel = "k_match"
    if "--kernel" in a:
        i = a.index("--kernel")
        kernel = a[i + 1]
        del a[i:i + 2]
    orders = None
    if "--orders-per-launch" in a:
        i = a.index("--orders-per-launch")
        orders = int(a[i + 1])
        del a[i:i + 2]
    last = None
    if "--last" in a:  # only the last N launches (the steady steps after warmup / seeding)
        i = a.index("--last")
        last = int(a[i + 1])
        del a[i:i + 2]
    merge_next = None
    if "--merge-next" in a:
        i = a.index("--merge-next")
        merge_next = a[i + 1]
        del a[i:i + 2]
    fdir, wdir = a[0], a[1]
    f = per_dispatch(fdir, "FETCH_SIZE", kernel, merge_next)
    w = per_dispatch(wdir, "WRITE_SIZE", kernel, merge_next)
    if last:
        f, w = f[-last:], w[-last:]
    if not f or not w:
        print(json.dumps({"error": "no samples", "fetch": len(f), "write": len(w)}))
        return 1
    fetch_kb = sum(f) / len(f)
    write_kb = sum(w) / len(w)
    # the two passes replay the same launches: pair them in dispatch order. The median launch is a
    # steady pipelined one (bucket + match + tape jobs, a full group) — what roofline.achieved's
    # algorithmic bytes describe; the first (bucket-only) and the flush launches are the tails.
    n = min(len(f), len(w))
    per = sorted((2.0 * f[i] + w[i]) * 1024.0 for i in range(n))
    med = per[n // 2] if n % 2 else 0.5 * (per[n // 2 - 1] + per[n // 2])
    out = {
        "kernel": kernel,
        "dispatches": [len(f), len(w)],
        "fetch_size_kb_avg": fetch_kb,
        "write_size_kb_avg": write_kb,
        "bytes_per_launch": med,
        "bytes_per_launch_statistic": "median over dispatches (steady full-group launches)",
        "bytes_per_launch_all_avg": (2.0 * fetch_kb + write_kb) * 1024.0,
        "bytes_per_dispatch": [round(x) for x in per],
        "correction": "FETCH_SIZE x2 (gfx950 half-count of wide reads), WRITE_SIZE x1, KB->B x1024",
        "fetch_bytes_median": sorted(2.0 * x * 1024.0 for x in f)[len(f) // 2],
        "write_bytes_median": sorted(x * 1024.0 for x in w)[len(w) // 2],
        "orders_per_launch": orders,
        "bytes_per_order": med / orders if orders else None,
    }
    print(json.dumps(out, indent=1))
    return 0


if __name__ == "__main__":
    sys.exit(main())
