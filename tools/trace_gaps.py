"""Timeline of a rocprofv3 kernel trace: per-kernel average duration and the gaps between
consecutive k_match launches (what the pipeline adds around the matching kernel).

    python tools/trace_gaps.py <dir with *kernel_trace.csv>
"""
import csv
import glob
import os
import sys
from collections import defaultdict


def main():
    rows = []
    for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:48]))
    rows.sort()
    dur = defaultdict(list)
    for s, e, n in rows:
        dur[n].append(e - s)
    for n, v in sorted(dur.items(), key=lambda x: -sum(x[1])):
        print(f"{n:48s} n={len(v):5d} avg_us={sum(v) / len(v) / 1e3:8.2f}")
    # the common match launch (k_match_reg<false>, or k_match for deep windows), not its continuation
    m = [(s, e) for s, e, n in rows if "k_match" in n and "<true>" not in n]
    if len(m) > 2:
        per = [(m[i + 1][0] - m[i][0]) / 1e3 for i in range(len(m) - 1)]
        per.sort()
        print(f"k_match start-to-start: median {per[len(per) // 2]:.2f} us, min {per[0]:.2f} us")
        # what runs between two matches
        i = len(m) // 2
        lo, hi = m[i][0], m[i + 1][1]
        for s, e, n in rows:
            if e >= lo and s <= hi:
                print(f"  {n:48s} start {(s - lo) / 1e3:8.2f} end {(e - lo) / 1e3:8.2f}")


if __name__ == "__main__":
    main()
