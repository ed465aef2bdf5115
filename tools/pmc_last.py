"""Per-dispatch SQ counters of the last N dispatches of a rocprofv3 --pmc run (the steady-state
steps of a bench, after warmup / seeding): python tools/pmc_last.py DIR [N] [RECORDS]"""
import collections
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 3
recs = float(sys.argv[3]) if len(sys.argv) > 3 else 0
acc = collections.defaultdict(list)
for f in glob.glob(f"{d}/**/*counter_collection*.csv", recursive=True):
    by = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        by[int(r["Dispatch_Id"])][r["Counter_Name"]] = float(r["Counter_Value"])
    for di in sorted(by)[-n:]:
        for k, v in by[di].items():
            acc[k].append(v)
for k, v in sorted(acc.items()):
    a = sum(v) / len(v)
    extra = f"  per_record={a / recs:.1f}" if recs else ""
    print(f"{k:28s} {a:14.4g}{extra}")
