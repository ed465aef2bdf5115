"""Print the last N kernels of a rocprofv3 CSV kernel trace: start (us from the first), duration, name.

    python tools/last_trace.py <dir with *kernel_trace.csv> [N]
"""
import csv
import glob
import os
import sys

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*kernel_trace.csv"), recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60]))
rows.sort()
n = int(sys.argv[2]) if len(sys.argv) > 2 else 14
for s, e, name in rows[-n:]:
    print(f"{(s - rows[0][0]) / 1e3:12.1f} {(e - s) / 1e3:9.1f} {name}")
