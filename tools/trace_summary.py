"""Per-kernel duration summary of a rocprofv3 kernel trace CSV: count, average, max, total (us)."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
d = defaultdict(list)
for r in rows:
    n = r["Kernel_Name"].replace("me::(anonymous namespace)::", "").replace("void ", "").split("(")[0]
    d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in sorted(d.items(), key=lambda x: -sum(x[1])):
    print(f"{n:44s} n={len(v):4d} avg={sum(v) / len(v):9.1f}us max={max(v):9.1f} total={sum(v):10.1f}")
