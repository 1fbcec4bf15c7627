"""Per-transition idle gaps between consecutive kernels of a rocprofv3 kernel trace (tooling).
usage: python tools/diag/gaps.py <kernel_trace.csv> [min_count]"""
import collections
import csv
import statistics
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0].replace("void ", "")))
rows.sort()
g = collections.defaultdict(list)
for a, b in zip(rows, rows[1:]):
    gap = (b[0] - a[1]) / 1e3
    if gap < 1000:
        g[(a[2], b[2])].append(gap)
mc = int(sys.argv[2]) if len(sys.argv) > 2 else 50
for k, v in sorted(g.items(), key=lambda kv: -len(kv[1])):
    if len(v) >= mc:
        print(f"{statistics.median(v):8.2f} us  x{len(v):4d}  {k[0]} -> {k[1]}")
