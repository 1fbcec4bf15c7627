"""Average each PMC counter per kernel (template instance) over rocprofv3 CSV passes (tooling)."""
import collections
import csv
import glob
import sys

d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name in sorted(vals):
    if "k_filter" not in name:
        continue
    print(name)
    for c in sorted(vals[name]):
        v = vals[name][c]
        print(f"   {c:32s} {sum(v) / len(v):14.6g}")
