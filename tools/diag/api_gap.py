"""Diagnostic (tooling, round 5): the host's share of a search's turnaround from a rocprofv3
--hip-trace --kernel-trace run: for each search (one k_query_prep kernel), the HIP API calls the
host made between the end of the previous search's last kernel and the start of this search's
query prep, summed by function (median over the steady searches), and the API calls issued while
the GPU ran the previous search's tail.
usage: python tools/diag/api_gap.py <dir with *_hip_api_trace.csv and *_kernel_trace.csv> [last_kernel]"""
import collections
import csv
import glob
import os
import statistics
import sys


def load(pattern):
    f = glob.glob(os.path.join(sys.argv[1], "**", pattern), recursive=True)
    return list(csv.DictReader(open(f[0]))) if f else []


def main():
    last_name = sys.argv[2] if len(sys.argv) > 2 else "k_merge_lists"
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in load("*kernel_trace.csv"))
    api = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in load("*hip_api_trace.csv"))
    preps = [k for k in ks if "k_query_prep" in k[2]]
    lasts = [k for k in ks if last_name in k[2]]
    rows = []
    for p in preps:
        prev = [x for x in lasts if x[1] <= p[0]]
        if not prev:
            continue
        t0, t1 = prev[-1][1], p[0]
        if t1 - t0 > 2_000_000:  # (another phase of the run)
            continue
        calls = [a for a in api if t0 <= a[0] < t1]
        by = collections.defaultdict(float)
        for a in calls:
            by[a[2]] += (a[1] - a[0]) / 1e3
        rows.append((t1 - t0, by, len(calls)))
    rows = rows[len(rows) // 5:]  # (steady state)
    if not rows:
        print("no searches")
        return
    print(f"searches: {len(rows)}; last kernel -> next query prep: median {statistics.median(r[0] for r in rows) / 1e3:.2f} us,"
          f" {statistics.median(r[2] for r in rows)} API calls in it (median)")
    names = collections.Counter()
    for _, by, _ in rows:
        for n in by:
            names[n] += 1
    for n, _ in names.most_common(25):
        v = [by.get(n, 0.0) for _, by, _ in rows]
        print(f"  {statistics.median(v):8.2f} us (median)  {n}")


if __name__ == "__main__":
    main()
