"""Per-search timeline from a rocprofv3 kernel trace (tooling).

usage: python tools/diag/timeline.py <kernel_trace.csv> [min_searches]

A search is the kernel sequence k_query_prep ... k_finalize on one queue.  Prints, over the
searches after the first few (steady state): the average duration of each kernel, the span
prep-start -> finalize-end, the kernels' busy time inside it, the idle gaps between them,
and the turnaround finalize-end -> next prep-start (host wait, readback, Python, launch)."""
import collections
import csv
import statistics
import sys


def main():
    path = sys.argv[1]
    skip = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    searches, cur = [], None
    for s, e, name in rows:
        if "k_query_prep" in name:
            cur = [(s, e, name)]
            searches.append(cur)
        elif cur is not None:
            cur.append((s, e, name))
    searches = [sr for sr in searches if any("k_finalize" in n for _, _, n in sr)]
    steady = searches[skip:]
    if not steady:
        print("no complete searches")
        return
    dur = collections.defaultdict(list)
    spans, busys, turns = [], [], []
    for i, sr in enumerate(steady):
        fin = max(j for j, (_, _, n) in enumerate(sr) if "k_finalize" in n)
        body = sr[:fin + 1]
        for s, e, n in body:
            dur[n.split("(")[0]].append((e - s) / 1e3)
        spans.append((body[-1][1] - body[0][0]) / 1e3)
        busys.append(sum(e - s for s, e, _ in body) / 1e3)
        nxt = searches[searches.index(sr) + 1] if searches.index(sr) + 1 < len(searches) else None
        if nxt:
            turns.append((nxt[0][0] - body[-1][1]) / 1e3)
    print(f"searches: {len(steady)} (after {skip})")
    for n, v in sorted(dur.items(), key=lambda kv: -statistics.mean(kv[1]) * len(kv[1])):
        print(f"  {statistics.mean(v):9.2f} us  x{len(v) / len(steady):4.2f}/search  {n}")
    print(f"span prep->finalize  {statistics.median(spans):9.2f} us (median)")
    print(f"kernels busy         {statistics.median(busys):9.2f} us")
    print(f"gaps between kernels {statistics.median(spans) - statistics.median(busys):9.2f} us")
    if turns:
        print(f"turnaround to next   {statistics.median(turns):9.2f} us (median)")


if __name__ == "__main__":
    main()
