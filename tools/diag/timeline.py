"""Per-search timeline from a rocprofv3 kernel trace (tooling).

usage: python tools/diag/timeline.py <kernel_trace.csv> [min_searches]

A search is the kernel sequence from one k_query_prep to the last kernel before the next one
(k_finalize or, since round 3, the second-chance k_rescore that finalizes in place).  Prints,
over the searches after the first few (steady state): the average duration of each kernel,
the span first-start -> last-end, the kernels' busy time inside it, the idle gaps between
them, and the turnaround last-end -> next prep-start (host wait, readback, Python, launch)."""
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
    # (a search's kernels follow each other within 1 ms; later launches belong to other work)
    trimmed = []
    for sr in searches:
        body = [sr[0]]
        for x in sr[1:]:
            if x[0] - body[-1][1] > 1_000_000:
                break
            body.append(x)
        trimmed.append(body)
    searches = trimmed
    # the dominant kernel sequence only (the batched searches; single-query, profiled-stage and
    # local-only passes have other sequences)
    sig = collections.Counter(tuple(n.split("(")[0] for _, _, n in sr) for sr in searches[skip:])
    main_sig = sig.most_common(1)[0][0] if sig else None
    steady = [sr for sr in searches[skip:] if tuple(n.split("(")[0] for _, _, n in sr) == main_sig]
    if not steady:
        print("no complete searches")
        return
    print(f"kernel sequences: {len(sig)}; the dominant one: {len(steady)} of {sum(sig.values())} searches")
    gaps = collections.defaultdict(list)
    for sr in steady:
        for j in range(1, len(sr)):
            gaps[j].append((sr[j][0] - sr[j - 1][1]) / 1e3)
    for j in sorted(gaps):
        print(f"  gap before {main_sig[j][:60]:60s} {statistics.median(gaps[j]):8.2f} us (median)")
    dur = collections.defaultdict(list)
    spans, busys, turns = [], [], []
    for i, sr in enumerate(steady):
        body = sr
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
    print(f"span first->last     {statistics.median(spans):9.2f} us (median)")
    print(f"kernels busy         {statistics.median(busys):9.2f} us")
    print(f"gaps between kernels {statistics.median(spans) - statistics.median(busys):9.2f} us")
    if turns:
        print(f"turnaround to next   {statistics.median(turns):9.2f} us (median)")


if __name__ == "__main__":
    main()
