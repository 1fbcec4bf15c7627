"""Turn rocprofv3 --pmc CSVs of bench.py into profiles/pmc_traffic.json (tooling).

HBM bytes per launch of the dominant kernel = FETCH_SIZE * 1024 * 2 + WRITE_SIZE * 1024:
on gfx950 FETCH_SIZE (KB) reports half of the bytes of a wide coalesced read
(MI355X_MICROARCH.md, HBM section), WRITE_SIZE is exact for 16-B stores.  FETCH_SIZE and
WRITE_SIZE are collected in separate passes (TCC counter slots).
usage: python tools/pmc_traffic.py <fetch_dir> <write_dir> <rows> <queries> <filter> <out.json>

out.json keeps one entry per (rows, queries, filter) shard shape under "entries", so the
bench finds the traffic of each rank's shard at every N; a rerun replaces its entry.
"""
import os
import csv
import glob
import json
import sys


def per_kernel(d, counter):
    vals = {}
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            name = r["Kernel_Name"].split("(")[0].replace("void ", "")
            vals.setdefault(name, []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in vals.items()}


def main():
    fdir, wdir, rows, queries, filt, out = sys.argv[1:7]
    fetch = per_kernel(fdir, "FETCH_SIZE")
    write = per_kernel(wdir, "WRITE_SIZE")
    # the emitting filter with the largest fetch (the skinny single-query filter matches too)
    emit = sorted((k for k in fetch if "k_filter" in k and "true" in k), key=lambda k: -fetch[k])
    res = {"rows": int(rows), "queries": int(queries), "filter": filt, "run": os.environ.get("PMC_RUN", ""),
           "kernels": {}}
    for k in sorted(set(fetch) | set(write)):
        f = fetch.get(k)
        w = write.get(k)
        res["kernels"][k] = {"fetch_size_kb": f, "write_size_kb": w,
                             "hbm_bytes_corrected": (f * 1024 * 2 if f is not None else 0) +
                                                    (w * 1024 if w is not None else 0)}
    if emit:
        res["dominant_kernel"] = emit[0]
        res["hbm_bytes_per_launch"] = res["kernels"][emit[0]]["hbm_bytes_corrected"]
    entries = []
    if os.path.exists(out):
        try:
            old = json.load(open(out))
            entries = old.get("entries", [old] if "rows" in old else [])
        except (OSError, ValueError):
            entries = []
    key = (res["rows"], res["queries"], res["filter"])
    entries = [e for e in entries if (e.get("rows"), e.get("queries"), e.get("filter")) != key] + [res]
    entries.sort(key=lambda e: (e.get("filter"), e.get("queries"), -e.get("rows", 0)))
    json.dump({"entries": entries}, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
