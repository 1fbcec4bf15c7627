"""Diagnostic (tooling): one line of a rocprofv3 --stats run -- the kernels whose names contain the
given substrings (calls x average us) -- and the bench line's q/s and spot check.
usage: python tools/diag/kstats.py PROF_DIR BENCH_JSON substring [substring ...]"""
import csv
import glob
import json
import sys


def main():
    d, bj, subs = sys.argv[1], sys.argv[2], sys.argv[3:]
    f = glob.glob(d + "/*kernel_stats.csv")[0]
    out = []
    for r in csv.DictReader(open(f)):
        n = r["Name"]
        if any(s in n for s in subs):
            out.append(f"{n.split('(')[0].replace('void bsr::', '').replace('bsr::', '')}: "
                       f"{r['Calls']} x {float(r['AverageNs']) / 1e3:.1f} us")
    j = json.load(open(bj))
    sc = j.get("parity_spot_check", {})
    print(d.rstrip("/").split("/")[-1], "|", " | ".join(out), "| q/s", j.get("value"), "| spot check",
          sc.get("indices_equal"), sc.get("distance_bits_equal"), flush=True)


if __name__ == "__main__":
    main()
