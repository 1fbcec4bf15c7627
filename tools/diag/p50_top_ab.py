"""p50 A/B (tooling, round 6): single-query latency over the configs[3] corpus (10M synthetic rows)
with the self-thresholded path on and off (BSR_SKINNY_TOP, read per search), interleaved in one
process on one index.  Usage: python tools/diag/p50_top_ab.py [rows] [rounds] [iters]
Prints per round and mode the median wall time of one bsr_local_top_k call (device query, host
outputs, as bench.py's p50), the search path bits, and checks both modes return the same bits."""
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (before libbsr: one HIP runtime per process)
import bsr  # noqa: E402


def set_mode(mode):
    os.environ["BSR_SKINNY_TOP"] = mode[0]
    base = mode.rstrip("g")
    if ":" in base:
        os.environ["BSR_TOP_LAYOUT"] = base.split(":")[1]
    else:
        os.environ.pop("BSR_TOP_LAYOUT", None)
    os.environ["BSR_SKINNY_GLDS"] = "1" if mode.endswith("g") else "0"


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    iters = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    D, K = 768, 10
    rows = torch.empty((n, D), dtype=torch.float32, device="cuda:0")
    bsr.synth_uniform(rows.data_ptr(), 0, n, D, 42)
    torch.cuda.synchronize()
    ix = bsr.Index(D, max_k=64, device=0, flags=bsr.BSR_FLAG_PROFILE)
    ix.load(rows)
    del rows
    torch.cuda.empty_cache()
    q = torch.empty((8, D), dtype=torch.float32, device="cuda:0")
    bsr.synth_uniform(q.data_ptr(), 0, 8, D, 43)
    torch.cuda.synchronize()
    lib = bsr.lib()
    oi = np.zeros((1, K), np.uint64)
    od = np.zeros((1, K), np.float32)
    oc = np.zeros(1, np.uint32)
    ix.set_profile(0)

    def one(j):
        st = lib.bsr_local_top_k(ix._h, q[j:j + 1].data_ptr(), 1, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
        assert st == 0, lib.bsr_last_error()

    res = {}
    t_end = time.time() + 1.0
    while time.time() < t_end:  # settle the clock
        one(1)
    modes = sys.argv[4].split(",") if len(sys.argv) > 4 else ["1", "0"]
    for r in range(rounds):
        for mode in modes:
            # "0": the thresholded path; "1": the self-thresholded path; "1:L": with the lab row layout L;
            # a trailing "g": the LDS-DMA skinny filter (BSR_SKINNY_GLDS=1; without it: =0, k_filter_skinny2)
            set_mode(mode)
            for _ in range(20):
                one(1)
            lat = []
            for _ in range(iters):
                t0 = time.perf_counter()
                one(1)
                lat.append((time.perf_counter() - t0) * 1e3)
            st = ix.last_stats()
            outs = []
            for j in range(8):
                one(j)
                outs.append((oi.copy(), od.copy().view(np.uint32), oc.copy()))
            if mode in res:
                assert all(np.array_equal(a, b) for x, y in zip(res[mode], outs) for a, b in zip(x, y))
            res[mode] = outs
            print(f"round {r} top={mode}: p50 {statistics.median(lat):.4f} ms  min {min(lat):.4f}  "
                  f"path {st.search_path} replay {st.graph_replay} fallback {st.n_fallback} rescued {st.n_rescued} "
                  f"emitted {st.n_emitted}", flush=True)
    same = all(np.array_equal(a, b) for m in modes for x, y in zip(res[modes[0]], res[m]) for a, b in zip(x, y))
    print(f"results of the {len(modes)} paths over 8 queries: {'IDENTICAL' if same else 'DIFFER'}", flush=True)
    # kernel times per mode (profile level 1: the filter events; level 2 every stage)
    for mode in modes:
        set_mode(mode)
        ix.set_profile(2)
        ix.profile(reset=True)
        for _ in range(20):
            one(1)
        p = ix.profile(reset=True).as_dict()
        print(f"top={mode} profile (level 2, per search): " +
              ", ".join(f"{k} {v / 20:.4f}" for k, v in p.items() if k.endswith("_ms")), flush=True)
    ix.close()
    return 0 if same else 2


if __name__ == "__main__":
    sys.exit(main())
