"""Diagnostic (tooling, round 5): where the global-threshold search's rescore of every emitted row
goes (mode B, one wave per query, ~32 rows per query per rank at N = 8), from the per-wave phase
stamps of the lab build (make -C better-search-rag-rust_amd lab-stamps), on rank 0's 1.25M-row
shard of the 10M corpus through a loopback communicator replaying a recorded 8-rank run.
Phases: 0 start, 1 query row in LDS, 2 (no selection in mode B), 3 rows scored, 4 finished.
usage: BSR_LIB=tools/ab/libbsr_stamps.so python tools/diag/rescore_stamps_gtau.py <loop8.npz>"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import torch  # noqa: E402
import bsr  # noqa: E402

P, NT, D, Q, K = 8, 10_000_000, 768, 1000, 10
iv = bsr.interval_by_rank(0, P, NT)
N = iv.get_count()
rows = torch.empty((N, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(rows.data_ptr(), 0, N, D, 42)
torch.cuda.synchronize()
ix = bsr.Index(D, max_k=64, device=0)
ix.load(rows, 0)
del rows
torch.cuda.empty_cache()
q = torch.empty((Q, D), dtype=torch.float32, device="cuda:0")  # (bench.py's batch: query 0 = row 0)
bsr.synth_uniform(q.data_ptr(), 0, Q, D, 43)
bsr.synth_uniform(q[0:1].data_ptr(), 0, 1, D, 42)
torch.cuda.synchronize()
rec = np.load(sys.argv[1])
comm = bsr.Comm.loopback(0, P, 0, [rec[f"rec{i}"] for i in range(int(rec["n_rec"]))])
L = bsr.lib()
oi, od, oc = np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)
for _ in range(30):
    assert L.bsr_parallel_top_k_similarity_search(comm._h, ix._h, q.data_ptr(), Q, K, oi.ctypes.data,
                                                  od.ctypes.data, oc.ctypes.data) == 0, L.bsr_last_error()
print("loopback replayed / missed:", comm.loopback_stats(), "emitted per query", ix.last_stats().n_emitted / Q)
st = np.zeros((4096, 8), np.uint64)
L.bsr_lab_rescore_stamps.restype = ctypes.c_int
assert L.bsr_lab_rescore_stamps(st.ctypes.data_as(ctypes.c_void_p), 4096) == 0
s = st[:Q, :5].astype(np.int64)
t0 = s[:, 0].min()
us = (s - t0) / 100.0  # 100 MHz ticks -> us
print(f"rank 0 of {P}: {N} rows, {Q} queries, mode B (every emitted row), one wave per query (last of 30)")
print(f"wave start  (from the first): median {np.median(us[:, 0]):7.2f} us, max {us[:, 0].max():7.2f}")
print(f"wave end    (from the first): median {np.median(us[:, 4]):7.2f} us, max {us[:, 4].max():7.2f}")
names = ["query row -> LDS", "(no selection)", "score the emitted rows (12 chunks)", "finish (norms, sort, bound, write)"]
for i, nm in enumerate(names):
    d = us[:, i + 1] - us[:, i]
    print(f"  {nm:38s} median {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f} us")
tot = us[:, 4] - us[:, 0]
print(f"  {'wave total':38s} median {np.median(tot):7.2f}  p90 {np.percentile(tot, 90):7.2f}  max {tot.max():7.2f} us")
