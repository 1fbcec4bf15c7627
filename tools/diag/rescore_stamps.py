"""Diagnostic (tooling): where the one-wave-per-query rescore's time goes, from per-wave phase
timestamps (s_memrealtime, 100 MHz) of the lab build (make -C better-search-rag-rust_amd
lab-stamps -> tools/ab/libbsr_stamps.so, run with BSR_LIB pointing at it).
Phases per wave: 0 start, 1 query row in LDS, 2 candidates selected, 3 rows scored,
4 list stored / certified / result rows written.
usage: BSR_LIB=tools/ab/libbsr_stamps.so python tools/diag/rescore_stamps.py [rows]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import torch  # noqa: E402
import bsr  # noqa: E402

N, D, Q, K = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000, 768, 1000, 10
rows = torch.empty((N, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(rows.data_ptr(), 0, N, D, 42)
torch.cuda.synchronize()
ix = bsr.Index(D, max_k=64, device=0)
ix.load(rows, 0)
del rows
torch.cuda.empty_cache()
q = torch.empty((Q, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(q.data_ptr(), 0, Q, D, 43)
torch.cuda.synchronize()
L = bsr.lib()
oi, od, oc = np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)
for _ in range(30):
    assert L.bsr_local_top_k(ix._h, q.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data) == 0
st = np.zeros((4096, 8), np.uint64)
L.bsr_lab_rescore_stamps.restype = ctypes.c_int
assert L.bsr_lab_rescore_stamps(st.ctypes.data_as(ctypes.c_void_p), 4096) == 0
s = st[:Q, :5].astype(np.int64)
t0 = s[:, 0].min()
us = (s - t0) / 100.0  # 100 MHz ticks -> us
print(f"rows {N}, {Q} queries, one wave per query (last of 30 searches)")
print(f"wave start  (from the first): median {np.median(us[:, 0]):7.2f} us, max {us[:, 0].max():7.2f}")
print(f"wave end    (from the first): median {np.median(us[:, 4]):7.2f} us, max {us[:, 4].max():7.2f}")
names = ["query row -> LDS", "select k' candidates", "score 63 rows (12 chunks)", "finish (norms, sort, certify, write)"]
for i, nm in enumerate(names):
    d = us[:, i + 1] - us[:, i]
    print(f"  {nm:38s} median {np.median(d):7.2f}  p90 {np.percentile(d, 90):7.2f}  max {d.max():7.2f} us")
tot = us[:, 4] - us[:, 0]
print(f"  {'wave total':38s} median {np.median(tot):7.2f}  p90 {np.percentile(tot, 90):7.2f}  max {tot.max():7.2f} us")
