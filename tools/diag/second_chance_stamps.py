"""Diagnostic (tooling): where the second chance's time goes at 10M x 1000 (the batch's last kernel,
k_rescore<E, 8, 2>: the queries that failed the first pass, every row they emitted), from the lab
stamps build (make -C better-search-rag-rust_amd lab-stamps; BSR_LIB=tools/ab/libbsr_stamps.so).
Per failed item (slots 2048 +): 0 start, 1 query in LDS, 3 rows scored, 4 list / rows written; the
publishing workgroup: its publish start and its flag (slot 4095).
usage: BSR_LIB=tools/ab/libbsr_stamps.so python tools/diag/second_chance_stamps.py [rows]"""
import ctypes
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import torch  # noqa: E402
import bsr  # noqa: E402

N, D, Q, K = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000, 768, 1000, 10
rows = torch.empty((N, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(rows.data_ptr(), 0, N, D, 42)
torch.cuda.synchronize()
ix = bsr.Index(D, max_k=64, device=0)
ix.load(rows, 0)
del rows
torch.cuda.empty_cache()
q = torch.empty((Q, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(q.data_ptr(), 0, Q, D, 43)
bsr.synth_uniform(q[0:1].data_ptr(), 0, 1, D, 42)
torch.cuda.synchronize()
L = bsr.lib()
oi, od, oc = np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)
for _ in range(20):
    assert L.bsr_local_top_k(ix._h, q.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data) == 0
stt = ix.last_stats()
st = np.zeros((4096, 8), np.uint64)
L.bsr_lab_rescore_stamps.restype = ctypes.c_int
assert L.bsr_lab_rescore_stamps(st.ctypes.data_as(ctypes.c_void_p), 4096) == 0
n = int(stt.n_rescued) + int(stt.n_fallback)
first = st[:Q, :5].astype(np.int64)
t0 = first[:, 0].min()
print(f"rows {N}, {Q} queries: rescued {stt.n_rescued}, fallback {stt.n_fallback}; first pass waves "
      f"{(first[:, 0].min() - t0) / 100:.2f} .. {(first[:, 4].max() - t0) / 100:.2f} us", flush=True)
for i in range(max(n, 2)):
    s = st[2048 + i, :5].astype(np.int64)
    if s[0] == 0:
        continue
    us = (s - t0) / 100.0
    print(f"second-chance item {i}: start {us[0]:.2f}, query in LDS +{us[1] - us[0]:.2f}, rows scored "
          f"+{us[3] - us[1]:.2f}, list and rows +{us[4] - us[3]:.2f} (end {us[4]:.2f} us)", flush=True)
p = st[4095, :2].astype(np.int64)
if p[0]:
    print(f"publish: start {(p[0] - t0) / 100:.2f}, flag {(p[1] - t0) / 100:.2f} us", flush=True)
