"""Diagnostic (tooling): the single-query search's rescore kernels (profile level 2 events), for
the A/B of the tiny-batch rescore (BSR_RESCORE_KP=1, k_rescore_kp) against the one-wave kernel
(BSR_RESCORE_KP=0).  The variable is read once per process: run once per setting.
usage: python tools/diag/p50_rescore.py [rows] [queries per search]"""
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import torch  # noqa: E402
import bsr  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
Q = int(sys.argv[2]) if len(sys.argv) > 2 else 1
D, K, NS = 768, 10, 200
rows = torch.empty((N, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(rows.data_ptr(), 0, N, D, 42)
torch.cuda.synchronize()
ix = bsr.Index(D, max_k=64, device=0, flags=bsr.BSR_FLAG_PROFILE)
ix.load(rows, 0)
del rows
torch.cuda.empty_cache()
q = torch.empty((NS, Q, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(q.data_ptr(), 0, NS * Q, D, 43)
torch.cuda.synchronize()
L = bsr.lib()
oi, od, oc = np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)


def call(i):
    st = L.bsr_local_top_k(ix._h, q[i].data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
    assert st == 0, L.bsr_last_error()


ix.set_profile(0)
for i in range(NS):
    call(i)
walls = []
for i in range(NS):
    t0 = time.perf_counter()
    call(i)
    walls.append((time.perf_counter() - t0) * 1e6)
ix.set_profile(2)
ix.profile(reset=True)
for i in range(NS):
    call(i)
p = ix.profile(reset=True)
print(f"kp={os.environ.get('BSR_RESCORE_KP', '1')} rows {N} queries {Q}: wall median {statistics.median(walls):.1f} us "
      f"| level-2 span {p.search_ms / max(p.searches, 1) * 1e3:.1f} us, rescore {p.rescore_ms / max(p.rescore_launches, 1) * 1e3:.1f} us "
      f"x {p.rescore_launches / max(p.searches, 1):.2f}/search, emit {p.gemm_emit_ms / max(p.gemm_emit_launches, 1) * 1e3:.1f} us",
      flush=True)
if os.environ.get("BSR_READ_STAMPS") == "1":
    # the lab build's per-query phase stamps of the last search (make lab-stamps; kp kernel:
    # 0 start, 5 keys arrived, 1 select, 2 rows of chunk 0 in LDS, 3 the 12 chunks walked, 4 finish)
    import ctypes
    st = np.zeros((4096, 8), np.uint64)
    L.bsr_lab_rescore_stamps.restype = ctypes.c_int
    assert L.bsr_lab_rescore_stamps(st.ctypes.data_as(ctypes.c_void_p), 4096) == 0
    s = st[:Q, :8].astype(np.int64)
    us = (s - s[:, :1]) / 100.0
    phases = [("keys arrive", 5, 0), ("select", 1, 5), ("rows -> LDS", 2, 1), ("walk chunks", 3, 2), ("finish", 4, 3)]
    if s[0, 6] and s[0, 7]:  # (the self-thresholded path: the selection's own stamps)
        phases[1:2] = [("  keys in, X", 6, 5), ("  lists, heads, H", 7, 6), ("  candidates", 1, 7)]
    for nm, i, j in phases:
        d = us[:, i] - us[:, j]
        print(f"  {nm:16s} median {np.median(d):7.2f} max {d.max():7.2f} us", flush=True)
    print(f"  {'total':16s} median {np.median(us[:, 4]):7.2f} max {us[:, 4].max():7.2f} us", flush=True)
