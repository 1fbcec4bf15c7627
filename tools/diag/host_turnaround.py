"""Diagnostic (tooling): where the per-batch time outside the kernels goes, at the 1.25M-row
shard of an 8-GPU configs[2] run (1000 queries, top-10).  Wall time per search vs the GPU
span of the same search (prep start -> result copy, events at profile level 2), for host
(numpy) outputs, device (torch) outputs and pinned host outputs, through bsr_local_top_k
and bsr_parallel_top_k_similarity_search (comm = NULL)."""
import ctypes
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import torch  # noqa: E402
import bsr  # noqa: E402

N, D, Q, K = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000, 768, 1000, 10
rows = torch.empty((N, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(rows.data_ptr(), 0, N, D, 42)
torch.cuda.synchronize()
ix = bsr.Index(D, max_k=64, device=0, flags=bsr.BSR_FLAG_PROFILE)
ix.load(rows, 0)
del rows
torch.cuda.empty_cache()
q = torch.empty((Q, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(q.data_ptr(), 0, Q, D, 43)
torch.cuda.synchronize()
L = bsr.lib()

outs = {
    "numpy": (np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)),
    "pinned": (torch.empty((Q, K), dtype=torch.int64, pin_memory=True),
               torch.empty((Q, K), dtype=torch.float32, pin_memory=True),
               torch.empty(Q, dtype=torch.int32, pin_memory=True)),
    "device": (torch.empty((Q, K), dtype=torch.int64, device="cuda:0"),
               torch.empty((Q, K), dtype=torch.float32, device="cuda:0"),
               torch.empty(Q, dtype=torch.int32, device="cuda:0")),
}


def ptrs(o):
    return [a.ctypes.data if isinstance(a, np.ndarray) else a.data_ptr() for a in o]


for name, o in outs.items():
    oi, od, oc = ptrs(o)
    for fn in ("local", "parallel"):
        def call():
            if fn == "local":
                st = L.bsr_local_top_k(ix._h, q.data_ptr(), Q, K, oi, od, oc)
            else:
                st = L.bsr_parallel_top_k_similarity_search(None, ix._h, q.data_ptr(), Q, K, oi, od, oc)
            assert st == 0, L.bsr_last_error()
        ix.set_profile(0)
        for _ in range(200):
            call()
        walls = []
        for _ in range(200):
            t0 = time.perf_counter()
            call()
            walls.append((time.perf_counter() - t0) * 1e6)
        ix.set_profile(2)
        ix.profile(reset=True)
        for _ in range(50):
            call()
        p = ix.profile(reset=True)
        span = p.search_ms / max(p.searches, 1) * 1e3
        emit = p.gemm_emit_ms / max(p.gemm_emit_launches, 1) * 1e3
        print(f"{name:7s} {fn:8s} wall median {statistics.median(walls):8.1f} us  min {min(walls):8.1f} us | "
              f"level-2 GPU span {span:8.1f} us (emit {emit:7.1f} us, sample {p.gemm_sample_ms / max(p.gemm_sample_launches, 1) * 1e3:6.1f},"
              f" rescore {p.rescore_ms / max(p.rescore_launches, 1) * 1e3:6.1f})", flush=True)
# graph-launch + wait floor: the smallest search (1 row index, 1 query)
ix1 = bsr.Index(D, max_k=16, device=0)
ix1.load(np.random.default_rng(0).uniform(-1, 1, (1, D)).astype(np.float32))
o = outs["numpy"]
oi, od, oc = ptrs(o)
for _ in range(100):
    L.bsr_local_top_k(ix1._h, q.data_ptr(), 1, 1, oi, od, oc)
w = []
for _ in range(300):
    t0 = time.perf_counter()
    L.bsr_local_top_k(ix1._h, q.data_ptr(), 1, 1, oi, od, oc)
    w.append((time.perf_counter() - t0) * 1e6)
print(f"1-row index, 1 query: wall median {statistics.median(w):.1f} us", flush=True)
w = []
for _ in range(300):
    t0 = time.perf_counter()
    L.bsr_index_count(ix1._h, ctypes.byref(ctypes.c_uint64()))
    w.append((time.perf_counter() - t0) * 1e6)
print(f"ctypes call floor: {statistics.median(w):.2f} us", flush=True)
