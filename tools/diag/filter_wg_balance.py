"""Diagnostic (tooling): load balance of the persistent emit filter -- per-workgroup start and
end timestamps (s_memrealtime, 100 MHz) of the lab build (make -C better-search-rag-rust_amd
lab-counters -> tools/ab/libbsr_counters.so; run with BSR_LIB pointing at it).  With a static
tile partition the kernel ends with its slowest workgroup: mean/max of the workgroup times
is what perfect balancing could recover.
usage: BSR_LIB=tools/ab/libbsr_counters.so python tools/diag/filter_wg_balance.py [rows] [xcd_xor]
(xcd_xor: the lab build hands XCD x's row streams to XCD x ^ xcd_xor -- does a slow XCD stay
slow with other tiles?)"""
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
torch.cuda.synchronize()
L = bsr.lib()
L.bsr_lab_filter_wg_stamps.restype = ctypes.c_int
XOR = int(sys.argv[2]) if len(sys.argv) > 2 else 0
assert L.bsr_lab_set_xcd_xor(ctypes.c_uint32(XOR)) == 0
oi, od, oc = np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)
G = 256  # filter_grid(n_qt = 4)
runs = []
for it in range(14):
    assert L.bsr_local_top_k(ix._h, q.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data) == 0
    if it < 4:
        continue
    st = np.zeros((4096, 9), np.uint64)
    assert L.bsr_lab_filter_wg_stamps(st.ctypes.data_as(ctypes.c_void_p)) == 0
    s = st[:G].astype(np.int64)
    start, end = s[:, 0], s[:, 1:].max(axis=1)
    t0 = start.min()
    runs.append(((start - t0) / 100.0, (end - t0) / 100.0))
    tl = np.zeros((4096, 2), np.uint32)
    assert L.bsr_lab_filter_wg_tiles(tl.ctypes.data_as(ctypes.c_void_p)) == 0
    tiles = tl[:G].astype(np.int64)
print(f"rows {N}, {Q} queries, grid {G}; {len(runs)} launches; streams of XCD x on XCD x ^ {XOR}")
for i, (st, en) in enumerate(runs):
    dur = en - st
    span = en.max()
    print(f"launch {i}: span {span:8.1f} us | WG time min {dur.min():8.1f} med {np.median(dur):8.1f} "
          f"max {dur.max():8.1f} | start spread {st.max():5.1f} us | mean/max {dur.mean() / span:.4f}")
st, en = runs[-1]
dur = en - st
b = np.arange(G)
xcd, slot = b & 7, b >> 3
qt = slot % 4
print("last launch, mean WG time by XCD:", " ".join(f"{dur[xcd == x].mean():.0f}" for x in range(8)))
print("last launch, mean WG time by query tile:", " ".join(f"{dur[qt == t].mean():.0f}" for t in range(4)))
tot, stat = tiles[:, 0], tiles[:, 1]
print(f"last launch, tiles per WG: min {tot.min()} max {tot.max()} | static {stat.min()}-{stat.max()} | "
      f"tail tiles per WG min {(tot - stat).min()} max {(tot - stat).max()}")
print("last launch, tail tiles by XCD:", " ".join(f"{(tot - stat)[xcd == x].mean():.1f}" for x in range(8)))
srt = np.argsort(dur)[::-1][:8]
print("slowest WGs (block: us):", ", ".join(f"{int(i)}: {dur[i]:.0f}" for i in srt))
