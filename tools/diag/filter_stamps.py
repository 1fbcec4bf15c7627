"""Diagnostic (tooling): where the emit filter's time goes, from s_memtime phase sums of the
lab build (make -C better-search-rag-rust_amd lab-fstamps -> tools/ab/libbsr_fstamps.so; run
with BSR_LIB pointing at it).  Per wave and tile: the level-1 epilogue, the level-2 epilogue
(per entry), the first barrier after the epilogue (kt = 1: where the workgroup waits for its
slowest wave's epilogue) and the other barriers, against the loop's total.  Stamps fence the
instruction stream (each drains the LDS reads in flight), so read shares, not lengths.
usage: BSR_LIB=tools/ab/libbsr_fstamps.so python tools/diag/filter_stamps.py [rows]"""
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
oi, od, oc = np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)
st = np.zeros(8, np.uint64)
for it in range(30):
    if it == 10:
        assert L.bsr_lab_filter_stamps(st.ctypes.data_as(ctypes.c_void_p), 1) == 0
    assert L.bsr_local_top_k(ix._h, q.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data) == 0
assert L.bsr_lab_filter_stamps(st.ctypes.data_as(ctypes.c_void_p), 0) == 0
s = st.astype(np.float64)
launches, waves = 20, 2048
l1, l2, n2, b1, bo, loop, vm, tiles = s
nb = tiles * 6
print(f"rows {N}, {Q} queries, top-{K}: {launches} launches, {waves} waves; emitted per query "
      f"{ix.last_stats().n_emitted / Q:.1f}")
print(f"wave-tiles {tiles:.0f} ({tiles / launches / waves:.1f} per wave per launch); level-2 entries {n2:.0f} "
      f"({n2 / tiles:.4f} of wave-tiles)")
per = loop / tiles
print(f"loop cycles per wave-tile {per:8.0f}  (includes ~40-cycle stamp pairs: {(tiles * 2 + nb * 2) * 40 / tiles:.0f} per tile)")
for name, v in (("level-1 epilogue", l1), ("level-2 epilogue", l2), ("barrier kt=1 (after epilogue)", b1),
                ("other barriers", bo), ("DMA waits (vmcnt) before barriers", vm)):
    print(f"  {name:32s} {v / tiles:8.1f} cycles per wave-tile = {v / loop:6.2%} of the loop")
print(f"  level-2 cycles per entry {l2 / max(n2, 1):8.1f}")
rest = loop - l1 - l2 - b1 - bo - vm
print(f"  MFMA stream + DMA + reads (rest)  {rest / tiles:8.1f} cycles per wave-tile = {rest / loop:6.2%}; "
      f"bare MFMA issue per wave-tile = 192 x 16 x 2 waves/SIMD = {192 * 16 * 2} SIMD cycles")
