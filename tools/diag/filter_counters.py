"""Diagnostic (tooling): how often the emit filter's epilogue levels fire, from the event
counters of the lab build (make -C better-search-rag-rust_amd lab-counters ->
tools/ab/libbsr_counters.so; run with BSR_LIB pointing at it).  Per (wave, row tile): level 1
(any of the wave's 64 lanes' integer maxima, scored with the tile's extreme block scale,
reaches tau), per query block (16 queries) the level-2 entry, per (query block, 16-row
block) a passing row block (its 4 rows per lane appended).
usage: BSR_LIB=tools/ab/libbsr_counters.so python tools/diag/filter_counters.py [rows]"""
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
L.bsr_lab_filter_counters.restype = ctypes.c_int
oi, od, oc = np.empty((Q, K), np.uint64), np.empty((Q, K), np.float32), np.empty(Q, np.uint32)
for _ in range(5):
    assert L.bsr_local_top_k(ix._h, q.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data) == 0
c = np.zeros(8, np.uint64)
assert L.bsr_lab_filter_counters(c.ctypes.data_as(ctypes.c_void_p), 1) == 0
S = 10
em = 0
for _ in range(S):
    assert L.bsr_local_top_k(ix._h, q.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data) == 0
    em += ix.last_stats().n_emitted
assert L.bsr_lab_filter_counters(c.ctypes.data_as(ctypes.c_void_p), 1) == 0
tiles, l1, nbp, rbp = (int(x) for x in c[:4])
print(f"rows {N}, {Q} queries, {S} searches")
print(f"(wave, tile) epilogues per search {tiles / S:12.0f}")
print(f"level 1 passes (wave ballot)      {l1 / tiles:8.4f} of the wave-tiles")
print(f"level 2 entries (query block)     {nbp / (2 * tiles):8.4f} of the (wave-tile, query block)s")
print(f"passing 16-row blocks             {rbp / (16 * tiles):8.5f} of the (wave-tile, query block, row block)s")
print(f"emitted rows per query            {em / S / Q:8.1f}  (appended rows checked: {rbp * 64 / S / Q:.0f} per query)")
