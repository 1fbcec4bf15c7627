# Diagnostic (tooling): does torch's CUDA init still work after the library captured a search graph?
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "better-search-rag-rust_amd"))
import bsr
n_search = int(sys.argv[1])
rng = np.random.default_rng(1)
rows = rng.uniform(-1, 1, (20000, 768)).astype(np.float32)
ix = bsr.Index(768, max_k=16, device=0)
ix.load(rows)
rep = 0
for _ in range(n_search):
    ix.local_top_k(rng.uniform(-1, 1, (1, 768)).astype(np.float32), 10)
    rep += ix.last_stats().graph_replay
import torch
print("searches", n_search, "replays", rep, "torch device_count", torch.cuda.device_count(), "available", torch.cuda.is_available(), flush=True)
t = torch.empty(4, device="cuda:0")
print("torch ok", flush=True)
