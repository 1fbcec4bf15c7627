"""Diagnostic (tooling): the configs[3] test's searches (4 single queries over the 10M synthetic
corpus, two planted, three repetitions) with their per-search stats, under whatever A/B variables
the environment sets (BSR_SELECT_TAU_M, BSR_SOLO_PUB, BSR_RESCORE_KP)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import torch  # noqa: E402
import bsr  # noqa: E402

D, N, K = 768, 10_000_000, 10
rows = torch.empty((N, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(rows.data_ptr(), 0, N, D, 42)
torch.cuda.synchronize()
ix = bsr.Index(D, max_k=16, device=0)
ix.load(rows, 0)
del rows
torch.cuda.empty_cache()
q = torch.empty((4, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(q.data_ptr(), 0, 4, D, 43)
for pos, row in ((0, 0), (3, N - 2)):
    bsr.synth_uniform(q[pos:pos + 1].data_ptr(), row, 1, D, 42)
torch.cuda.synchronize()
qs = q.cpu().numpy()
env = {k: v for k, v in os.environ.items() if k in ("BSR_SELECT_TAU_M", "BSR_SOLO_PUB", "BSR_RESCORE_KP")}
first = {}
for rep in range(3):
    for j in range(4):
        gi, gd, gc = ix.local_top_k(qs[j:j + 1], K)
        st = ix.last_stats()
        same = ""
        if rep == 0:
            first[j] = (gi.copy(), gd.copy())
        else:
            same = " same-as-rep0" if np.array_equal(first[j][0], gi) and np.array_equal(first[j][1].view(np.uint32), gd.view(np.uint32)) else " DIFFERENT"
        print(f"{env} rep {rep} q{j}: emitted {st.n_emitted} rescued {st.n_rescued} fallback {st.n_fallback} "
              f"replay {st.graph_replay} top {gi[0, :3].tolist()}{same}", flush=True)
