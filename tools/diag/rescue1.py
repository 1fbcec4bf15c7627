"""Diagnostic (tooling): test_published_rescue_and_fallback_rows' single-query case (one query,
200 near-duplicates of it among 60k rows) with its per-search stats, under the tiny-batch A/B
variables the environment sets (BSR_SELECT_TAU_M, BSR_SOLO_PUB, BSR_RESCORE_KP)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import bsr  # noqa: E402

nq_all = int(sys.argv[1]) if len(sys.argv) > 1 else 1
m_dup = int(sys.argv[2]) if len(sys.argv) > 2 else 200
rng = np.random.default_rng(404)
n, dim, k = 60000, 768, 10
rows = rng.uniform(-1, 1, (n, dim)).astype(np.float32)
qs = rng.uniform(-1, 1, (nq_all, dim)).astype(np.float32)
perm = rng.permutation(n)
rows[perm[:m_dup]] = qs[0] + rng.normal(0, 1e-3, (m_dup, dim)).astype(np.float32)
ix = bsr.Index(dim, max_k=64, device=0)
ix.load(rows, 0)
env = {e: v for e, v in os.environ.items() if e in ("BSR_SELECT_TAU_M", "BSR_SOLO_PUB", "BSR_RESCORE_KP")}
for rep in range(3):
    gi, gd, gc = ix.local_top_k(qs, k)
    st = ix.last_stats()
    print(f"{env} nq {nq_all} dups {m_dup} rep {rep}: emitted {st.n_emitted} rescued {st.n_rescued} fallback {st.n_fallback} "
          f"replay {st.graph_replay} top {gi[0, :3].tolist()}", flush=True)
