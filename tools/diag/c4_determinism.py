"""configs[4] shard (6.25M bf16 rows x 4096 queries, top-100) searched several times in one
process: per-run stats (fallbacks, second-chance rescues, emitted rows) and bitwise equality
of the results across runs (tooling: determinism check)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import torch  # noqa: E402  (before libbsr: one HIP runtime)
import bsr  # noqa: E402

D, n, nq, k = 768, 6_250_000, 4096, 100
rows = torch.empty((n, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(rows.data_ptr(), 0, n, D, 42)
torch.cuda.synchronize()
rows = rows.to(torch.bfloat16)
ix = bsr.Index(D, max_k=k, device=0, dtype=bsr.BSR_BF16)
ix.load(rows, 0)
del rows
torch.cuda.empty_cache()
q = torch.empty((nq, D), dtype=torch.float32, device="cuda:0")
bsr.synth_uniform(q.data_ptr(), 0, nq, D, 43)
torch.cuda.synchronize()
oi = torch.empty((nq, k), dtype=torch.int64, device="cuda:0")
od = torch.empty((nq, k), dtype=torch.float32, device="cuda:0")
oc = torch.empty(nq, dtype=torch.int32, device="cuda:0")
ref = None
for r in range(int(sys.argv[1]) if len(sys.argv) > 1 else 4):
    ix.local_top_k_device(q, nq, k, oi, od, oc)
    st = ix.last_stats()
    got = (oi.cpu().numpy().copy(), od.cpu().numpy().copy(), oc.cpu().numpy().copy())
    same = None if ref is None else all(np.array_equal(a, b) for a, b in zip(ref, got))
    ref = ref or got
    print(f"run {r}: fallback {st.n_fallback} rescued {st.n_rescued} emitted {st.n_emitted} "
          f"graph {st.graph_replay} identical_to_run0 {same}", flush=True)
