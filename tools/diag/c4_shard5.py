"""Diagnostic (tooling): configs[4] shard 5 (rows 31.25M..37.5M of the 50M bf16 corpus) x the
4096-query batch of tests/test_gpu_full_size.py, k = 100.  Round 3's 50M test found the
global top-100 of query 0 missing row 37,467,117 (shard 5, local row 6,217,117).  This
searches shard 5 alone: the batch (repeated), query 0 alone, and an exact-only index, each
against the oracle over the shard for a few queries, and prints the search stats."""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
for p in (os.path.join(ROOT, "better-search-rag-rust_amd"), os.path.join(ROOT, "oracle"), ROOT):
    sys.path.insert(0, p)
import torch  # noqa: E402  (before libbsr)
import bsr  # noqa: E402
import oracle  # noqa: E402

D, K, NQ = 768, 100, 4096
N, P, R = 50_000_000, 8, int(sys.argv[1]) if len(sys.argv) > 1 else 5
iv = bsr.interval_by_rank(R, P, N)
s, cnt = iv.start_index, iv.get_count()
print(f"shard {R}: rows [{s}, {s + cnt})", flush=True)


def gen(n, row0, seed=42, bf16=False):
    t = torch.empty((n, D), dtype=torch.float32, device="cuda:0")
    bsr.synth_uniform(t.data_ptr(), row0, n, D, seed)
    torch.cuda.synchronize()
    return t.to(torch.bfloat16) if bf16 else t


q = gen(NQ, 0, seed=43)
for pos, row in [(0, 0), (1, N - 1), (2, 43_750_123), (3, 6_250_000), (4, 31_000_007)]:
    q[pos] = gen(1, row, bf16=True).to(torch.float32)[0]
torch.cuda.synchronize()
rows = gen(cnt, s, bf16=True)
rows_h = rows.to(torch.float32).cpu().numpy()
ix = bsr.Index(D, max_k=K, device=0, dtype=bsr.BSR_BF16)
ix.load(rows, s)
print("loaded", flush=True)

sub = [0, 1, 2, 3, 4, 5, 100, 4095]
t0 = time.time()
wi, wd, wc = oracle.parallel_top_k(rows_h, q[sub].cpu().numpy(), K, size=16, threads=16)
wi = wi + np.uint64(s)
print(f"oracle {time.time() - t0:.1f}s", flush=True)


def search(qq, n):
    oi = torch.empty((n, K), dtype=torch.int64, device="cuda:0")
    od = torch.empty((n, K), dtype=torch.float32, device="cuda:0")
    oc = torch.empty(n, dtype=torch.int32, device="cuda:0")
    ix.local_top_k_device(qq, n, K, oi, od, oc)
    st = ix.last_stats()
    return (oi.cpu().numpy().astype(np.uint64), od.cpu().numpy(), oc.cpu().numpy()), st


def report(tag, got, st, rowsel):
    gi, gd, gc = got
    bad = []
    for j, qi in enumerate(rowsel):
        c = int(wc[j])
        ok = gc[qi] == c and np.array_equal(gi[qi, :c], wi[j, :c]) and \
            np.array_equal(gd[qi, :c].view(np.uint32), wd[j, :c].view(np.uint32))
        if not ok:
            miss = sorted(set(wi[j, :c].tolist()) - set(gi[qi, :c].tolist()))
            extra = sorted(set(gi[qi, :c].tolist()) - set(wi[j, :c].tolist()))
            bad.append((sub[j], miss[:5], extra[:5]))
    print(f"{tag}: fallback {st.n_fallback} rescued {st.n_rescued} exact_direct {st.n_exact_direct} "
          f"emitted/q {st.n_emitted / max(st.n_queries, 1):.0f} graph {st.graph_replay} ebound {st.row_ebound:.6f} "
          f"bad {bad}", flush=True)


for rep in range(3):
    got, st = search(q, NQ)
    report(f"batch rep {rep}", got, st, sub)
got, st = search(q[:1].contiguous(), 1)
report("query 0 alone", got, st, [0])
got, st = search(q[:64].contiguous(), 64)
report("first 64 queries", got, st, [i for i in range(6)])
ix.close()
ix = bsr.Index(D, max_k=K, device=0, dtype=bsr.BSR_BF16, flags=bsr.BSR_FLAG_EXACT_ONLY)
ix.load(rows, s)
got, st = search(q[:8].contiguous(), 8)
report("exact-only, first 8", got, st, [0, 1, 2, 3, 4, 5])
