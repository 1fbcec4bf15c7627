"""GPU parity over a seeded random sweep of shapes and data (round 6): corpus sizes from 1 row to
~600k, widths from 1 to 1100, batches of 1 to 300 queries, k from 1 to 256, one to five shards
merged as the reference merges rank blocks (src/mpi_helpers/metrics.rs:141-171), and data that
stresses the filter's certification: near-duplicate clusters, integer-valued rows (exact distance
ties, broken by index), rows scaled over six decades, duplicate and zero rows, queries that copy
or scale corpus rows and zero queries.  Every case is compared with the oracle bit for bit
(indices, order, f32 distance bits); each case's oracle work is bounded to a few seconds."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

DIMS = [1, 2, 7, 31, 64, 100, 257, 384, 768, 1000, 1024, 1100]
NQS = [1, 2, 5, 16, 17, 33, 100, 300]
KS = [1, 2, 10, 33, 64, 100, 200, 256]
KINDS = ["uniform", "clusters", "integers", "scaled"]
N_CASES = 24
OPS_CAP = 2.0e9  # n * nq * dim per case (the oracle's work)


def _case(i):
    rng = np.random.default_rng(20261018 + i)
    dim = int(rng.choice(DIMS))
    nq = int(rng.choice(NQS))
    k = int(rng.choice(KS))
    kind = KINDS[i % len(KINDS)]
    n_max = max(1, min(600_000, int(OPS_CAP / (nq * dim))))
    n = int(np.exp(rng.uniform(0.4, 1.0) * np.log(n_max + 1.0)))  # (mostly past the candidate cap)
    n = max(1, min(n, n_max))
    P = int(rng.choice([1, 1, 2, 3, 5]))
    return rng, dim, nq, k, kind, n, P


def _data(rng, kind, n, dim, nq):
    if kind == "uniform":
        rows = rng.uniform(-1, 1, (n, dim))
    elif kind == "clusters":
        c = rng.uniform(-1, 1, (int(rng.integers(4, 33)), dim))
        rows = c[rng.integers(0, len(c), n)] + 0.05 * rng.standard_normal((n, dim))
    elif kind == "integers":
        rows = rng.integers(-2, 3, (n, dim)).astype(np.float64)
    else:
        rows = rng.uniform(-1, 1, (n, dim)) * 10.0 ** rng.uniform(-3, 3, (n, 1))
    rows = rows.astype(np.float32)
    if n > 8:
        rows[n - 1] = rows[1]        # a duplicate pair far apart
        rows[4] = 0                  # a zero row
    if kind == "integers":
        qs = rng.integers(-2, 3, (nq, dim)).astype(np.float32)
    else:
        qs = rng.uniform(-1, 1, (nq, dim)).astype(np.float32)
    for j in range(nq):
        r = int(rng.integers(0, n))
        pick = j % 5
        if pick == 1:
            qs[j] = rows[r]                          # a corpus row: distance 0 leads
        elif pick == 2:
            qs[j] = rows[r] * np.float32(3.0)        # a scaled corpus row
        elif pick == 3 and j > 0 and j % 15 == 3:
            qs[j] = 0                                # a zero query: the exact scan
    return rows, qs


@pytest.mark.parametrize("i", range(N_CASES))
def test_random_sweep_vs_oracle(bsr_mod, oracle_mod, gpu, i):
    rng, dim, nq, k, kind, n, P = _case(i)
    rows, qs = _data(rng, kind, n, dim, nq)
    ctx = f"case {i}: n={n} dim={dim} nq={nq} k={k} kind={kind} P={P}"
    li = np.zeros((P, nq, k), np.uint64)
    ld = np.zeros((P, nq, k), np.float32)
    lc = np.zeros((P, nq), np.uint32)
    for r in range(P):
        iv = bsr_mod.interval_by_rank(r, P, n)
        s, e = iv.start_index, max(iv.start_index, iv.end_index)
        if s >= n or e <= s:
            continue  # (an empty block: the reference's rank contributes nothing)
        ix = bsr_mod.Index(dim, max_k=256, device=0)
        ix.load(rows[s:e], s)
        li[r], ld[r], lc[r] = ix.local_top_k(qs, k)
        ix.close()
    got = bsr_mod.merge_top_k_lists(li, ld, lc, k) if P > 1 else (li[0], ld[0], lc[0])
    wi, wd, wc = oracle_mod.parallel_top_k(rows, qs, k, size=P, threads=8)
    gi, gd, gc = got
    assert np.array_equal(gc, wc), (ctx, gc, wc)
    for q in range(nq):
        c = int(wc[q])
        assert np.array_equal(gi[q, :c], wi[q, :c]), (ctx, q, gi[q, :c], wi[q, :c])
        assert np.array_equal(gd[q, :c].view(np.uint32), wd[q, :c].view(np.uint32)), (ctx, q)
