"""The self-thresholded single-query path (round 6, DESIGN.md §5 tiny batches): a batch of <= 16
queries over a shard of >= 2^21 rows (k' <= 63, i.e. k <= 10) takes no sample pass and no tau0.
The skinny filter keeps every workgroup's 4 best (score, row) keys per query over strided pairs of
rows; the tiny-batch rescore selects the k' best of those 512 lists with a radix select, and
certifies against max(the (k'+1)-th score, the best 4th key) -- every row a workgroup left out
scores at most its 4th.  A query that fails takes the second chance (every listed key above that
bound, exactly rescored); one that fails again sends the batch through the thresholded path
(sample pass, tau0, emit), whose own failures take the exact scan.

Everything is bit-exact against the oracle over the whole shard (src/metrics.rs:143-165,
src/mpi_helpers/metrics.rs:16-53) and against BSR_SKINNY_TOP=0, the thresholded path."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

D = 768
N = 2_300_017           # > 2^21 rows, not a multiple of 16 (a partial last unit)
THREADS = 16


def _same(got, want, ctx):
    gi, gd, gc = got
    wi, wd, wc = want
    assert np.array_equal(gc, wc), (ctx, gc, wc)
    for q in range(len(wc)):
        c = int(wc[q])
        assert np.array_equal(gi[q, :c], wi[q, :c]), (ctx, q, gi[q, :c], wi[q, :c])
        assert np.array_equal(gd[q, :c].view(np.uint32), wd[q, :c].view(np.uint32)), (ctx, q)


@pytest.fixture(scope="module")
def shard(bsr_mod, gpu):
    """N synthetic rows (the counter-based generator) with planted near-duplicate clusters of
    queries 0-2 of the fixture's query set: 150 scattered rows (q0), a run of 300 consecutive
    rows (q1), 5000 scattered rows (q2).  Returns (index, host rows, queries)."""
    import torch
    rows = torch.empty((N, D), dtype=torch.float32, device="cuda:0")
    bsr_mod.synth_uniform(rows.data_ptr(), 0, N, D, 42)
    q = torch.empty((16, D), dtype=torch.float32, device="cuda:0")
    bsr_mod.synth_uniform(q.data_ptr(), 0, 16, D, 43)
    g = torch.Generator(device="cuda:0")
    g.manual_seed(7)
    perm = torch.randperm(N, generator=g, device="cuda:0")
    plant = [(0, perm[:150]), (1, torch.arange(1_000_003, 1_000_303, device="cuda:0")),
             (2, perm[150:5150])]
    for j, idx in plant:
        rows[idx] = q[j] + 1e-3 * torch.randn((len(idx), D), generator=g, device="cuda:0")
    q[5] = rows[N - 1]   # self-matches: the last row (the partial last unit) and a middle one
    q[6] = rows[N // 3]
    torch.cuda.synchronize()
    ix = bsr_mod.Index(D, max_k=64, device=0)
    ix.load(rows)
    host = rows.cpu().numpy()
    qh = q.cpu().numpy()
    del rows
    torch.cuda.empty_cache()
    yield ix, host, qh
    ix.close()


def _oracle(oracle_mod, host, qs, k):
    return oracle_mod.parallel_top_k(host, np.ascontiguousarray(qs), k, size=THREADS, threads=THREADS)


@pytest.mark.parametrize("sel,k", [([3], 10), ([4, 5, 6, 7], 10), (list(range(3, 16)), 10), ([3, 5], 1),
                                   ([8], 7)])
def test_top_path_matches_oracle(bsr_mod, oracle_mod, shard, sel, k):
    """Plain queries (no planted cluster): certified on the first pass, no sample pass, graph
    replays after the first two searches; identical to the thresholded path and the oracle."""
    ix, host, qh = shard
    qs = np.ascontiguousarray(qh[sel])
    want = _oracle(oracle_mod, host, qs, k)
    for rep in range(3):
        got = ix.local_top_k(qs, k)
        st = ix.last_stats()
        assert st.search_path & bsr_mod.BSR_PATH_SKINNY_TOP, st.search_path
        assert not st.search_path & bsr_mod.BSR_PATH_TOP_RERUN
        assert st.n_fallback == 0, st.n_fallback
        _same(got, want, f"top {sel} k={k} rep {rep}")
    assert st.graph_replay == 1
    if 5 in sel:
        assert got[0][sel.index(5), 0] == N - 1 and got[1][sel.index(5), 0] == 0.0


def test_top_path_off_switch(bsr_mod, oracle_mod, shard, monkeypatch):
    """BSR_SKINNY_TOP=0: the thresholded path (sample pass, tau0), the same bits."""
    ix, host, qh = shard
    qs = np.ascontiguousarray(qh[[3, 9]])
    want = _oracle(oracle_mod, host, qs, 10)
    monkeypatch.setenv("BSR_SKINNY_TOP", "0")
    got = ix.local_top_k(qs, 10)
    assert not ix.last_stats().search_path & bsr_mod.BSR_PATH_SKINNY_TOP
    _same(got, want, "thresholded")
    monkeypatch.delenv("BSR_SKINNY_TOP")
    got = ix.local_top_k(qs, 10)
    assert ix.last_stats().search_path & bsr_mod.BSR_PATH_SKINNY_TOP
    _same(got, want, "self-thresholded")


@pytest.mark.parametrize("top", ["1", "0"])
def test_skinny_filter_kernels_agree(bsr_mod, oracle_mod, shard, monkeypatch, top):
    """768-byte rows take the LDS-DMA skinny filter (k_filter_skinny_glds); BSR_SKINNY_GLDS=0 runs
    k_filter_skinny2 instead -- both row modes (self-thresholded, thresholded), the same bits, the
    planted clusters included (their second chance and rerun)."""
    ix, host, qh = shard
    qs = np.ascontiguousarray(qh[[0, 1, 3, 5, 6, 11]])
    want = _oracle(oracle_mod, host, qs, 10)
    monkeypatch.setenv("BSR_SKINNY_TOP", top)
    for glds in ("1", "0", "1"):
        monkeypatch.setenv("BSR_SKINNY_GLDS", glds)
        for rep in range(2):
            got = ix.local_top_k(qs, 10)
            assert bool(ix.last_stats().search_path & bsr_mod.BSR_PATH_SKINNY_TOP) == (top == "1")
            _same(got, want, f"top={top} glds={glds} rep {rep}")


def test_top_path_near_duplicate_clusters(bsr_mod, oracle_mod, shard):
    """q0: 150 scattered near-duplicates -- the first pass's k' candidates are all duplicates, so
    it cannot certify; the second chance (every listed key above the wave bound) does.  q1: a run
    of 300 consecutive near-duplicates -- spread over 150 workgroups by the strided pairs, the same.
    q2: 5000 scattered near-duplicates -- some workgroup holds more than 4, so its 4th key is a
    duplicate and nothing certifies: the batch runs again on the thresholded path, whose
    overflowing list sends q2 to the exact scan.  Every result bit-exact."""
    ix, host, qh = shard
    for sel, rerun in [([0], False), ([1], False), ([0, 1, 3], False), ([2], True), ([0, 2, 4], True)]:
        qs = np.ascontiguousarray(qh[sel])
        want = _oracle(oracle_mod, host, qs, 10)
        for rep in range(2):
            got = ix.local_top_k(qs, 10)
            st = ix.last_stats()
            _same(got, want, f"clusters {sel} rep {rep}")
            path = st.search_path
            assert path & bsr_mod.BSR_PATH_SKINNY_TOP, path
            assert bool(path & bsr_mod.BSR_PATH_TOP_RERUN) == rerun, (sel, path)
            if not rerun:
                assert st.n_rescued >= sum(1 for j in sel if j in (0, 1)) and st.n_fallback == 0, \
                    (sel, st.n_rescued, st.n_fallback)
            else:
                assert st.n_fallback == 1, (sel, st.n_fallback)   # q2 only, by the exact scan


def test_top_path_zero_query_takes_exact_scan(bsr_mod, oracle_mod, shard):
    """A query the filter cannot serve (zero vector: the reference's distance 1.0 for every row)
    in a self-thresholded batch: its list is empty and it takes the exact scan; the others are
    certified as usual."""
    ix, host, qh = shard
    qs = np.ascontiguousarray(qh[[3, 4]])
    qs[1] = 0.0
    want = _oracle(oracle_mod, host, qs, 10)
    got = ix.local_top_k(qs, 10)
    st = ix.last_stats()
    _same(got, want, "zero query")
    assert st.n_exact_direct == 1, st.n_exact_direct


@pytest.mark.parametrize("dim,nq,k", [(256, 3, 10), (200, 1, 5)])
def test_top_path_other_widths(bsr_mod, oracle_mod, gpu, dim, nq, k):
    """The self-thresholded path on rows of other widths (4 K slices: k_filter_skinny2<kSkTop, 4>;
    200: a partial last slice and a zero-padded row tail), over 2.2M rows, with a planted
    self-match in the last partial unit: bit-exact against the oracle, twice (graph replay)."""
    import torch
    n = 2_200_003
    rows = torch.empty((n, dim), dtype=torch.float32, device="cuda:0")
    bsr_mod.synth_uniform(rows.data_ptr(), 0, n, dim, 9)
    q = torch.empty((nq, dim), dtype=torch.float32, device="cuda:0")
    bsr_mod.synth_uniform(q.data_ptr(), 0, nq, dim, 10)
    q[0] = rows[n - 1]
    torch.cuda.synchronize()
    ix = bsr_mod.Index(dim, max_k=64, device=0)
    ix.load(rows)
    host, qh = rows.cpu().numpy(), q.cpu().numpy()
    del rows
    torch.cuda.empty_cache()
    want = oracle_mod.parallel_top_k(host, qh, k, size=THREADS, threads=THREADS)
    for rep in range(3):
        got = ix.local_top_k(qh, k)
        st = ix.last_stats()
        assert st.search_path & bsr_mod.BSR_PATH_SKINNY_TOP, st.search_path
        assert st.n_fallback == 0
        _same(got, want, f"dim {dim} nq {nq} k {k} rep {rep}")
    assert got[0][0, 0] == n - 1 and got[1][0, 0] == 0.0
    ix.close()


@pytest.mark.parametrize("top", ["1", "0"])
def test_top_path_bf16_corpus(bsr_mod, oracle_mod, gpu, monkeypatch, top):
    """configs[4]'s corpus type on the single-query paths: a bf16 corpus (widened exactly to f32 at
    load; the reference's values are the widened ones) of 2.2M rows, 768 wide -- the LDS-DMA skinny
    filter in both row modes (self-thresholded and thresholded) -- with a planted self-match:
    bit-exact against the oracle over the widened rows."""
    import torch
    n, dim, nq, k = 2_200_011, 768, 4, 10
    rows = torch.empty((n, dim), dtype=torch.float32, device="cuda:0")
    bsr_mod.synth_uniform(rows.data_ptr(), 0, n, dim, 21)
    rows16 = rows.to(torch.bfloat16)
    del rows
    q = rows16[[7, n // 2, n - 1, 12345]].float()
    q[3] = q[3] * 0.5 + 0.25
    torch.cuda.synchronize()
    ix = bsr_mod.Index(dim, max_k=64, device=0, dtype=bsr_mod.BSR_BF16)
    ix.load(rows16)
    host = rows16.float().cpu().numpy()
    del rows16
    torch.cuda.empty_cache()
    qh = np.ascontiguousarray(q.cpu().numpy())
    want = oracle_mod.parallel_top_k(host, qh, k, size=THREADS, threads=THREADS)
    monkeypatch.setenv("BSR_SKINNY_TOP", top)
    for rep in range(2):
        got = ix.local_top_k(qh, k)
        assert bool(ix.last_stats().search_path & bsr_mod.BSR_PATH_SKINNY_TOP) == (top == "1")
        _same(got, want, f"bf16 top={top} rep {rep}")
    assert list(got[0][:3, 0]) == [7, n // 2, n - 1]
    ix.close()
