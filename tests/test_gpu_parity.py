"""GPU parity: the HIP path (through the C ABI) against the oracle, bit for bit.

Indices, their order and the f32 distance bits must equal the reference restatement's
(north_star: indices/ranks bit-exact, distances within 1e-5 -- we require
exact bits, the stronger bar).  Sizes keep the oracle to seconds."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def _assert_same(got, want, ctx=""):
    gi, gd, gc = got
    wi, wd, wc = want
    assert np.array_equal(gc, wc), (ctx, gc, wc)
    for q in range(len(wc)):
        c = int(wc[q])
        assert np.array_equal(gi[q, :c], wi[q, :c]), (ctx, q, gi[q, :c], wi[q, :c])
        assert np.array_equal(gd[q, :c].view(np.uint32), wd[q, :c].view(np.uint32)), (ctx, q)


def _index(bsr_mod, rows, max_k=256, flags=0, offset=0):
    ix = bsr_mod.Index(rows.shape[1], max_k=max_k, device=0, flags=flags)
    ix.load(rows, offset)
    return ix


# ---- a-1 ---------------------------------------------------------------------------------
def test_cosine_known_answers_on_gpu(bsr_mod, gpu):
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        ka = json.load(f)
    for c in ka["cosine_distance"]:
        got = bsr_mod.cosine_distance(np.array(c["a"], np.float32), np.array(c["b"], np.float32))
        assert np.float32(got).view(np.uint32) == c["expected_bits"], c["name"]


def test_cosine_random_pairs_bitexact(bsr_mod, oracle_mod, gpu):
    rng = np.random.default_rng(0)
    for i in range(60):
        d = int(rng.choice([1, 2, 3, 17, 768, 1024]))
        a = (rng.uniform(-1, 1, d) * 10.0 ** rng.integers(-20, 20)).astype(np.float32)
        b = (rng.uniform(-1, 1, d) * 10.0 ** rng.integers(-20, 20)).astype(np.float32)
        if i % 7 == 0:
            b = a.copy()
        if i % 11 == 0:
            b = a + np.float32(3e-11)
        want = oracle_mod.cosine_distance(a, b)
        got = bsr_mod.cosine_distance(a, b)
        assert np.float32(got).view(np.uint32) == np.float32(want).view(np.uint32), (i, got, want)


# ---- golden fixtures ------------------------------------------------------------------
@pytest.mark.parametrize("exact_only", [False, True])
def test_golden_search(bsr_mod, gpu, exact_only):
    from golden.make_golden import corpus_case
    g = np.load(os.path.join(GOLDEN, "search_golden.npz"))
    for ci in range(int(g["n_cases"])):
        seed, n, dim, nq, k, P = (int(x) for x in g[f"c{ci}_spec"])
        rows = corpus_case(seed, n, dim) if n > 20 else bsr_mod.synth_uniform_np(0, n, dim, seed)
        q = bsr_mod.synth_uniform_np(0, nq, dim, seed + 1000)
        if n > 20:
            q[0] = rows[5]
        if nq > 1:
            q[1] = rows[min(3, n - 1)]
        ix = _index(bsr_mod, rows, flags=1 if exact_only else 0)
        # repeat the queries so the batched MFMA filter path (>= 16 queries) runs too
        reps = 1 if exact_only else 8
        qq = np.concatenate([q] * reps)
        gi, gd, gc = ix.local_top_k(qq, k)
        want = (g[f"c{ci}_idx"], g[f"c{ci}_dist_bits"].view(np.float32), g[f"c{ci}_count"])
        for r in range(reps):
            sl = slice(r * nq, (r + 1) * nq)
            _assert_same((gi[sl], gd[sl], gc[sl]), want, f"case {ci} rep {r}")


# ---- small batches: int8 skinny filter (k > 200: exact scan) vs the oracle -----------------
@pytest.mark.parametrize("n,dim,nq,k", [
    (1, 768, 1, 10), (5, 768, 3, 10), (257, 768, 2, 1), (1000, 768, 5, 64), (3000, 130, 9, 100),
    (4097, 768, 4, 256), (20000, 768, 8, 50), (100000, 768, 16, 10), (70000, 96, 1, 10),
    (3000, 130, 9, 10), (8000, 200, 3, 5), (50000, 1024, 2, 10),
    (1200000, 128, 3, 10),   # (1172 compact sample maxima: one wave per query selects tau)
    (2200000, 64, 2, 10)])   # (2149 maxima: the 16-wave tau selection, k_select_tau_m)
def test_small_batches_vs_oracle(bsr_mod, oracle_mod, gpu, n, dim, nq, k):
    rng = np.random.default_rng(n + dim + k)
    rows = rng.uniform(-1, 1, (n, dim)).astype(np.float32)
    if n > 10:
        rows[n // 2] = rows[1]
        rows[3] = 0
    qs = rng.uniform(-1, 1, (nq, dim)).astype(np.float32)
    qs[0] = rows[min(1, n - 1)]
    ix = _index(bsr_mod, rows, flags=0)
    got = ix.local_top_k(qs, k)
    st = ix.last_stats()
    if k > 200:
        assert st.n_exact_direct == nq
    else:
        assert st.n_exact_direct == 0 and st.n_fallback == 0, (st.n_exact_direct, st.n_fallback)
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, k), f"n={n} k={k}")


@pytest.mark.parametrize("n,dim,nq,k", [
    (20000, 768, 32, 10),   # config 1 stand-in (JabRef ~20k chunks, 32 queries, top-10)
    (20000, 768, 40, 50),   # the reference's own k = 50 (src/main.rs:110)
    (30000, 256, 20, 100),
    (2500, 768, 64, 10),    # n <= candidate cap: no sample pass, tau = -inf
    (50000, 96, 17, 200),
    (100000, 768, 24, 10),  # large shard: compact sample (maxima over 32 sampled rows)
    (5000, 40, 16, 10),     # 64-byte int8 rows: one K slice per tile
    (6000, 1100, 20, 10),   # rows longer than the rescore's LDS query copy (1024 floats)
])
def test_filter_path_vs_oracle(bsr_mod, oracle_mod, gpu, n, dim, nq, k):
    rng = np.random.default_rng(7 * n + k)
    rows = rng.uniform(-1, 1, (n, dim)).astype(np.float32)
    rows[n - 1] = rows[0]            # duplicate pair far apart
    rows[10] = 0                     # zero row
    rows[12] = rows[20] * np.float32(3.0)
    qs = rng.uniform(-1, 1, (nq, dim)).astype(np.float32)
    qs[0] = rows[0]
    qs[1] = rows[20]
    ix = _index(bsr_mod, rows, flags=0)
    got = ix.local_top_k(qs, k)
    st = ix.last_stats()
    assert st.n_exact_direct == 0 and st.n_candidates >= k
    assert st.filter_op == 0
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, k), f"n={n} k={k}")
    # both copies of row 0 lead query 0's list at distance 0, smaller index first
    assert list(got[0][0, :2]) == [0, n - 1] and got[1][0, 0] == 0 and got[1][0, 1] == 0


def test_filter_certifies_uniform_data(bsr_mod, oracle_mod, gpu):
    # Independent U(-1,1) queries over a U(-1,1) corpus (the bench's data): the filter must
    # certify every query (a broken filter would still be exact, through fallbacks).
    rng = np.random.default_rng(11)
    rows = rng.uniform(-1, 1, (60000, 768)).astype(np.float32)
    qs = rng.uniform(-1, 1, (48, 768)).astype(np.float32)
    qs[0] = rows[123]
    ix = _index(bsr_mod, rows, flags=0)
    got = ix.local_top_k(qs, 10)
    st = ix.last_stats()
    assert st.n_fallback == 0 and st.n_exact_direct == 0, (st.n_fallback, st.n_exact_direct)
    assert st.n_emitted >= 48 * 64
    assert 1e-3 < st.row_ebound < 6e-3, st.row_ebound
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 10), "uniform")


def test_large_k_certifies_without_fallback(bsr_mod, oracle_mod, gpu):
    # k = 100 over a large shard (config 5's k): k' ~ 3k candidates must certify every
    # independent query (k' = k + 54 failed them all at 6.25M rows).
    rng = np.random.default_rng(21)
    rows = rng.uniform(-1, 1, (300000, 768)).astype(np.float32)
    qs = rng.uniform(-1, 1, (24, 768)).astype(np.float32)
    qs[0] = rows[4242]
    ix = _index(bsr_mod, rows, max_k=100)
    got = ix.local_top_k(qs, 100)
    st = ix.last_stats()
    assert st.n_fallback == 0 and st.n_candidates == 383, (st.n_fallback, st.n_rescued, st.n_candidates)
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 100), "k=100")


def test_large_k_many_queries_dense_emission(bsr_mod, oracle_mod, gpu):
    # 2048 queries, k = 100: every filter workgroup sees ~48 emitted rows per query, more
    # than a lane's candidate ring holds (the rest append to the global lists directly).
    # All queries must still certify; parity on a subset (the oracle's cost).
    rng = np.random.default_rng(33)
    rows = rng.uniform(-1, 1, (100000, 768)).astype(np.float32)
    qs = rng.uniform(-1, 1, (2048, 768)).astype(np.float32)
    qs[0] = rows[777]
    ix = _index(bsr_mod, rows, max_k=100)
    gi, gd, gc = ix.local_top_k(qs, 100)
    st = ix.last_stats()
    assert st.n_fallback == 0 and st.n_exact_direct == 0, (st.n_fallback, st.n_exact_direct)
    sub = np.r_[0:8, 1020:1024, 2040:2048]
    _assert_same((gi[sub], gd[sub], gc[sub]), oracle_mod.parallel_top_k(rows, qs[sub], 100), "k=100 Q=2048")


def test_duplicate_runs_overflow_lane_rings(bsr_mod, oracle_mod, gpu):
    # Runs of 400 identical rows: a query equal to one of them passes the filter on a whole
    # run (64 rows per lane per tile, more than a lane's candidate ring); ties resolve by
    # index and every result stays exact (through the fallback when uncertifiable).
    rng = np.random.default_rng(5)
    base = rng.uniform(-1, 1, (100, 768)).astype(np.float32)
    rows = np.repeat(base, 400, axis=0)
    qs = base[rng.integers(0, 100, 40)].copy()
    qs[1::2] += rng.uniform(-0.05, 0.05, (20, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, flags=0)
    got = ix.local_top_k(qs, 10)
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 10), "duplicate runs")


def test_filter_path_normal_data_with_clusters(bsr_mod, oracle_mod, gpu):
    # Clustered embeddings (dense neighbourhoods) stress the certification; any query it
    # cannot certify must fall back to the exact scan and still be exact.
    rng = np.random.default_rng(42)
    centers = rng.normal(size=(20, 768)).astype(np.float32)
    rows = (centers[rng.integers(0, 20, 40000)] + 0.05 * rng.normal(size=(40000, 768))).astype(np.float32)
    qs = (centers[rng.integers(0, 20, 24)] + 0.05 * rng.normal(size=(24, 768))).astype(np.float32)
    ix = _index(bsr_mod, rows, flags=0)
    got = ix.local_top_k(qs, 10)
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 10), "clusters")


@pytest.mark.parametrize("k", [10, 50])
def test_filter_outlier_block_scales(bsr_mod, oracle_mod, gpu, k):
    """Rows with one dominant component get large int8 block scales: the emit filter's integer
    pre-test threshold (from the LARGEST block scale of the shard) is then far below most
    blocks' own -- a loose pre-test, but the emitted set must still be exactly the float test's
    and every result exact.  Some queries are outlier rows themselves."""
    rng = np.random.default_rng(8)
    n = 60000
    rows = rng.uniform(-1, 1, (n, 768)).astype(np.float32)
    spikes = rng.choice(n, 300, replace=False)
    rows[spikes, rng.integers(0, 768, 300)] = np.float32(60.0)   # max|a_i|/|a| ~ 0.96
    qs = rng.uniform(-1, 1, (40, 768)).astype(np.float32)
    qs[:5] = rows[spikes[:5]]
    qs[5:10, 7] += np.float32(30.0)                              # queries leaning on one dim
    ix = _index(bsr_mod, rows, max_k=64)
    got = ix.local_top_k(qs, k)
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, k, size=8, threads=8), f"outlier scales k={k}")
    for j in range(5):
        assert got[0][j, 0] == spikes[j] and got[1][j, 0] == 0.0


def test_global_offset_and_get_many(bsr_mod, gpu):
    rng = np.random.default_rng(1)
    rows = rng.uniform(-1, 1, (300, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, offset=1000)
    assert ix.get_count() == 300 and ix.global_offset() == 1000
    assert np.array_equal(ix.get_many(bsr_mod.SliceArgs(10, 5)), rows[10:15])
    assert np.array_equal(ix.get(299), rows[299])
    assert np.array_equal(ix.get_many(), rows)
    gi, gd, gc = ix.local_top_k(rows[[42]], 3)
    assert gi[0, 0] == 1042 and gd[0, 0] == 0


def test_append_many_then_search(bsr_mod, oracle_mod, gpu):
    rng = np.random.default_rng(2)
    rows = rng.uniform(-1, 1, (3000, 768)).astype(np.float32)
    ix = bsr_mod.Index(768, max_k=16, device=0)
    ix.load(rows[:1000])
    ix.append_many(rows[1000:2500])
    ix.append_many(rows[2500:])
    assert ix.get_count() == 3000
    qs = rng.uniform(-1, 1, (20, 768)).astype(np.float32)
    _assert_same(ix.local_top_k(qs, 16), oracle_mod.parallel_top_k(rows, qs, 16), "append")


def test_load_and_append_device_rows_from_side_stream(bsr_mod, oracle_mod, gpu):
    """Device rows written on a torch side stream, not synchronized by the caller: load and
    append must read the rows written (polars.rs:121-156 -- the slab read is the slab written),
    not what the buffer held before."""
    import torch
    rng = np.random.default_rng(12)
    n = 40000
    rows = rng.uniform(-1, 1, (n, 768)).astype(np.float32)
    src = torch.from_numpy(rows).cuda()
    dst = torch.zeros_like(src)
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        delay = torch.randn(4096, 4096, device="cuda")
        for _ in range(40):  # tens of ms of side-stream work ahead of the copies
            delay = torch.tanh(delay @ delay)
        dst[: n // 2].copy_(src[: n // 2])
    ix = bsr_mod.Index(768, max_k=10, device=0)
    ix.load(dst[: n // 2])  # no synchronisation by the caller
    with torch.cuda.stream(side):
        for _ in range(40):
            delay = torch.tanh(delay @ delay)
        dst[n // 2:].copy_(src[n // 2:])
    ix.append_many(dst[n // 2:])
    assert np.array_equal(ix.get_many(), rows)
    qs = rng.uniform(-1, 1, (24, 768)).astype(np.float32)
    qs[0] = rows[n - 5]
    _assert_same(ix.local_top_k(qs, 10), oracle_mod.parallel_top_k(rows, qs, 10), "side stream")
    torch.cuda.synchronize()


def test_errors(bsr_mod, gpu):
    ix = bsr_mod.Index(768, max_k=10, device=0)
    with pytest.raises(bsr_mod.BsrError) as e:
        ix.local_top_k(np.zeros((1, 768), np.float32), 5)
    assert e.value.status == -7  # not loaded
    rows = np.ones((10, 768), np.float32)
    rows[3, 4] = np.nan
    with pytest.raises(bsr_mod.BsrError) as e:
        ix.load(rows)
    assert e.value.status == -2
    ix.load(np.ones((10, 768), np.float32))
    with pytest.raises(bsr_mod.BsrError) as e:
        ix.local_top_k(np.zeros((1, 768), np.float32), 11)
    assert e.value.status == -1
    q = np.zeros((1, 768), np.float32)
    q[0, 0] = np.inf
    with pytest.raises(bsr_mod.BsrError) as e:
        ix.local_top_k(q, 5)
    assert e.value.status == -2
    with pytest.raises(bsr_mod.BsrError) as e:
        ix.local_top_k(np.zeros((1, 700), np.float32), 5)
    assert e.value.status == -6


def test_zero_and_tiny_queries_take_exact_path(bsr_mod, oracle_mod, gpu):
    rng = np.random.default_rng(3)
    rows = rng.uniform(-1, 1, (5000, 768)).astype(np.float32)
    rows[17] = 0
    rows[18] = np.float32(1e-12)  # within 1e-10 of the zero query -> identical -> 0.0
    qs = rng.uniform(-1, 1, (20, 768)).astype(np.float32)
    qs[2] = 0
    qs[3] = np.float32(1e-25)
    ix = _index(bsr_mod, rows)
    got = ix.local_top_k(qs, 10)
    assert ix.last_stats().n_exact_direct >= 2
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 10), "zero query")


def test_overflowing_rows_force_exact(bsr_mod, oracle_mod, gpu):
    rng = np.random.default_rng(4)
    rows = rng.uniform(-1, 1, (3000, 768)).astype(np.float32)
    rows[5] *= np.float32(1e19)   # |a|^2 overflows -> reference distance 1.0 or 2.0
    qs = rng.uniform(-1, 1, (20, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows)
    got = ix.local_top_k(qs, 10)
    assert ix.last_stats().n_exact_direct == 20
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 10), "overflow")


@pytest.mark.parametrize("nq,n_rescue,n_over", [(64, 16, 4), (8, 5, 2), (1, 1, 0)])
def test_published_rescue_and_fallback_rows(bsr_mod, oracle_mod, gpu, nq, n_rescue, n_over):
    """The published result (rescore kernels writing every row into the pinned host mirror, the
    last kernel copying only the status words, round 4) with all three sources of rows in one
    batch, replayed as a graph: rows certified by the first rescore, rows of queries rescued by
    the second chance (200 near-duplicates of the query: the first pass's k' candidates cannot
    be certified), and rows of queries whose emitted list overflows (1500 near-duplicates: the
    exact scan, read back by a D2H copy over the same host buffer).  Tiny batches (<= 16 queries)
    take the one-workgroup-per-query first pass and a one-workgroup second chance."""
    rng = np.random.default_rng(404)
    n, dim, k = 60000, 768, 10
    rows = rng.uniform(-1, 1, (n, dim)).astype(np.float32)
    qs = rng.uniform(-1, 1, (nq, dim)).astype(np.float32)
    # The near-duplicates sit only at rows the sample pass never reads (row % 32 != 0, the
    # every-32nd-row sample, csrc/index.cpp sample_pass): tau0 is then set by the uniform rows for
    # any seed, the duplicates all pass it, and the rescue queries' first pass cannot certify -- the
    # second chance runs by construction.
    unsampled = np.flatnonzero(np.arange(n) % 32 != 0)
    perm = unsampled[rng.permutation(len(unsampled))]
    at = 0
    m_rescue = 200
    for q, m in [(q, m_rescue) for q in range(n_rescue)] + [(q, 1500) for q in range(n_rescue, n_rescue + n_over)]:
        pos = perm[at:at + m]
        at += m
        rows[pos] = qs[q] + rng.normal(0, 1e-3, (m, dim)).astype(np.float32)
    ix = _index(bsr_mod, rows, max_k=64)
    want = oracle_mod.parallel_top_k(rows, qs, k, size=4, threads=4)
    rescued = fallback = replays = 0
    for rep in range(3):
        got = ix.local_top_k(qs, k)
        st = ix.last_stats()
        rescued += st.n_rescued
        fallback += st.n_fallback
        replays += st.graph_replay
        _assert_same(got, want, f"rep {rep}")
    assert rescued > 0 and (fallback > 0) == (n_over > 0) and replays > 0, (rescued, fallback, replays)


def test_bf16_filter_operand_retired(bsr_mod, gpu):
    # the bf16 filter OPERAND (rounds 1-3) is retired; a bf16 CORPUS is served on the int8 filter
    with pytest.raises(bsr_mod.BsrError) as e:
        bsr_mod.Index(768, max_k=10, device=0, flags=bsr_mod.BSR_FLAG_FILTER_BF16)
    assert e.value.status == -1 and "retired" in str(e.value)


def test_bf16_corpus_widened(bsr_mod, oracle_mod, gpu):
    rng = np.random.default_rng(5)
    f = rng.uniform(-1, 1, (4000, 768)).astype(np.float32)
    bits = (f.view(np.uint32) + 0x7FFF + ((f.view(np.uint32) >> 16) & 1)) >> 16
    b16 = bits.astype(np.uint16)
    widened = (b16.astype(np.uint32) << 16).view(np.float32)
    ix = bsr_mod.Index(768, max_k=100, device=0, dtype=bsr_mod.BSR_BF16)
    ix.load(b16)
    qs = widened[:20].copy()
    _assert_same(ix.local_top_k(qs, 100), oracle_mod.parallel_top_k(widened, qs, 100), "bf16")


# ---- sharding: results independent of the number of shards ----------------------------
@pytest.mark.parametrize("P", [2, 3, 8])
def test_shards_on_one_gpu_merge_to_single(bsr_mod, oracle_mod, gpu, P):
    rng = np.random.default_rng(P)
    N = 24001
    rows = rng.uniform(-1, 1, (N, 768)).astype(np.float32)
    rows[N - 3] = rows[2]
    qs = rng.uniform(-1, 1, (32, 768)).astype(np.float32)
    qs[0] = rows[2]
    k = 10
    li = np.zeros((P, 32, k), np.uint64)
    ld = np.zeros((P, 32, k), np.float32)
    lc = np.zeros((P, 32), np.uint32)
    for r in range(P):
        iv = bsr_mod.interval_by_rank(r, P, N)
        s, e = iv.start_index, max(iv.start_index, iv.end_index)
        if s >= N:
            continue
        ix = _index(bsr_mod, rows[s:e], max_k=k, offset=s)
        li[r], ld[r], lc[r] = ix.local_top_k(qs, k)
    got = bsr_mod.merge_top_k_lists(li, ld, lc, k)
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, k, size=P), f"P={P}")


def test_parallel_search_single_rank_comm(bsr_mod, oracle_mod, gpu):
    rng = np.random.default_rng(8)
    rows = rng.uniform(-1, 1, (10000, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, max_k=50)
    comm = bsr_mod.Comm(bsr_mod.Comm.unique_id(), 0, 1, 0)
    res = bsr_mod.parallel_top_k_similarity_search(comm, 0, 1, ix, 50, rows[0])
    wi, wd, wc = oracle_mod.parallel_top_k(rows, rows[[0]], 50)
    assert [i for i, _ in res] == [int(x) for x in wi[0]]
    assert np.array_equal(np.array([d for _, d in res], np.float32).view(np.uint32), wd[0].view(np.uint32))
    assert bsr_mod.calculate_accuracy_metrics(res, 0, 50) == (1.0, 1.0, 1.0)
    comm.close()


def test_synth_uniform_device_matches_host_replica(bsr_mod, gpu):
    import torch
    t = torch.empty((37, 768), dtype=torch.float32, device="cuda:0")
    bsr_mod.synth_uniform(t.data_ptr(), 1000, 37, 768, 42)
    torch.cuda.synchronize()
    assert np.array_equal(t.cpu().numpy(), bsr_mod.synth_uniform_np(1000, 37, 768, 42))


def test_device_pointer_inputs(bsr_mod, oracle_mod, gpu):
    import torch
    rng = np.random.default_rng(9)
    rows = rng.uniform(-1, 1, (6000, 768)).astype(np.float32)
    qs = rng.uniform(-1, 1, (33, 768)).astype(np.float32)
    ix = bsr_mod.Index(768, max_k=10, device=0)
    ix.load(torch.from_numpy(rows).cuda())
    torch.cuda.synchronize()
    dq = torch.from_numpy(qs).cuda()
    oi = torch.empty((33, 10), dtype=torch.int64, device="cuda:0")
    od = torch.empty((33, 10), dtype=torch.float32, device="cuda:0")
    oc = torch.empty(33, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    ix.local_top_k_device(dq, 33, 10, oi, od, oc)
    got = (oi.cpu().numpy().astype(np.uint64), od.cpu().numpy(), oc.cpu().numpy().astype(np.uint32))
    _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 10), "device ptrs")


# ---- captured search graphs (small batches replay one hipGraph) ---------------------------
def test_small_batch_graph_replay_reads_fresh_queries(bsr_mod, oracle_mod, gpu):
    """Batches of <= 16 queries replay a captured graph from their third search of a shape on;
    every replay must read the queries of ITS call (host staging and device pointers), and
    shape changes must not replay a stale graph."""
    import torch
    rng = np.random.default_rng(21)
    rows = rng.uniform(-1, 1, (40000, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, max_k=64)
    replays = 0
    for it in range(8):
        for nq, k in ((1, 10), (1, 10), (3, 10), (1, 25)):
            qs = rng.uniform(-1, 1, (nq, 768)).astype(np.float32)
            qs[0] = rows[(it * 7919) % len(rows)]
            got = ix.local_top_k(qs, k)
            replays += ix.last_stats().graph_replay
            _assert_same(got, oracle_mod.parallel_top_k(rows, qs, k), f"host it={it} nq={nq} k={k}")
    assert replays > 0
    # device-pointer queries: same buffer, contents rewritten between searches
    dq = torch.empty((2, 768), dtype=torch.float32, device="cuda:0")
    oi = torch.empty((2, 10), dtype=torch.int64, device="cuda:0")
    od = torch.empty((2, 10), dtype=torch.float32, device="cuda:0")
    oc = torch.empty(2, dtype=torch.int32, device="cuda:0")
    dev_replays = 0
    for it in range(6):
        qs = rng.uniform(-1, 1, (2, 768)).astype(np.float32)
        dq.copy_(torch.from_numpy(qs))
        torch.cuda.synchronize()
        ix.local_top_k_device(dq, 2, 10, oi, od, oc)
        dev_replays += ix.last_stats().graph_replay
        got = (oi.cpu().numpy().astype(np.uint64), od.cpu().numpy(), oc.cpu().numpy().astype(np.uint32))
        _assert_same(got, oracle_mod.parallel_top_k(rows, qs, 10), f"device it={it}")
    assert dev_replays > 0


@pytest.mark.parametrize("staging", ["device", "host"])
def test_large_batch_graph_replay_reads_fresh_queries(bsr_mod, oracle_mod, gpu, staging):
    """Filtered batches of Q >= 256 replay a captured graph (prep -> sample pass -> tau0 ->
    emit filter -> rescore -> finalize -> D2H) from their second search of a shape on.  Same
    buffer (device pointer, or the library's host staging copy), same shape, new contents every
    round -- one round turns some queries into corpus rows, another into a scaled row -- and
    every round must equal the oracle on ALL queries (a stale tau0, candidate count or query
    operand baked into the graph would show here).  Each call is an independent search
    (src/mpi_helpers/metrics.rs:174-206)."""
    import torch
    rng = np.random.default_rng(77)
    n, nq, k = 50000, 256, 10
    rows = rng.uniform(-1, 1, (n, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, max_k=16)
    dq = torch.empty((nq, 768), dtype=torch.float32, device="cuda:0")
    oi = torch.empty((nq, k), dtype=torch.int64, device="cuda:0")
    od = torch.empty((nq, k), dtype=torch.float32, device="cuda:0")
    oc = torch.empty(nq, dtype=torch.int32, device="cuda:0")
    hq = np.empty((nq, 768), np.float32)  # one host buffer, rewritten in place
    replays = []
    for it in range(7):
        qs = rng.uniform(-1, 1, (nq, 768)).astype(np.float32)
        if it == 3:   # queries that are corpus rows (self-match at distance 0)
            for j in range(0, nq, 17):
                qs[j] = rows[(j * 7919 + it) % n]
        if it == 5:   # a scaled corpus row: distance 0 without being identical
            qs[1] = rows[123] * np.float32(4.0)
        if staging == "device":
            dq.copy_(torch.from_numpy(qs))
            torch.cuda.synchronize()
            ix.local_top_k_device(dq, nq, k, oi, od, oc)
            got = (oi.cpu().numpy().astype(np.uint64), od.cpu().numpy(), oc.cpu().numpy().astype(np.uint32))
        else:
            hq[:] = qs
            got = ix.local_top_k(hq, k)
        st = ix.last_stats()
        replays.append(st.graph_replay)
        assert st.n_exact_direct == 0
        _assert_same(got, oracle_mod.parallel_top_k(rows, qs, k, size=8, threads=8), f"{staging} round {it}")
        if it == 3:
            for j in range(0, nq, 17):
                assert got[0][j, 0] == (j * 7919 + it) % n and got[1][j, 0] == 0.0
    assert replays[0] == 0 and all(replays[1:]), replays


def test_profile_levels(bsr_mod, oracle_mod, gpu):
    """bsr_index_set_profile: level 1 times only the emit filter / scan kernels (events recorded
    on the stream around their direct launch), 2 every stage, 0 none (graph replay) -- results
    identical at every level."""
    rng = np.random.default_rng(31)
    rows = rng.uniform(-1, 1, (30000, 768)).astype(np.float32)
    qs = rng.uniform(-1, 1, (40, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, max_k=16, flags=bsr_mod.BSR_FLAG_PROFILE)
    want = oracle_mod.parallel_top_k(rows, qs, 10)
    seen = {}
    for level in (2, 1, 0):
        ix.set_profile(level)
        ix.profile(reset=True)
        _assert_same(ix.local_top_k(qs, 10), want, f"level {level}")
        seen[level] = ix.profile(reset=True)
    # k = 10: the candidate selection runs inside the rescore kernel (no select launch)
    assert seen[2].gemm_emit_launches == 1 and seen[2].select_launches == 0 and seen[2].searches == 1
    assert seen[2].rescore_launches == 1
    assert seen[1].gemm_emit_launches == 1 and seen[1].select_launches == 0 and seen[1].searches == 0
    assert seen[1].gemm_emit_ms > 0.0 and seen[1].gemm_sample_launches == 0
    assert seen[2].gemm_sample_launches == 1
    assert seen[0].gemm_emit_launches == 0 and seen[0].searches == 0
    with pytest.raises(bsr_mod.BsrError):
        ix.set_profile(3)


def test_driver_search_stage_reference_report(bsr_mod, oracle_mod, gpu):
    """src/main.rs:109-163: query = row 0, k = 50, the result list and the accuracy metrics
    printed in the reference's format; the self-query ranks first (MRR = recall = overlap = 1)."""
    import io
    rng = np.random.default_rng(50)
    rows = rng.uniform(-1, 1, (12000, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, max_k=64)
    buf = io.StringIO()
    res, metrics, secs = bsr_mod.run_search_stage(None, 0, 1, ix, top_k=50, out=buf)
    wi, wd, wc = oracle_mod.parallel_top_k(rows, rows[:1], 50)
    assert [i for i, _ in res] == list(wi[0, :wc[0]])
    assert np.array_equal(np.array([d for _, d in res], np.float32).view(np.uint32), wd[0, :wc[0]].view(np.uint32))
    assert metrics == (1.0, 1.0, 1.0) and secs > 0
    lines = buf.getvalue().splitlines()
    assert lines[0] == "Global top-50 results:"
    assert lines[1] == "  1. Index: 0, Distance: 0"
    assert lines[51:55] == ["Accuracy Metrics:", "  Mean Reciprocal Rank (MRR): 1.0000", "  Recall@50: 1.0000",
                            "  Top-k Overlap: 1.0000"]
    # then the report's similarity_search entry (src/mpi_helpers/benchmark.rs:296-413), one rank
    assert lines[55:58] == ["==== PARALLEL PERFORMANCE REPORT ====", "", "Operation: similarity_search"]
    assert lines[58].startswith("  Min time: ") and lines[58].endswith(" sec (Rank 0)")
    assert lines[59].startswith("  Max time: ") and lines[60].startswith("  Avg time: ")


def test_driver_search_stage_broadcast_single_rank_comm(bsr_mod, oracle_mod, gpu):
    """The driver stage with a communicator (size 1): the root's row query_idx is broadcast
    through the comm (src/main.rs:117-125) and the search runs the exchange + merge path."""
    import io
    rng = np.random.default_rng(51)
    rows = rng.uniform(-1, 1, (9000, 768)).astype(np.float32)
    ix = _index(bsr_mod, rows, max_k=64)
    comm = bsr_mod.Comm(bsr_mod.Comm.unique_id(), 0, 1, 0)
    buf = io.StringIO()
    res, metrics, secs = bsr_mod.run_search_stage(comm, 0, 1, ix, top_k=50, query_idx=7, out=buf)
    wi, wd, wc = oracle_mod.parallel_top_k(rows, rows[7:8], 50)
    assert [i for i, _ in res] == list(wi[0, :wc[0]]) and res[0] == (7, 0.0)
    assert np.array_equal(np.array([d for _, d in res], np.float32).view(np.uint32), wd[0, :wc[0]].view(np.uint32))
    assert metrics == (1.0, 1.0, 1.0)
    v = np.zeros(768, np.float32)
    v[:] = 3.0
    comm.broadcast(v, 0)
    assert (v == 3.0).all()
    assert comm.allgather_bytes(b"abc") == [b"abc"]
    comm.close()
