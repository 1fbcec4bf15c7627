"""The C-ABI library on CPU: it loads, exports every symbol include/bsr.h declares, and its
host-only entry points (interval_by_rank, compute_global_top_k merge) match the oracle.
No compute kernels run here (no GPU in this container)."""
import ctypes
import json
import os
import re

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def header_functions(header="bsr.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = re.findall(r"^\s*(?:const\s+)?[a-z_0-9]+\s*\*?\s*(bsr_[a-z_0-9]+)\s*\(", src, flags=re.M)
    return sorted(set(names))


def test_header_parsed():
    names = header_functions()
    assert "bsr_local_top_k" in names and "bsr_parallel_top_k_similarity_search" in names
    assert len(names) >= 20


def test_library_exports_every_declared_symbol(bsr_mod):
    lib = ctypes.CDLL(bsr_mod.LIB_PATH)
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_vstore_library_exports_every_declared_symbol(bsr_mod):
    lib = bsr_mod.vstore_lib()
    names = header_functions("bsr_vstore.h")
    assert "bsr_index_load_vstore" in names and len(names) >= 14
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_library_is_native_gfx950(bsr_mod):
    # the .so carries a gfx950 code object (kernels are compiled for MI355X, not a fallback)
    blob = open(bsr_mod.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"k_filter" in blob and b"k_scan_exact" in blob


def test_interval_matches_known_and_oracle(bsr_mod, oracle_mod):
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        ka = json.load(f)
    for c in ka["interval_by_rank"]:
        iv = bsr_mod.interval_by_rank(c["rank"], c["size"], c["count"])
        assert (iv.start_index, iv.end_index) == (c["start_index"], c["end_index"])
    rng = np.random.default_rng(3)
    for _ in range(500):
        size = int(rng.integers(1, 40))
        count = int(rng.integers(0, 200))
        rank = int(rng.integers(0, size))
        iv = bsr_mod.interval_by_rank(rank, size, count)
        assert (iv.start_index, iv.end_index) == oracle_mod.interval_by_rank(rank, size, count)


def test_interval_blocks_cover_corpus(bsr_mod):
    for count in [0, 1, 5, 10, 17, 1000, 1_000_003]:
        for size in [1, 2, 3, 4, 7, 8]:
            covered = 0
            for r in range(size):
                iv = bsr_mod.interval_by_rank(r, size, count)
                s, e = iv.start_index, max(iv.start_index, iv.end_index)
                if s < count:
                    assert s == covered
                    covered = min(e, count)
            assert covered == count


def test_interval_rejects_bad_rank(bsr_mod):
    with pytest.raises(bsr_mod.BsrError):
        bsr_mod.interval_by_rank(4, 4, 10)


def test_global_top_k_known(bsr_mod):
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        ka = json.load(f)
    for c in ka["compute_global_top_k"]:
        got = bsr_mod.compute_global_top_k(c["indices"], c["distances"], c["top_k"])
        assert [i for i, _ in got] == c["expected_indices"], c["name"]
        assert np.array_equal(np.array([d for _, d in got], np.float32),
                              np.array(c["expected_distances"], np.float32)), c["name"]


def test_global_top_k_random_vs_oracle(bsr_mod, oracle_mod):
    rng = np.random.default_rng(5)
    for _ in range(50):
        n = int(rng.integers(0, 80))
        idx = rng.integers(0, 40, n).astype(np.uint64)  # duplicates on purpose
        dist = rng.choice(np.array([0.0, 0.25, 0.5, 1.0, 1.5], np.float32), n)
        k = int(rng.integers(1, 30))
        want_i, want_d = oracle_mod.global_top_k(idx, dist, k)
        got = bsr_mod.compute_global_top_k(idx, dist, k)
        assert [i for i, _ in got] == [int(x) for x in want_i]
        assert np.array_equal(np.array([d for _, d in got], np.float32), want_d)


def test_merge_lists_many_queries(bsr_mod, oracle_mod):
    rng = np.random.default_rng(9)
    rows = rng.uniform(-1, 1, (900, 32)).astype(np.float32)
    qs = rng.uniform(-1, 1, (6, 32)).astype(np.float32)
    P, k = 4, 12
    li = np.zeros((P, 6, k), np.uint64)
    ld = np.zeros((P, 6, k), np.float32)
    lc = np.zeros((P, 6), np.uint32)
    for r in range(P):
        for q in range(6):
            i, d = oracle_mod.local_top_k(rows, r, P, k, qs[q])
            li[r, q, :len(i)] = i
            ld[r, q, :len(d)] = d
            lc[r, q] = len(i)
    oi, od, oc = bsr_mod.merge_top_k_lists(li, ld, lc, k)
    wi, wd, wc = oracle_mod.parallel_top_k(rows, qs, k, size=1)
    assert np.array_equal(oi, wi) and np.array_equal(od.view(np.uint32), wd.view(np.uint32))


def test_no_cpu_fallback_without_gpu(bsr_mod):
    if bsr_mod.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(bsr_mod.BsrError) as e:
        bsr_mod.Index(768)
    assert e.value.status == -8
    with pytest.raises(bsr_mod.BsrError):
        bsr_mod.cosine_distance([1.0, 2.0], [1.0, 2.0])


def test_synth_generator_replica_is_deterministic(bsr_mod):
    a = bsr_mod.synth_uniform_np(10, 4, 768, 42)
    b = bsr_mod.synth_uniform_np(0, 14, 768, 42)[10:]
    assert np.array_equal(a, b)
    assert a.min() >= -1 and a.max() < 1 and abs(float(a.mean())) < 0.05


def _lists_from(oracle_mod, rows, qs, P, k, offsets=None):
    """Per-rank local lists [P, Q, k] (+ counts) of the oracle over interval_by_rank blocks;
    `offsets` (optional) shifts each rank's indices (caller-chosen global offsets)."""
    Q = len(qs)
    li = np.zeros((P, Q, k), np.uint64)
    ld = np.zeros((P, Q, k), np.float32)
    lc = np.zeros((P, Q), np.uint32)
    for r in range(P):
        for q in range(Q):
            i, d = oracle_mod.local_top_k(rows, r, P, k, qs[q])
            if offsets is not None:
                i = i - np.uint64(oracle_mod.interval_by_rank(r, P, len(rows))[0]) + np.uint64(offsets[r])
            li[r, q, :len(i)] = i
            ld[r, q, :len(d)] = d
            lc[r, q] = len(i)
    return li, ld, lc


def _oracle_merge(oracle_mod, li, ld, lc, k):
    """compute_global_top_k of the oracle over the rank-order concatenation, per query."""
    P, Q, _ = li.shape
    out = []
    for q in range(Q):
        gi = np.concatenate([li[r, q, :lc[r, q]] for r in range(P)])
        gd = np.concatenate([ld[r, q, :lc[r, q]] for r in range(P)])
        out.append(oracle_mod.global_top_k(gi, gd, k))
    return out


@pytest.mark.parametrize("P", [2, 3, 4, 5, 6, 7, 8])
def test_merge_p_way_vs_oracle(bsr_mod, oracle_mod, P):
    """The root merge of the parallel path (merge.cpp) vs the reference's rank-order
    concatenation + stable sort + dedupe, at P = 2..8: cross-rank distance ties (duplicate
    rows in different blocks, an all-equal-distance corpus slice), empty blocks (N < P)."""
    rng = np.random.default_rng(100 + P)
    for n in (P - 1, P + 1, 257):
        if n < 1:
            continue
        rows = rng.uniform(-1, 1, (n, 24)).astype(np.float32)
        if n > 200:
            rows[200] = rows[3]      # tie across ranks
            rows[150:170] = rows[10]  # a run of equal distances spanning block boundaries
        qs = rng.uniform(-1, 1, (5, 24)).astype(np.float32)
        qs[0] = rows[min(3, n - 1)]
        for k in (1, 4, 16):
            li, ld, lc = _lists_from(oracle_mod, rows, qs, P, k)
            oi, od, oc = bsr_mod.merge_top_k_lists(li, ld, lc, k)
            wi, wd, wc = oracle_mod.parallel_top_k(rows, qs, k, size=P)
            assert np.array_equal(oc, wc), (n, k)
            for q in range(len(qs)):
                c = int(wc[q])
                assert np.array_equal(oi[q, :c], wi[q, :c]), (n, k, q)
                assert np.array_equal(od[q, :c].view(np.uint32), wd[q, :c].view(np.uint32))
                assert (oi[q, c:] == np.uint64(2**64 - 1)).all() and np.isinf(od[q, c:]).all()


def test_merge_overlapping_offsets_and_unsorted_vs_oracle(bsr_mod, oracle_mod):
    """Overlapping blocks (every rank's offset 0: the same index from several ranks, kept
    once, first occurrence) and lists not ordered by distance (the literal stable sort)."""
    rng = np.random.default_rng(8)
    rows = rng.uniform(-1, 1, (90, 16)).astype(np.float32)
    qs = rng.uniform(-1, 1, (4, 16)).astype(np.float32)
    for P in (2, 5, 8):
        li, ld, lc = _lists_from(oracle_mod, rows, qs, P, 12, offsets=[0] * P)
        for shuffle in (False, True):
            if shuffle:
                for r in range(P):
                    for q in range(4):
                        perm = rng.permutation(int(lc[r, q]))
                        li[r, q, :lc[r, q]] = li[r, q, perm]
                        ld[r, q, :lc[r, q]] = ld[r, q, perm]
            oi, od, oc = bsr_mod.merge_top_k_lists(li, ld, lc, 12)
            for q, (wi, wd) in enumerate(_oracle_merge(oracle_mod, li, ld, lc, 12)):
                assert int(oc[q]) == len(wi)
                assert np.array_equal(oi[q, :len(wi)], wi) and np.array_equal(od[q, :len(wd)].view(np.uint32),
                                                                              wd.view(np.uint32))
                assert len(set(oi[q, :oc[q]].tolist())) == int(oc[q])  # deduped


def test_merge_nan_is_an_error(bsr_mod):
    li = np.zeros((2, 1, 2), np.uint64)
    ld = np.array([[[0.1, np.nan]], [[0.2, 0.3]]], np.float32)
    lc = np.full((2, 1), 2, np.uint32)
    with pytest.raises(bsr_mod.BsrError) as e:
        bsr_mod.merge_top_k_lists(li, ld, lc, 2)
    assert e.value.status == -2


def test_merge_large_batch_threads_vs_single(bsr_mod):
    """The host merge splits big batches over threads: same result as query by query."""
    rng = np.random.default_rng(4)
    P, Q, k = 8, 3000, 100
    ld = np.sort(rng.choice(np.linspace(0, 1, 50, dtype=np.float32), (P, Q, k)), axis=2).astype(np.float32)
    li = (np.arange(P, dtype=np.uint64)[:, None, None] * 1000 + rng.integers(0, 1000, (P, Q, k)).astype(np.uint64))
    lc = rng.integers(0, k + 1, (P, Q)).astype(np.uint32)
    oi, od, oc = bsr_mod.merge_top_k_lists(li, ld, lc, k)
    for q in (0, 1, 1499, 2998, 2999):
        ri, rd, rc = bsr_mod.merge_top_k_lists(li[:, q:q + 1], ld[:, q:q + 1], lc[:, q:q + 1], k)
        assert oc[q] == rc[0] and np.array_equal(oi[q], ri[0]) and np.array_equal(od[q].view(np.uint32),
                                                                                 rd[0].view(np.uint32))
