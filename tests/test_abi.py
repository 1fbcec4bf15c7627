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
