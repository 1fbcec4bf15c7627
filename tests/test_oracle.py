"""The oracle (CPU restatement, test infrastructure) against the hand-derived known answers
and the independent numpy restatement.  No GPU."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope="module")
def known():
    with open(os.path.join(GOLDEN, "known_answers.json")) as f:
        return json.load(f)


def test_cosine_known_answers(oracle_mod, known):
    for case in known["cosine_distance"]:
        got = oracle_mod.cosine_distance(np.array(case["a"], np.float32), np.array(case["b"], np.float32))
        assert np.float32(got).view(np.uint32) == case["expected_bits"], case["name"]


def test_interval_known_answers(oracle_mod, known):
    for c in known["interval_by_rank"]:
        assert oracle_mod.interval_by_rank(c["rank"], c["size"], c["count"]) == (c["start_index"], c["end_index"])


def test_global_top_k_known_answers(oracle_mod, known):
    for c in known["compute_global_top_k"]:
        gi, gd = oracle_mod.global_top_k(np.array(c["indices"], np.uint64), np.array(c["distances"], np.float32),
                                         c["top_k"])
        assert [int(x) for x in gi] == c["expected_indices"], c["name"]
        assert np.array_equal(gd, np.array(c["expected_distances"], np.float32)), c["name"]


@pytest.mark.parametrize("seed", [0, 1, 2])
def test_c_matches_numpy_bitwise(oracle_mod, seed):
    rng = np.random.default_rng(seed)
    rows = rng.uniform(-1, 1, (400, 768)).astype(np.float32)
    rows[::37] *= np.float32(1e-3)
    q = rng.normal(size=768).astype(np.float32)
    a = np.array([oracle_mod.cosine_distance(r, q) for r in rows], np.float32)
    b = oracle_mod.np_cosine_distances(rows, q)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_pairwise_sum_would_not_match(oracle_mod):
    # Guard the premise of the restatement: a reordered (pairwise) sum differs in the last bits.
    rng = np.random.default_rng(7)
    rows = rng.uniform(-1, 1, (200, 768)).astype(np.float32)
    q = rng.uniform(-1, 1, 768).astype(np.float32)
    seq = oracle_mod.np_cosine_distances(rows, q)
    pair = (1 - np.clip(np.sum(rows * q, axis=1, dtype=np.float32) /
                        (np.sqrt(np.sum(rows * rows, axis=1, dtype=np.float32)) *
                         np.sqrt(np.sum(q * q, dtype=np.float32))), -1, 1)).astype(np.float32)
    assert not np.array_equal(seq.view(np.uint32), pair.view(np.uint32))


@pytest.mark.parametrize("P", [1, 2, 3, 4, 7, 8, 13])
def test_result_independent_of_rank_count(oracle_mod, P):
    rng = np.random.default_rng(11)
    rows = rng.uniform(-1, 1, (1500, 64)).astype(np.float32)
    rows[100] = rows[50]  # tie
    qs = np.stack([rows[50], rng.uniform(-1, 1, 64).astype(np.float32)])
    i1, d1, c1 = oracle_mod.parallel_top_k(rows, qs, 25, size=1)
    iP, dP, cP = oracle_mod.parallel_top_k(rows, qs, 25, size=P, threads=min(P, 4))
    assert np.array_equal(i1, iP) and np.array_equal(d1.view(np.uint32), dP.view(np.uint32))
    assert np.array_equal(c1, cP)
    assert int(i1[0, 0]) == 50 and int(i1[0, 1]) == 100 and d1[0, 0] == 0 and d1[0, 1] == 0


def test_golden_search_reproduces(oracle_mod):
    import bsr  # synth_uniform_np is pure numpy
    from golden.make_golden import corpus_case  # noqa
    g = np.load(os.path.join(GOLDEN, "search_golden.npz"))
    for ci in range(int(g["n_cases"])):
        seed, n, dim, nq, k, P = (int(x) for x in g[f"c{ci}_spec"])
        rows = corpus_case(seed, n, dim) if n > 20 else bsr.synth_uniform_np(0, n, dim, seed)
        q = bsr.synth_uniform_np(0, nq, dim, seed + 1000)
        if n > 20:
            q[0] = rows[5]
        if nq > 1:
            q[1] = rows[min(3, n - 1)]
        idx, dist, cnt = oracle_mod.parallel_top_k(rows, q, k, size=P)
        assert np.array_equal(cnt, g[f"c{ci}_count"])
        assert np.array_equal(idx, g[f"c{ci}_idx"])
        assert np.array_equal(dist.view(np.uint32), g[f"c{ci}_dist_bits"])


def test_print_top_k_results_reference_format(bsr_mod):
    """src/mpi_helpers/metrics.rs:209-214 with Rust's f32 Display (shortest round trip, positional)."""
    import io
    buf = io.StringIO()
    bsr_mod.print_top_k_results([(0, np.float32(0.0)), (17, np.float32(0.83125)), (3, np.float32(1e-8)),
                                 (9, np.float32(1.0))], out=buf)
    assert buf.getvalue().splitlines() == ["Global top-4 results:", "  1. Index: 0, Distance: 0",
                                           "  2. Index: 17, Distance: 0.83125", "  3. Index: 3, Distance: 0.00000001",
                                           "  4. Index: 9, Distance: 1"]
    assert bsr_mod.calculate_accuracy_metrics([(4, 0.0), (0, 0.1)], 0, 50) == (0.5, 1.0, 1.0)
    assert bsr_mod.calculate_accuracy_metrics([(4, 0.0)], 0, 50) == (0.0, 0.0, 0.0)
