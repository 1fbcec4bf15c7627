"""Generate the committed golden fixtures of tests/golden/.

* known_answers.json -- hand-derived from the reference source (no execution of it is
  possible here): each cosine_distance case states which line of src/metrics.rs:143-165
  decides it; interval_by_rank cases follow src/mpi_helpers/load_balance.rs:24-42;
  compute_global_top_k cases follow src/mpi_helpers/metrics.rs:141-171.  Numeric values of
  the non-trivial cases are the f32 evaluation of the formula.
* search_golden.npz -- seeded search cases: inputs are regenerated from (seed, shape) with
  bsr.synth_uniform_np (splitmix64; deterministic), plus deterministic edits for edge rows;
  expected outputs (indices, distance bits) come from the C oracle, cross-checked here
  against the independent numpy restatement.

Run: python tests/golden/make_golden.py   (re-running must reproduce the committed files)
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
import oracle  # noqa: E402
from bsr import synth_uniform_np  # noqa: E402  (pure numpy; no GPU)

F = np.float32


def f32(x):
    return float(np.float32(x))


def known_answers():
    s2 = np.sqrt(F(2.0))
    cos_cases = [
        # name, a (row), b (query), expected, deciding line
        ("identical", [1, 2, 3], [1, 2, 3], 0.0, "metrics.rs:149-151"),
        ("orthogonal", [1, 0], [0, 1], 1.0, "metrics.rs:161-164 (s=0)"),
        ("opposite", [1, 0], [-1, 0], 2.0, "metrics.rs:161-164 (s=-1)"),
        ("parallel_scaled", [3, 4], [6, 8], 0.0, "metrics.rs:161-164 (s=50/50=1)"),
        ("zero_row", [0, 0, 0], [1, 2, 3], 1.0, "metrics.rs:157-159"),
        ("zero_query", [1, 2, 3], [0, 0, 0], 1.0, "metrics.rs:157-159"),
        ("len_mismatch", [1, 2], [1, 2, 3], 1.0, "metrics.rs:144-146"),
        ("empty", [], [], 1.0, "metrics.rs:144-146"),
        ("tiny_opposite_identical", [1e-11, 0], [-1e-11, 0], 0.0,
         "metrics.rs:13 |a-b|=2e-11 <= 1e-10 -> identical"),
        ("threshold_equal", [1, 0], [1, 1e-10], 0.0, "metrics.rs:13 |a-b| == 1e-10f is not > tol"),
        ("diag", [1, 1], [1, 0], f32(F(1.0) - F(F(1.0) / F(s2 * F(1.0)))), "metrics.rs:161-164"),
        ("overflow_nan_clamps_to_minus_one", [1e20, 0], [1e20, 1e19], 2.0,
         "metrics.rs:153-164: dot=inf, |a|*|b|=inf, s=NaN, NaN.max(-1)=-1 -> 2"),
        ("overflow_finite_dot", [1e20, 0], [1, 1], 1.0,
         "metrics.rs:154-164: |a|=inf, s=dot/inf=0 -> 1"),
    ]
    cos = []
    for name, a, b, want, line in cos_cases:
        got_c = oracle.cosine_distance(np.array(a, F), np.array(b, F))
        assert np.float32(got_c).view(np.uint32) == np.float32(want).view(np.uint32), (name, got_c, want)
        cos.append({"name": name, "a": [float(x) for x in np.array(a, F)],
                    "b": [float(x) for x in np.array(b, F)], "expected": float(np.float32(want)),
                    "expected_bits": int(np.float32(want).view(np.uint32)), "reference": line})
    iv_cases = [  # (rank, size, count) -> (start, end); per = size>count ? 1 : ceil(count/size)
        (0, 4, 10, 0, 3), (1, 4, 10, 3, 6), (3, 4, 10, 9, 10), (3, 4, 5, 6, 5), (2, 4, 5, 4, 5),
        (6, 7, 10, 12, 10), (5, 7, 10, 10, 10), (0, 1, 0, 0, 0), (0, 1, 7, 0, 7), (2, 3, 2, 2, 2),
        (1, 3, 2, 1, 2), (7, 8, 10_000_000, 8_750_000, 10_000_000),
        (0, 8, 10_000_000, 0, 1_250_000), (3, 8, 1_000_003, 375_003, 500_004),
    ]
    iv = []
    for r, s, c, st, en in iv_cases:
        assert oracle.interval_by_rank(r, s, c) == (st, en), (r, s, c, oracle.interval_by_rank(r, s, c))
        iv.append({"rank": r, "size": s, "count": c, "start_index": st, "end_index": en})
    g_cases = [
        ("stable_ties_keep_input_order", [7, 2, 9, 4], [0.5, 0.25, 0.25, 0.75], 3, [2, 9, 7]),
        ("dedupe_keeps_first", [3, 3, 5, 1], [0.1, 0.1, 0.2, 0.3], 3, [3, 5, 1]),
        ("fewer_than_k", [8, 6], [0.5, 0.5], 5, [8, 6]),
        ("empty", [], [], 4, []),
        ("k_one", [11, 12, 13], [0.3, 0.2, 0.2], 1, [12]),
    ]
    gl = []
    for name, idx, dist, k, want in g_cases:
        gi, gd = oracle.global_top_k(np.array(idx, np.uint64), np.array(dist, F), k)
        assert [int(x) for x in gi] == want, (name, gi, want)
        gl.append({"name": name, "indices": idx, "distances": [float(np.float32(d)) for d in dist],
                   "top_k": k, "expected_indices": want,
                   "expected_distances": [float(x) for x in gd]})
    return {"cosine_distance": cos, "interval_by_rank": iv, "compute_global_top_k": gl,
            "note": "hand-derived from the reference source; see make_golden.py"}


def corpus_case(seed, n, dim):
    """Deterministic corpus with edge rows: duplicates, a zero row, near-identical rows."""
    rows = synth_uniform_np(0, n, dim, seed)
    rows[7] = rows[3]            # exact duplicate -> tie broken by index
    rows[11] = 0.0               # zero row -> distance 1.0
    rows[13] = rows[5] * F(2.5)  # parallel -> distance ~0
    rows[17] = rows[5] + F(5e-11)  # within 1e-10 of row 5 -> identical to a query equal to row 5
    return rows


def search_golden():
    cases = []
    spec = [  # (seed, n, dim, n_queries, k, P)
        (101, 2000, 768, 4, 10, 1),
        (102, 2000, 768, 3, 50, 4),
        (103, 5, 768, 2, 10, 4),      # N < k, N < P
        (104, 10, 64, 2, 3, 7),       # (N=10, P=7): empty blocks
        (105, 3000, 96, 5, 100, 3),   # k = 100, small dim
        (106, 1500, 768, 2, 1, 2),
    ]
    out = {}
    for ci, (seed, n, dim, nq, k, P) in enumerate(spec):
        rows = corpus_case(seed, n, dim) if n > 20 else synth_uniform_np(0, n, dim, seed)
        q = synth_uniform_np(0, nq, dim, seed + 1000)
        if n > 20:
            q[0] = rows[5]           # query in corpus (identical shortcut + near-identical row 17)
        if nq > 1:
            q[1] = rows[min(3, n - 1)]
        idx, dist, cnt = oracle.parallel_top_k(rows, q, k, size=P, threads=1)
        for j in range(nq):
            ni, nd = oracle.np_top_k(rows, q[j], k)
            assert np.array_equal(idx[j, :cnt[j]], ni), (seed, j)
            assert np.array_equal(dist[j, :cnt[j]].view(np.uint32), nd.view(np.uint32)), (seed, j)
        pre = f"c{ci}_"
        out[pre + "spec"] = np.array([seed, n, dim, nq, k, P], np.int64)
        out[pre + "idx"] = idx
        out[pre + "dist_bits"] = dist.view(np.uint32)
        out[pre + "count"] = cnt
        cases.append(spec)
    out["n_cases"] = np.array(len(spec))
    return out


def main():
    ka = known_answers()
    with open(os.path.join(HERE, "known_answers.json"), "w") as f:
        json.dump(ka, f, indent=1)
    sg = search_golden()
    np.savez(os.path.join(HERE, "search_golden.npz"), **sg)
    print("wrote", os.listdir(HERE))


if __name__ == "__main__":
    main()
