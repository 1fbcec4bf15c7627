"""The multi-rank composition on the GPU: bsr_parallel_top_k_similarity_search with 2 and 3
rank processes on the one GPU, each searching its interval_by_rank block with the HIP path,
the library's own exchange (over gloo: Comm.host) and the root's device merge
(src/mpi_helpers/metrics.rs:174-206).  The root's lists must equal the oracle's bit for bit.

Failure cases (collective safety, :185-191): a rank whose GPU search fails (its index was
built with max_k < k) still completes the exchange with an empty list; the root's result is
then the global top-k over the other blocks.  A failing non-root rank raises its error; a
failing root warns (BSR_PARTIAL) and returns the other blocks' result, as the reference's
root returns Some(..).  Ranks that disagree on the batch shape are all rejected before any
list is exchanged."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import mr_worker

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(world, case, tmp_path):
    out = str(tmp_path / f"mr_{case}_{world}")
    port = _free_port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mr_worker.py"), "--rank", str(r), "--world",
                               str(world), "--port", str(port), "--case", case, "--out", out],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env) for r in range(world)]
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=100)
            logs.append(o.decode(errors="replace"))
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    for r, p in enumerate(procs):
        assert p.returncode == 0, f"rank {r} exited {p.returncode}:\n{logs[r][-3000:]}"
    return [dict(np.load(f"{out}.rank{r}.npz")) for r in range(world)]


@pytest.fixture(scope="module")
def corpus(bsr_mod):
    return bsr_mod.synth_uniform_np(0, mr_worker.N, mr_worker.D, mr_worker.SEED), mr_worker.queries()


def _want(oracle_mod, rows, q, lo=0, hi=None):
    """Oracle global top-k over rows [lo, hi) with global indices."""
    hi = rows.shape[0] if hi is None else hi
    wi, wd, wc = oracle_mod.parallel_top_k(np.ascontiguousarray(rows[lo:hi]), q, mr_worker.K, size=4, threads=4)
    return wi + np.uint64(lo), wd, wc


def _same(r, want):
    wi, wd, wc = want
    assert np.array_equal(r["cnt"], wc)
    for q in range(len(wc)):
        c = int(wc[q])
        assert np.array_equal(r["idx"][q, :c], wi[q, :c]), q
        assert np.array_equal(r["dist"][q, :c].view(np.uint32), wd[q, :c].view(np.uint32)), q


@pytest.mark.parametrize("world,case", [(2, "normal"), (3, "normal"), (8, "normal"), (3, "no_gtau"),
                                        (3, "gtau_fallback")])
def test_parallel_search_multirank_matches_oracle(bsr_mod, oracle_mod, gpu, corpus, tmp_path, world, case):
    """normal: the global-threshold search (every rank emits against the threshold selected from
    every rank's sample, rescores all it emitted; the merged lists certified); no_gtau: the
    standard path (local certified searches); gtau_fallback: every merged list uncertified, so
    every query takes the collective fallback -- all bit-exact against the oracle."""
    rows, q = corpus
    res = _run(world, case, tmp_path)
    for r in range(world):
        assert int(res[r]["status"]) == 0, res[r]["msg"].tobytes()
    for r in range(1, world):
        assert int(res[r]["is_none"]) == 1  # the reference's None
    _same(res[0], _want(oracle_mod, rows, q))
    # self-matches: the planted rows come first at distance 0
    assert [int(res[0]["idx"][i, 0]) for i in range(3)] == [0, mr_worker.N // 2 + 3, mr_worker.N - 1]
    assert not res[0]["dist"][:3, 0].any()
    nq = len(q)
    if case == "normal":
        # the global threshold: ~256 rows per query over the whole corpus, not per rank
        total = sum(int(res[r]["emitted"]) for r in range(world))
        assert total / nq < 600, total / nq
        assert int(res[0]["fallback"]) == 0
    if case == "gtau_fallback":
        assert int(res[0]["fallback"]) == nq


def test_parallel_search_failing_rank(bsr_mod, oracle_mod, gpu, corpus, tmp_path):
    world = 3
    rows, q = corpus
    res = _run(world, "fail_last", tmp_path)
    s_last = bsr_mod.interval_by_rank(world - 1, world, mr_worker.N).start_index
    # the failing rank raised its own error after the exchange
    assert int(res[world - 1]["status"]) == -1 and b"max_k" in res[world - 1]["msg"].tobytes()
    assert int(res[1]["status"]) == 0 and int(res[0]["status"]) == 0
    # the root's result is the top-k over the other blocks
    _same(res[0], _want(oracle_mod, rows, q, 0, s_last))
    assert int(res[0]["idx"][2, 0]) != mr_worker.N - 1  # the last block's self-match is missing


def test_parallel_search_header_hook_fault(bsr_mod, oracle_mod, gpu, corpus, tmp_path):
    # a header collective that failed before it was posted must be posted again
    # with the error status (no rank left blocked, no mismatched collectives)
    world = 3
    rows, q = corpus
    res = _run(world, "hook_fault", tmp_path)
    s_last = bsr_mod.interval_by_rank(world - 1, world, mr_worker.N).start_index
    assert int(res[world - 1]["status"]) == -4 and b"injected fault" in res[world - 1]["msg"].tobytes()
    assert int(res[1]["status"]) == 0 and int(res[0]["status"]) == 0
    _same(res[0], _want(oracle_mod, rows, q, 0, s_last))


def test_parallel_search_failing_root(bsr_mod, oracle_mod, gpu, corpus, tmp_path):
    world = 2
    rows, q = corpus
    res = _run(world, "fail_root", tmp_path)
    s1 = bsr_mod.interval_by_rank(1, world, mr_worker.N).start_index
    # the root warns (BSR_PARTIAL) and returns the other block's global top-k
    assert int(res[0]["status"]) == 0 and int(res[0]["is_none"]) == 0
    assert b"local search failed" in res[0]["warned"].tobytes()
    assert int(res[1]["status"]) == 0
    _same(res[0], _want(oracle_mod, rows, q, s1))


def test_parallel_search_shape_mismatch_rejected(bsr_mod, gpu, tmp_path):
    world = 3
    res = _run(world, "shape", tmp_path)
    for r in range(world):
        assert int(res[r]["status"]) == -1, (r, res[r]["msg"].tobytes())
        assert b"disagree on the batch shape" in res[r]["msg"].tobytes()
