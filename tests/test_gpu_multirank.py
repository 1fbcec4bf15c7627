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


def _run(world, case, tmp_path, timeout=100):
    out = str(tmp_path / f"mr_{case}_{world}")
    port = _free_port()
    env = dict(os.environ, PYTHONUNBUFFERED="1")
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, "mr_worker.py"), "--rank", str(r), "--world",
                               str(world), "--port", str(port), "--case", case, "--out", out],
                              stdout=subprocess.PIPE, stderr=subprocess.STDOUT, env=env) for r in range(world)]
    logs = []
    try:
        for p in procs:
            o, _ = p.communicate(timeout=timeout)
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


def test_parallel_search_phase_a_faults(bsr_mod, oracle_mod, gpu, corpus, tmp_path):
    """a failing global-threshold phase A never leaves a peer blocked.  Before the
    header (phase_a0) the failure rides in the header and every rank takes the standard path (the
    failing rank contributes an empty list); after it (phase_a1) the rank stays in every collective
    with a poisoned contribution, no merged list certifies, and the collective fallback -- where
    the rank searches again -- gives the complete result."""
    world = 3
    rows, q = corpus
    s_last = bsr_mod.interval_by_rank(world - 1, world, mr_worker.N).start_index
    res = _run(world, "phase_a0", tmp_path)
    assert int(res[world - 1]["status"]) == -3 and b"phase A, query prep" in res[world - 1]["msg"].tobytes()
    assert int(res[1]["status"]) == 0 and int(res[0]["status"]) == 0
    _same(res[0], _want(oracle_mod, rows, q, 0, s_last))
    res = _run(world, "phase_a1", tmp_path)
    assert int(res[world - 1]["status"]) == -3 and b"phase A, sample pass" in res[world - 1]["msg"].tobytes()
    assert int(res[1]["status"]) == 0 and int(res[0]["status"]) == 0
    assert int(res[0]["fallback"]) == len(q)
    _same(res[0], _want(oracle_mod, rows, q))


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


# ---- the global-threshold path at BASELINE's full sizes -----------------
@pytest.mark.parametrize("case", ["c3", "c5"])
def test_global_threshold_full_size_8_ranks(bsr_mod, oracle_mod, gpu, tmp_path, case):
    """The N > 1 product path at the configs an 8-GPU run executes, with 8 rank processes on the
    one GPU over the host transport: configs[2] (10M f32 rows, 8 x 1.25M, 1000 queries, k = 10)
    and configs[4] (50M bf16 rows, 8 x 6.25M, 4096 queries, k = 100: ks = 48 sample keys per
    query, a 1.5 MB key all-gather, k_global_tau, rescore of every emitted row, the merge and its
    certification).  Asserts: the global-threshold path was taken on every rank (every emitted
    row rescored: no k' candidates) with about 1/8 of a single shard's emission per rank, every
    merged list count-correct and in (distance, index) order, the planted self-matches first,
    and a subset of queries -- one planted in the last shard -- bit-exact against the oracle over
    the whole corpus (src/mpi_helpers/metrics.rs:141-171,174-206)."""
    import torch
    import test_gpu_full_size as fs
    n, nq, k, bf16, plant = mr_worker.PRESETS[case]
    world = 8
    res = _run(world, case, tmp_path, timeout=480)
    for r in range(world):
        assert int(res[r]["status"]) == 0, res[r]["msg"].tobytes()
        # the global-threshold path reports no k' candidates (every emitted row was rescored)
        assert int(res[r]["candidates"]) == 0, (r, int(res[r]["candidates"]))
    per_rank = [int(res[r]["emitted"]) / nq for r in range(world)]
    single_shard = 256 if k <= 10 else 1600  # rows per query one shard of the whole corpus emits
    assert max(per_rank) < single_shard * 3 / world, per_rank
    fb = int(res[0]["fallback"])
    print(f"{case}: emitted per query per rank {[round(x, 1) for x in per_rank]}, fallback queries {fb}")
    assert fb <= nq // 200, fb
    for r in range(1, world):
        assert int(res[r]["is_none"]) == 1
    got = (res[0]["idx"].astype(np.uint64), res[0]["dist"], res[0]["cnt"].astype(np.uint32))
    fs._check_properties(got, n, k, f"{case} merged")
    for pos, row in plant:
        assert got[0][pos, 0] == row and got[1][pos, 0] == 0.0, (pos, row, got[0][pos, :3])
    q = mr_worker.device_queries(bsr_mod, torch, nq, plant, bf16)
    sub = [0, 1, 2, 4, nq - 1]
    want = fs._chunked_oracle(bsr_mod, oracle_mod, n, q[sub].cpu().numpy(), k, bf16=bf16)
    fs._assert_same(got, want, sub, f"{case} 8 ranks vs oracle")


# ---- the loopback communicator: RCCL's enqueue-only control flow ---------
def test_loopback_replicated_matches_own_shard(bsr_mod, oracle_mod, gpu, corpus):
    """A loopback communicator (one process acting as rank 0 of 8; every all-gather one device
    kernel where ncclAllGather sits, no host wait) replicating this rank's contributions: the
    parallel search runs the RCCL branch -- header on the communicator's stream, keys and results
    on the index's stream, the merge publishing its result -- and its merged lists are the rank's
    own top-k, bit for bit.  A non-root loopback rank returns None."""
    rows, q = corpus
    ix = bsr_mod.Index(mr_worker.D, max_k=64, device=0)
    ix.load(rows, 0)
    comm = bsr_mod.Comm.loopback(0, 8, 0)
    got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, mr_worker.K)
    st = ix.last_stats()
    assert st.n_candidates == 0  # the global-threshold path (every emitted row rescored)
    # (replicated contributions: the union is this rank's ~1/8-size emission, so many merged lists
    # fail certification and take the collective fallback -- exact either way)
    print(f"loopback (replicated, P = 8): {st.n_fallback} of {len(q)} queries through the fallback")
    _same({"idx": got[0], "dist": got[1], "cnt": got[2]}, _want(oracle_mod, rows, q))
    again = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, mr_worker.K)
    assert all(np.array_equal(a, b) for a, b in zip(got, again))
    # the standard path through the loopback (the three list all-gathers, the device root merge)
    c3 = bsr_mod.Comm.loopback(3, 8, 0)
    assert bsr_mod.parallel_top_k_similarity_search_batch(c3, ix, q, mr_worker.K) is None
    small = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q[:5], mr_worker.K)  # (<= 16: standard path)
    _same({"idx": small[0], "dist": small[1], "cnt": small[2]}, _want(oracle_mod, rows, q[:5]))
    c3.close()
    comm.close()
    ix.close()


@pytest.mark.parametrize("dim,k", [(200, 10), (200, 70), (64, 33)])
def test_loopback_global_threshold_other_widths(bsr_mod, oracle_mod, gpu, dim, k):
    """The global-threshold path (k_rescore_flat's generic-width walk, partial last chunks, lists
    of more than 64 entries) through a replicating loopback communicator on rows of other widths:
    the merged lists are the rank's own top-k, bit for bit."""
    rng = np.random.default_rng(dim * 1000 + k)
    rows = rng.uniform(-1, 1, (40000, dim)).astype(np.float32)
    q = rng.uniform(-1, 1, (40, dim)).astype(np.float32)
    q[0] = rows[7]
    ix = bsr_mod.Index(dim, max_k=128, device=0)
    ix.load(rows, 0)
    comm = bsr_mod.Comm.loopback(0, 8, 0)
    got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, k)
    assert ix.last_stats().n_candidates == 0  # (the global-threshold path)
    wi, wd, wc = oracle_mod.parallel_top_k(rows, q, k, size=4, threads=4)
    assert np.array_equal(got[2], wc)
    for j in range(len(q)):
        c = int(wc[j])
        assert np.array_equal(got[0][j, :c], wi[j, :c]), j
        assert np.array_equal(got[1][j, :c].view(np.uint32), wd[j, :c].view(np.uint32)), j
    assert got[0][0, 0] == 7
    comm.close()
    ix.close()


def test_loopback_replays_recorded_run(bsr_mod, gpu, corpus, tmp_path):
    """Rank 0 of a real 3-rank run (host transport) records its all-gathers; a loopback
    communicator replaying them on rank 0's shard alone reproduces that run's global result bit
    for bit, every all-gather replayed (the bench's per-rank step of an N-rank run)."""
    world = 3
    res = _run(world, "record", tmp_path)
    assert int(res[0]["status"]) == 0, res[0]["msg"].tobytes()
    script = [res[0][f"rec{i}"] for i in range(int(res[0]["n_rec"]))]
    assert len(script) == 3  # header, sample keys, result buffers
    rows, q = corpus
    iv = bsr_mod.interval_by_rank(0, world, mr_worker.N)
    ix = bsr_mod.Index(mr_worker.D, max_k=64, device=0)
    ix.load(rows[iv.start_index:iv.end_index], iv.start_index)
    comm = bsr_mod.Comm.loopback(0, world, 0, script)
    for rep in range(2):
        got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, mr_worker.K)
        _same({"idx": got[0], "dist": got[1], "cnt": got[2]},
              (res[0]["idx"], res[0]["dist"], res[0]["cnt"]))
    assert comm.loopback_stats() == (6, 0)
    # root outputs in coherent pinned host memory: the merge writes the rows there directly
    oi = bsr_mod.host_array((len(q), mr_worker.K), np.uint64)
    od = bsr_mod.host_array((len(q), mr_worker.K), np.float32)
    oc = bsr_mod.host_array(len(q), np.uint32)
    oi[:] = 7
    od[:] = -1.0
    oc[:] = 999
    qq = np.ascontiguousarray(q, np.float32)
    st = bsr_mod.lib().bsr_parallel_top_k_similarity_search(comm._h, ix._h, qq.ctypes.data, len(q), mr_worker.K,
                                                            oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
    assert st == 0, bsr_mod.lib().bsr_last_error()
    _same({"idx": oi, "dist": od, "cnt": oc}, (res[0]["idx"], res[0]["dist"], res[0]["cnt"]))
    assert comm.loopback_stats() == (9, 0)
    comm.close()
    ix.close()


# ---- real RCCL at P = 1: every collective of the parallel search ---------
def _search_into_host_arrays(bsr_mod, comm, ix, q, k):
    """The parallel search with the root's outputs in coherent pinned host memory (bsr_host_alloc):
    the global-threshold merge writes its rows there directly (BSR_PATH_DIRECT_OUT)."""
    oi = bsr_mod.host_array((len(q), k), np.uint64)
    od = bsr_mod.host_array((len(q), k), np.float32)
    oc = bsr_mod.host_array(len(q), np.uint32)
    oi[:] = 7
    od[:] = -1.0
    oc[:] = 999
    qq = np.ascontiguousarray(q, np.float32)
    st = bsr_mod.lib().bsr_parallel_top_k_similarity_search(comm._h, ix._h, qq.ctypes.data, len(q), k,
                                                            oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
    assert st == 0, bsr_mod.lib().bsr_last_error()
    return {"idx": oi, "dist": od, "cnt": oc}


def test_rccl_forced_collectives_single_rank(bsr_mod, oracle_mod, gpu, corpus, monkeypatch):
    """BSR_FORCE_COLLECTIVES=1 makes a one-rank RCCL communicator take the multi-rank branch
    (src/mpi_helpers/metrics.rs:174-206 with size 1), so every RCCL call the 8-GPU run makes runs
    here on hardware: the header all-gather on the communicator's stream; the global threshold's
    sample-key and result-buffer all-gathers on the index's stream, the merge, its certification
    and publication (into the caller's pinned outputs directly, with the uncertified queries'
    rows patched in); the collective fallback; and the standard path's group of three list
    all-gathers with the device merge.  Every result bit-exact against the oracle."""
    monkeypatch.setenv("BSR_FORCE_COLLECTIVES", "1")
    P = bsr_mod
    rows, q = corpus
    want = _want(oracle_mod, rows, q)
    ix = bsr_mod.Index(mr_worker.D, max_k=64, device=0)
    ix.load(rows, 0)
    comm = bsr_mod.Comm(bsr_mod.Comm.unique_id(), 0, 1, 0)
    gt_bits = P.BSR_PATH_COLLECTIVE | P.BSR_PATH_GLOBAL_TAU
    # 1. the global-threshold search, twice (buffers reused)
    for rep in range(2):
        got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, mr_worker.K)
        st = ix.last_stats()
        assert st.search_path & gt_bits == gt_bits, (rep, st.search_path)
        assert st.n_candidates == 0 and st.n_fallback == 0, (st.n_candidates, st.n_fallback)
        _same({"idx": got[0], "dist": got[1], "cnt": got[2]}, want)
    # 2. the root's outputs in coherent pinned memory: the merge writes them directly
    r = _search_into_host_arrays(bsr_mod, comm, ix, q, mr_worker.K)
    assert ix.last_stats().search_path == gt_bits | P.BSR_PATH_DIRECT_OUT, ix.last_stats().search_path
    _same(r, want)
    # 3. no merged list certifies: every query's rows come from the collective fallback (the
    # standard path's RCCL group and device merge), patched into the direct outputs
    monkeypatch.setenv("BSR_INJECT_FAULT", "gtau_uncertified")
    r = _search_into_host_arrays(bsr_mod, comm, ix, q, mr_worker.K)
    st = ix.last_stats()
    assert st.search_path == gt_bits | P.BSR_PATH_DIRECT_OUT | P.BSR_PATH_FALLBACK, st.search_path
    assert st.n_fallback == len(q)
    _same(r, want)
    # 4. phase A fails after the header (poisoned contribution): every query through the fallback,
    # where this rank searches again -- the root's rows are complete
    monkeypatch.setenv("BSR_INJECT_FAULT", "phase_a1")
    got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, mr_worker.K)
    st = ix.last_stats()
    assert st.search_path & P.BSR_PATH_FALLBACK and st.n_fallback == len(q), (st.search_path, st.n_fallback)
    _same({"idx": got[0], "dist": got[1], "cnt": got[2]}, want)
    monkeypatch.delenv("BSR_INJECT_FAULT")
    # 5. the standard path: header from the search's hook, the group of three all-gathers, the
    # device merge -- a 40-query batch with the global threshold off, and a 5-query batch (<= 16)
    monkeypatch.setenv("BSR_GLOBAL_TAU", "0")
    got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, mr_worker.K)
    assert ix.last_stats().search_path == P.BSR_PATH_COLLECTIVE | P.BSR_PATH_DEVICE_MERGE
    _same({"idx": got[0], "dist": got[1], "cnt": got[2]}, want)
    monkeypatch.delenv("BSR_GLOBAL_TAU")
    small = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q[:5], mr_worker.K)
    assert ix.last_stats().search_path == P.BSR_PATH_COLLECTIVE | P.BSR_PATH_DEVICE_MERGE
    _same({"idx": small[0], "dist": small[1], "cnt": small[2]}, _want(oracle_mod, rows, q[:5]))
    # 6. without the switch a one-rank communicator skips the header and the global threshold: the
    # local search, then the standard exchange (one rank's lists) and the device merge
    monkeypatch.delenv("BSR_FORCE_COLLECTIVES")
    got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, mr_worker.K)
    assert ix.last_stats().search_path == P.BSR_PATH_COLLECTIVE | P.BSR_PATH_DEVICE_MERGE
    _same({"idx": got[0], "dist": got[1], "cnt": got[2]}, want)
    comm.close()
    ix.close()


def test_rccl_forced_collectives_configs2_shard(bsr_mod, oracle_mod, gpu, monkeypatch):
    """The same at an 8-GPU run's operating point: rank 0's configs[2] shard (1.25M of the 10M
    synthetic rows, 1000 queries on the device, k = 10) through a one-rank RCCL communicator with
    the collectives forced -- the global-threshold path with every all-gather real RCCL; a subset
    of queries (planted rows among them) bit-exact against the oracle over the shard."""
    import torch
    import test_gpu_full_size as fs
    monkeypatch.setenv("BSR_FORCE_COLLECTIVES", "1")
    n_total, nq, k = 10_000_000, 1000, 10
    iv = bsr_mod.interval_by_rank(0, 8, n_total)
    n = iv.get_count()
    rows = torch.empty((n, mr_worker.D), dtype=torch.float32, device="cuda:0")
    bsr_mod.synth_uniform(rows.data_ptr(), 0, n, mr_worker.D, mr_worker.SEED)
    torch.cuda.synchronize()
    ix = bsr_mod.Index(mr_worker.D, max_k=k, device=0)
    ix.load(rows, 0)
    del rows
    torch.cuda.empty_cache()
    plant = [(0, 0), (1, n - 1), (2, 600_001)]
    q = mr_worker.device_queries(bsr_mod, torch, nq, plant, False)
    comm = bsr_mod.Comm(bsr_mod.Comm.unique_id(), 0, 1, 0)
    for rep in range(2):
        got = bsr_mod.parallel_top_k_similarity_search_batch(comm, ix, q, k)
        st = ix.last_stats()
        bits = bsr_mod.BSR_PATH_COLLECTIVE | bsr_mod.BSR_PATH_GLOBAL_TAU
        assert st.search_path & bits == bits, st.search_path
        assert st.n_fallback <= nq // 200, st.n_fallback
        fs._check_properties(got, n, k, "forced collectives, 1.25M shard")
        for pos, row in plant:
            assert got[0][pos, 0] == row and got[1][pos, 0] == 0.0, (pos, row, got[0][pos, :3])
    sub = [0, 1, 2, 5, nq - 1]
    want = fs._chunked_oracle(bsr_mod, oracle_mod, n, q[sub].cpu().numpy(), k)
    fs._assert_same(got, want, sub, "forced collectives, 1.25M shard vs oracle")
    comm.close()
    ix.close()
