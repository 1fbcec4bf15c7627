"""Multi-rank runs of the exchange step on CPU (gloo, world size 2 and 3).

Every rank takes its interval_by_rank block (C ABI) and its local top-k lists -- computed by
the oracle here, standing in for the GPU kernel whose parity the gpu tests cover -- and
hands them to the library's exchange + root merge (bsr_gather_global_top_k, the same code
bsr_parallel_top_k_similarity_search runs after its local search), over a host transport:
the library calls back into torch.distributed (gloo) for its all-gathers, where the product
uses RCCL.  The root's result must equal the single-rank answer bit for bit
(src/mpi_helpers/metrics.rs:56-206)."""
import io
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N, D, K = 1203, 96, 15


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _corpus():
    rng = np.random.default_rng(1234)
    rows = rng.uniform(-1, 1, (N, D)).astype(np.float32)
    rows[700] = rows[10]   # duplicate across rank blocks -> tie resolved by index
    rows[1100] = rows[11]
    queries = np.stack([rows[10], rows[11]] + [rng.uniform(-1, 1, D).astype(np.float32) for _ in range(4)])
    return rows, queries


def _init(rank, world, port):
    for p in (os.path.join(ROOT, "better-search-rag-rust_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    return dist


def _local_lists(oracle, rows, rank, world, queries, k, offset_shift=0):
    li = np.zeros((len(queries), k), np.uint64)
    ld = np.zeros((len(queries), k), np.float32)
    lc = np.zeros(len(queries), np.uint32)
    for q, qv in enumerate(queries):
        i, d = oracle.local_top_k(rows, rank, world, k, qv)
        li[q, :len(i)] = i + np.uint64(offset_shift)
        ld[q, :len(d)] = d
        lc[q] = len(i)
    return li, ld, lc


def _worker(rank, world, port, out_path):
    dist = _init(rank, world, port)
    import bsr
    import oracle

    rows, queries = _corpus()
    comm = bsr.Comm.host(dist.group.WORLD)
    assert comm.transport == "host" and comm.size == world
    # 1) the exchange + merge of the parallel search, batch of queries
    iv = bsr.interval_by_rank(rank, world, N)
    li, ld, lc = _local_lists(oracle, rows, rank, world, queries, K)
    for q in range(len(queries)):
        assert all(iv.start_index <= i < max(iv.start_index, iv.end_index) for i in li[q, :lc[q]])
    got = bsr.gather_global_top_k(comm, li, ld, lc, K)
    # 2) a rank whose local search failed contributes an empty list; the others complete
    got_fail = bsr.gather_global_top_k(comm, None if rank == world - 1 else li, None if rank == world - 1 else ld,
                                       None if rank == world - 1 else lc, K)
    # 3) the reference-shaped single-query gather (lists of pairs) through the C exchange
    local = [(int(i), float(d)) for i, d in zip(li[0, :lc[0]], ld[0, :lc[0]])]
    gi, gd = bsr.gather_top_k_results(comm, rank, local)
    # 4) broadcast of the query (src/main.rs:123-125) and the timing report
    tv = np.zeros(D, np.float32)
    if rank == 0:
        tv[:] = rows[10]
    comm.broadcast(tv, 0)
    assert np.array_equal(tv, rows[10])
    rep = bsr.similarity_search_report(comm, rank, 0.5 + rank)
    dist.barrier()
    if rank == 0:
        np.savez(out_path, idx=got[0], dist=got[1], cnt=got[2], fidx=got_fail[0], fdist=got_fail[1],
                 fcnt=got_fail[2], gi=np.array(gi, np.uint64), gd=np.array(gd, np.float32),
                 rep=np.frombuffer(rep.encode(), np.uint8))
    else:
        assert got is None and got_fail is None and gi == [] and gd == [] and rep == ""
    comm.close()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_exchange_matches_single_rank(tmp_path, world, oracle_mod):
    out = str(tmp_path / "res.npz")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    r = np.load(out)
    rows, queries = _corpus()
    wi, wd, wc = oracle_mod.parallel_top_k(rows, queries, K, size=1)
    assert np.array_equal(r["cnt"], wc)
    assert np.array_equal(r["idx"], wi) and np.array_equal(r["dist"].view(np.uint32), wd.view(np.uint32))
    assert list(r["idx"][0, :2]) == [10, 700] and list(r["idx"][1, :2]) == [11, 1100]
    # the last rank contributed nothing: the result is the top-k over the other blocks
    s_last = oracle_mod.interval_by_rank(world - 1, world, N)[0]
    ei, ed, ec = oracle_mod.parallel_top_k(rows[:s_last], queries, K, size=1)
    assert np.array_equal(r["fcnt"], ec) and np.array_equal(r["fidx"], ei)
    assert np.array_equal(r["fdist"].view(np.uint32), ed.view(np.uint32))
    # gather_top_k_results: the rank-order concatenation of the per-rank lists
    want_i, want_d = [], []
    for rk in range(world):
        i, d = oracle_mod.local_top_k(rows, rk, world, K, queries[0])
        want_i.extend(i)
        want_d.extend(d)
    assert list(r["gi"]) == want_i and np.array_equal(r["gd"], np.array(want_d, np.float32))
    rep = r["rep"].tobytes().decode()
    assert rep.splitlines() == [
        "==== PARALLEL PERFORMANCE REPORT ====", "", "Operation: similarity_search",
        "  Min time: 0.5000 sec (Rank 0)", f"  Max time: {world - 0.5:.4f} sec (Rank {world - 1})",
        f"  Avg time: {(0.5 + world - 0.5) / 2:.4f} sec"]


def _worker_edge(rank, world, port, out_path):
    """Edge cases of the exchange: more ranks than rows (empty blocks, the (5,4) case of
    interval_by_rank), overlapping blocks (caller-chosen offsets: the same index arrives
    from two ranks, deduped as the reference's HashSet), k larger than the corpus."""
    dist = _init(rank, world, port)
    import bsr
    import oracle

    comm = bsr.Comm.host(dist.group.WORLD)
    rng = np.random.default_rng(77)
    small = rng.uniform(-1, 1, (2, 8)).astype(np.float32)
    qs = rng.uniform(-1, 1, (3, 8)).astype(np.float32)
    li, ld, lc = _local_lists(oracle, small, rank, world, qs, 4)
    got_small = bsr.gather_global_top_k(comm, li, ld, lc, 4)
    # overlapping: every rank submits the full-corpus list of the same 50 rows
    rows = rng.uniform(-1, 1, (50, 8)).astype(np.float32)
    li, ld, lc = _local_lists(oracle, rows, 0, 1, qs, 6)
    got_overlap = bsr.gather_global_top_k(comm, li, ld, lc, 6)
    if rank == 0:
        np.savez(out_path, si=got_small[0], sd=got_small[1], sc=got_small[2], oi=got_overlap[0],
                 od=got_overlap[1], oc=got_overlap[2])
    comm.close()
    dist.destroy_process_group()


def test_gloo_exchange_edge_cases(tmp_path, oracle_mod):
    world = 3
    out = str(tmp_path / "edge.npz")
    mp.spawn(_worker_edge, args=(world, _free_port(), out), nprocs=world, join=True)
    r = np.load(out)
    rng = np.random.default_rng(77)
    small = rng.uniform(-1, 1, (2, 8)).astype(np.float32)
    qs = rng.uniform(-1, 1, (3, 8)).astype(np.float32)
    rows = rng.uniform(-1, 1, (50, 8)).astype(np.float32)
    wi, wd, wc = oracle_mod.parallel_top_k(small, qs, 4, size=world)
    assert np.array_equal(r["sc"], wc) and (wc == 2).all()
    assert np.array_equal(r["si"][:, :2], wi[:, :2]) and np.array_equal(r["sd"][:, :2].view(np.uint32),
                                                                        wd[:, :2].view(np.uint32))
    wi, wd, wc = oracle_mod.parallel_top_k(rows, qs, 6, size=1)
    assert np.array_equal(r["oc"], wc) and np.array_equal(r["oi"], wi)
    assert np.array_equal(r["od"].view(np.uint32), wd.view(np.uint32))


def _worker_collective_safety(rank, world, port, out_path):
    """bsr_parallel_top_k_similarity_search's collective safety without a GPU: every rank
    passes no index (a local failure before any search), so the library's own header
    exchange, empty contributions and root merge run over gloo.  Then one rank passes a
    different batch size: every rank must be rejected, none left blocked."""
    import warnings
    dist = _init(rank, world, port)
    import bsr

    comm = bsr.Comm.host(dist.group.WORLD)
    q = np.zeros((4, D), np.float32)
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        try:
            res = bsr.parallel_top_k_similarity_search_batch(comm, None, q, K)
            st = 0
        except bsr.BsrError as e:
            res, st = None, e.status
        warned = "|".join(str(x.message) for x in w)
    try:
        bsr.parallel_top_k_similarity_search_batch(comm, None, q[:3] if rank == world - 1 else q, K)
        st2, msg2 = 0, ""
    except bsr.BsrError as e:
        st2, msg2 = e.status, str(e)
    # a rank whose queries fail the Python-side checks (here a float64 tensor) still
    # takes part in the collective -- an empty contribution -- and raises afterwards; nobody hangs
    import torch
    bad_q = torch.zeros((4, D), dtype=torch.float64) if rank == 1 else q
    try:
        bsr.parallel_top_k_similarity_search_batch(comm, None, bad_q, K)
        st3, msg3 = 0, ""
    except bsr.BsrError as e:
        st3, msg3 = e.status, str(e)
    # gather_global_top_k: a malformed local list on one rank, then a batch size
    # that differs on one rank -- every rank raises, before any list moves
    li = np.zeros((4, K), np.uint64)
    ld = np.zeros((4, K), np.float32)
    lc = np.zeros(4, np.uint32)
    msgs = []
    for bad in ((li[:, :K - 1] if rank == 1 else li, ld, lc), (li[:3], ld[:3], lc[:3]) if rank == world - 1 else
                (li, ld, lc)):
        try:
            bsr.gather_global_top_k(comm, *bad, K)
            msgs.append("")
        except bsr.BsrError as e:
            msgs.append(str(e))
    dist.barrier()
    np.savez(f"{out_path}.{rank}.npz", st=st, st2=st2, msg2=np.frombuffer((msg2 or " ").encode(), np.uint8),
             st3=st3, msg3=np.frombuffer((msg3 or " ").encode(), np.uint8),
             g1=np.frombuffer((msgs[0] or " ").encode(), np.uint8),
             g2=np.frombuffer((msgs[1] or " ").encode(), np.uint8),
             warned=np.frombuffer((warned or " ").encode(), np.uint8),
             cnt=res[2] if res is not None else np.zeros(0, np.uint32), none=res is None)
    comm.close()
    dist.destroy_process_group()


def test_gloo_parallel_search_collective_safety(tmp_path):
    world = 3
    out = str(tmp_path / "cs")
    mp.spawn(_worker_collective_safety, args=(world, _free_port(), out), nprocs=world, join=True)
    r = [np.load(f"{out}.{i}.npz") for i in range(world)]
    # no index anywhere: the root reports BSR_PARTIAL (a warning) with every list empty;
    # the other ranks raise their local error
    assert int(r[0]["st"]) == 0 and not bool(r[0]["none"]) and not r[0]["cnt"].any() and len(r[0]["cnt"]) == 4
    assert b"null index" in r[0]["warned"].tobytes()
    for i in range(1, world):
        assert int(r[i]["st"]) == -1 and bool(r[i]["none"])
    # batch sizes that disagree: all ranks rejected, collectively
    for i in range(world):
        assert int(r[i]["st2"]) == -1 and b"disagree on the batch shape" in r[i]["msg2"].tobytes()
    # rank 1's float64 queries: it raises its own check's error after the collective; the others
    # completed it (no index anywhere here: rank 2 reports its null index, the root its partial result)
    assert int(r[1]["st3"]) == -1 and b"contiguous float32" in r[1]["msg3"].tobytes()
    assert int(r[0]["st3"]) == 0
    assert int(r[2]["st3"]) == -1 and b"null index" in r[2]["msg3"].tobytes()
    # gather_global_top_k: malformed lists on rank 1, then Q = 3 on the last rank: all raise
    for i in range(world):
        g1, g2 = r[i]["g1"].tobytes(), r[i]["g2"].tobytes()
        assert (b"local lists must be" if i == 1 else b"rank(s) [1] passed invalid local lists") in g1, (i, g1)
        assert b"disagree on the batch shape" in g2, (i, g2)
