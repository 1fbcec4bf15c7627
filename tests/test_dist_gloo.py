"""World-size-2 (and 3) gloo runs of the distributed composition on CPU: each rank takes its
interval_by_rank block (C ABI), computes its local top-k (the oracle stands in for the GPU
kernel here -- the GPU kernel's parity is covered by the gpu tests), gathers through
torch.distributed (gather_top_k_results) and the root merges with the C ABI's
compute_global_top_k.  The result must equal the single-rank answer bit for bit."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    for p in (os.path.join(ROOT, "better-search-rag-rust_amd"), os.path.join(ROOT, "oracle")):
        sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    import bsr
    import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(1234)
    N, D, K = 1203, 96, 15
    rows = rng.uniform(-1, 1, (N, D)).astype(np.float32)
    rows[700] = rows[10]  # duplicate across rank blocks -> tie resolved by index
    queries = np.stack([rows[10], rng.uniform(-1, 1, D).astype(np.float32)])
    results = []
    for q in queries:
        iv = bsr.interval_by_rank(rank, world, N)
        li, ld = oracle.local_top_k(rows, rank, world, K, q)
        assert all(iv.start_index <= i < max(iv.start_index, iv.end_index) for i in li)
        local = [(int(i), float(d)) for i, d in zip(li, ld)]
        gi, gd = bsr.gather_top_k_results(dist.group.WORLD, rank, local)
        if rank == bsr.ROOT:
            results.append(bsr.compute_global_top_k(gi, gd, K))
        else:
            assert gi == [] and gd == []
    dist.barrier()
    if rank == 0:
        np.save(out_path, np.array([[i for i, _ in r] for r in results], np.int64))
        np.save(out_path + ".d.npy", np.array([[d for _, d in r] for r in results], np.float32))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_distributed_matches_single_rank(tmp_path, world, oracle_mod):
    out = str(tmp_path / "res.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got_i = np.load(out)
    got_d = np.load(out + ".d.npy")
    rng = np.random.default_rng(1234)
    N, D, K = 1203, 96, 15
    rows = rng.uniform(-1, 1, (N, D)).astype(np.float32)
    rows[700] = rows[10]
    queries = np.stack([rows[10], rng.uniform(-1, 1, D).astype(np.float32)])
    wi, wd, wc = oracle_mod.parallel_top_k(rows, queries, K, size=1)
    assert np.array_equal(got_i, wi.astype(np.int64))
    assert np.array_equal(got_d.view(np.uint32), wd.view(np.uint32))
    assert got_i[0, 0] == 10 and got_i[0, 1] == 700
