"""One rank of the multi-rank parallel search (tests/test_gpu_multirank.py): a separate
process per rank, all on the one GPU, the exchange over gloo (bsr.Comm.host).

Every rank loads its interval_by_rank(rank, world, N) block of the synthetic corpus (global
offset), then calls bsr_parallel_top_k_similarity_search on the whole query batch
(src/mpi_helpers/metrics.rs:174-206).  Cases:
  normal     every rank searches;
  fail_last  the last rank's index has max_k < k, so its GPU search fails;
  fail_root  the same on rank 0;
  shape      the last rank passes one query fewer (collective rejection);
  hook_fault the last rank's header all-gather fails before it is posted (BSR_INJECT_FAULT):
             the rank must still post it, with its error status;
  gtau_fallback  no merged list of the global-threshold search certifies (BSR_INJECT_FAULT):
             every query takes the collective fallback (the standard parallel search);
  no_gtau    the global threshold turned off (BSR_GLOBAL_TAU=0): the standard parallel search.
  phase_a0   the last rank's global-threshold phase A fails before its header (BSR_INJECT_FAULT):
             the header carries the failure, every rank takes the standard path;
  phase_a1   the same after its header: the rank takes part in every collective, poisoned, and
             every query takes the collective fallback.
  record     as normal, and every all-gather's receive buffer is recorded (Comm.host's record):
             the script a loopback communicator replays (tests/test_gpu_multirank.py).
  c3, c5     BASELINE configs at full size on the global-threshold path: configs[2]
             (10M f32 rows, 8 ranks x 1.25M, 1000 queries, k = 10) and configs[4] (50M bf16 rows,
             8 ranks x 6.25M, 4096 queries, k = 100).  The shards are generated on the GPU and
             loaded one rank at a time (configs[4]: ~24 GB per rank resident, ~34 GB while
             loading, 288 GB per GPU); queries on the device, with planted corpus rows.
The rank writes {status, message, and on the root the lists} to <out>.rank<r>.npz.
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "better-search-rag-rust_amd"), ROOT):
    sys.path.insert(0, p)

N, D, K, SEED = 60000, 768, 10, 42

# full-size presets: (corpus rows, queries, k, bf16 corpus, planted (query position, corpus row))
PRESETS = {
    "c3": (10_000_000, 1000, 10, False, [(0, 0), (1, 10_000_000 - 1), (2, 5_600_000), (3, 1_250_000)]),
    "c5": (50_000_000, 4096, 100, True, [(0, 0), (1, 50_000_000 - 1), (2, 43_750_123), (3, 6_250_000),
                                          (4, 31_000_007)]),
}


def device_queries(bsr, torch, nq, plant, bf16):
    """nq seed-43 queries on cuda:0; position p of `plant` is corpus row r (its bf16 rounding
    for a bf16 corpus: the stored row exactly)."""
    q = torch.empty((nq, D), dtype=torch.float32, device="cuda:0")
    bsr.synth_uniform(q.data_ptr(), 0, nq, D, 43)
    for pos, row in plant:
        bsr.synth_uniform(q[pos:pos + 1].data_ptr(), row, 1, D, SEED)
        if bf16:
            q[pos:pos + 1] = q[pos:pos + 1].to(torch.bfloat16).to(torch.float32)
    torch.cuda.synchronize()
    return q


def queries():
    """Rows 0, N/2 + 3 and N - 1 of the corpus (self-matches in the first, a middle and the
    last block), then random queries up to 40."""
    import bsr
    q = [bsr.synth_uniform_np(r, 1, D, SEED)[0] for r in (0, N // 2 + 3, N - 1)]
    rng = np.random.default_rng(5)
    q += list(rng.uniform(-1, 1, (37, D)).astype(np.float32))
    return np.ascontiguousarray(np.stack(q), np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--world", type=int, required=True)
    ap.add_argument("--port", type=int, required=True)
    ap.add_argument("--case", default="normal")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(a.port)
    if a.case == "hook_fault":
        os.environ["BSR_INJECT_FAULT"] = f"header_hook:{a.world - 1}"
    if a.case == "gtau_fallback":
        os.environ["BSR_INJECT_FAULT"] = "gtau_uncertified"
    if a.case in ("phase_a0", "phase_a1"):
        os.environ["BSR_INJECT_FAULT"] = f"{a.case}:{a.world - 1}"
    if a.case == "no_gtau":
        os.environ["BSR_GLOBAL_TAU"] = "0"
    import torch  # noqa: F401  (before libbsr: one HIP runtime per process, tests/conftest.py)
    import torch.distributed as dist
    import bsr

    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    comm = bsr.Comm.host(dist.group.WORLD)
    if a.case in PRESETS:
        return preset_main(a, dist, comm, bsr)
    iv = bsr.interval_by_rank(a.rank, a.world, N)
    n_local = iv.get_count()
    failing = (a.case == "fail_last" and a.rank == a.world - 1) or (a.case == "fail_root" and a.rank == 0)
    ix = bsr.Index(D, max_k=(K - 1) if failing else 64, device=0)
    ix.load(bsr.synth_uniform_np(iv.start_index, n_local, D, SEED), iv.start_index)
    q = queries()
    if a.case == "shape" and a.rank == a.world - 1:
        q = q[:-1]
    status, msg, res, warned = 0, "", None, []
    if a.case == "record":
        comm.record = []
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        try:
            res = bsr.parallel_top_k_similarity_search_batch(comm, ix, q, K)
        except bsr.BsrError as e:
            status, msg = e.status, str(e)
        warned = [str(x.message) for x in w]
    dist.barrier()
    st = ix.last_stats()
    out = {"status": np.int32(status), "msg": np.frombuffer(msg.encode() or b" ", np.uint8),
           "emitted": np.uint64(st.n_emitted), "fallback": np.uint32(st.n_fallback),
           "warned": np.frombuffer(("|".join(warned) or " ").encode(), np.uint8)}
    if res is not None:
        out.update(idx=res[0], dist=res[1], cnt=res[2])
    if a.case == "record":
        out["n_rec"] = np.int32(len(comm.record))
        for i, buf in enumerate(comm.record):
            out[f"rec{i}"] = buf
    if a.rank == 0 or res is None:
        out["is_none"] = np.int32(res is None)
    np.savez(f"{a.out}.rank{a.rank}.npz", **out)
    print(f"rank {a.rank}: status {status} graph_replay {st.graph_replay} emitted {st.n_emitted}", flush=True)
    comm.close()
    ix.close()
    dist.destroy_process_group()


def preset_main(a, dist, comm, bsr):
    import time
    import torch
    n_total, nq, k, bf16, plant = PRESETS[a.case]
    iv = bsr.interval_by_rank(a.rank, a.world, n_total)
    s0, n_local = iv.start_index, iv.get_count()
    ix = bsr.Index(D, max_k=k, device=0, dtype=bsr.BSR_BF16 if bf16 else bsr.BSR_F32)
    t0 = time.perf_counter()
    for r in range(a.world):  # one rank at a time: the load's peak memory is per rank
        if r == a.rank:
            rows = torch.empty((n_local, D), dtype=torch.float32, device="cuda:0")
            bsr.synth_uniform(rows.data_ptr(), s0, n_local, D, SEED)
            torch.cuda.synchronize()
            if bf16:
                rows = rows.to(torch.bfloat16)
            ix.load(rows, s0)
            del rows
            torch.cuda.empty_cache()
        dist.barrier()
    load_s = time.perf_counter() - t0
    q = device_queries(bsr, torch, nq, plant, bf16)
    status, msg, res = 0, "", None
    t0 = time.perf_counter()
    try:
        res = bsr.parallel_top_k_similarity_search_batch(comm, ix, q, k)
    except bsr.BsrError as e:
        status, msg = e.status, str(e)
    search_s = time.perf_counter() - t0
    st = ix.last_stats()
    out = {"status": np.int32(status), "msg": np.frombuffer(msg.encode() or b" ", np.uint8),
           "emitted": np.uint64(st.n_emitted), "fallback": np.uint32(st.n_fallback),
           "candidates": np.uint32(st.n_candidates), "n_local": np.uint64(n_local)}
    if res is not None:
        out.update(idx=res[0], dist=res[1], cnt=res[2])
    out["is_none"] = np.int32(res is None)
    np.savez(f"{a.out}.rank{a.rank}.npz", **out)
    print(f"rank {a.rank}: {a.case} status {status} emitted/query {st.n_emitted / nq:.1f} fallback {st.n_fallback} "
          f"candidates {st.n_candidates} load {load_s:.1f} s search {search_s:.2f} s", flush=True)
    dist.barrier()
    comm.close()
    ix.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
