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
    if a.case == "no_gtau":
        os.environ["BSR_GLOBAL_TAU"] = "0"
    import torch  # noqa: F401  (before libbsr: one HIP runtime per process, tests/conftest.py)
    import torch.distributed as dist
    import bsr

    dist.init_process_group("gloo", rank=a.rank, world_size=a.world)
    comm = bsr.Comm.host(dist.group.WORLD)
    iv = bsr.interval_by_rank(a.rank, a.world, N)
    n_local = iv.get_count()
    failing = (a.case == "fail_last" and a.rank == a.world - 1) or (a.case == "fail_root" and a.rank == 0)
    ix = bsr.Index(D, max_k=(K - 1) if failing else 64, device=0)
    ix.load(bsr.synth_uniform_np(iv.start_index, n_local, D, SEED), iv.start_index)
    q = queries()
    if a.case == "shape" and a.rank == a.world - 1:
        q = q[:-1]
    status, msg, res, warned = 0, "", None, []
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
    if a.rank == 0 or res is None:
        out["is_none"] = np.int32(res is None)
    np.savez(f"{a.out}.rank{a.rank}.npz", **out)
    print(f"rank {a.rank}: status {status} graph_replay {st.graph_replay} emitted {st.n_emitted}", flush=True)
    comm.close()
    ix.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
