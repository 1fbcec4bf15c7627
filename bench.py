"""Benchmark: batched exact cosine top-k search (better-search-rag-rust's search hot path).

Workload (BASELINE.json configs[1] per GPU): every rank holds a 1M-row shard of a synthetic
768-d U(-1,1) f32 corpus (the shard is interval_by_rank(rank, N, N*1M) of one global corpus
generated on the device), 1000 queries (query 0 = corpus row 0, the reference's self-query),
top-10.  One step = parallel_top_k_similarity_search for the whole query batch: local search
on every GPU (int8 MFMA candidate filter + exact f32 rescore), RCCL all-gather of the partial lists,
host merge on rank 0.  Weak scaling: the corpus grows with N (1M rows per GPU); `value`
counts each query once per 1M-row shard, so at N=1 it is plain queries/s over 1M vectors.

Usage: python bench.py [--gpus N --steps K --warmup W]   (N>1 via torch.distributed.run)
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PEAK_BF16_DENSE = 2.5e15   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_I8_DENSE = 5.0e15     # MI355X dense int8 MFMA: 2x the bf16 rate per clock (same guide)
PEAK_HBM = 8.0e12          # MI355X HBM3E (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--rows-per-gpu", type=int, default=1_000_000)
    ap.add_argument("--queries", type=int, default=1000)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--p50-iters", type=int, default=20)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed searches before the warmup steps (setup): the GPU leaves its idle "
                         "clocks only after some ms of load, longer than a few warmup steps take")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--verify", type=int, default=4, help="queries checked against the oracle (rank 0, N=1)")
    ap.add_argument("--filter", choices=["i8", "bf16"], default="i8",
                    help="MFMA candidate-filter operand type (results are exact either way)")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--config", choices=["c2", "c4", "c5"], default="c2",
                    help="BASELINE.json configs: c2 = 1M f32 rows/GPU, 1000 queries, top-10 (the "
                         "headline line); c4 = 10M rows, single queries, top-10 (p50 path); c5 = the "
                         "per-GPU shard of 50M bf16 rows over 8 GPUs (6.25M), 4096 queries, top-100")
    a = ap.parse_args()
    if a.config == "c4":
        a.rows_per_gpu, a.queries, a.k = 10_000_000, 1, 10
        a.p50_iters = max(a.p50_iters, 100)
    elif a.config == "c5":
        a.rows_per_gpu, a.queries, a.k = 6_250_000, 4096, 100
    return a


def main():
    args = parse()
    import torch
    import bsr

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE", file=sys.stderr)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)  # bootstrap + timing only
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)

    def barrier():
        torch.cuda.synchronize()
        if dist:
            dist.barrier()

    D, Q, K = args.dim, args.queries, args.k
    n_total = args.rows_per_gpu * world
    iv = bsr.interval_by_rank(rank, world, n_total)
    start, n_local = iv.start_index, iv.get_count()

    # Corpus shard, generated on this GPU (never crosses PCIe), loaded into the index
    # (config 5: rounded to a bf16 corpus first; parity is on the widened bf16 values).
    fflag = bsr.BSR_FLAG_FILTER_BF16 if args.filter == "bf16" else 0
    corpus_bf16 = args.config == "c5"
    index = bsr.Index(D, max_k=max(K, 64), device=local_rank, flags=bsr.BSR_FLAG_PROFILE | fflag,
                      dtype=bsr.BSR_BF16 if corpus_bf16 else bsr.BSR_F32)
    shard = torch.empty((max(n_local, 1), D), dtype=torch.float32, device=dev)
    if n_local:
        bsr.synth_uniform(shard.data_ptr(), start, n_local, D, 42)
    if corpus_bf16:
        shard = shard.to(torch.bfloat16)
    torch.cuda.synchronize()
    index.load(shard[:n_local] if n_local else np.zeros((0, D), np.float32), start)
    del shard
    torch.cuda.empty_cache()

    # Queries: row 0 of the global corpus (self-query) + seed-43 rows; resident in HBM.
    qdev = torch.empty((Q, D), dtype=torch.float32, device=dev)
    bsr.synth_uniform(qdev.data_ptr(), 0, Q, D, 43)
    bsr.synth_uniform(qdev[0:1].data_ptr(), 0, 1, D, 42)
    torch.cuda.synchronize()

    comm = None
    if world > 1:
        uid = [bsr.Comm.unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = bsr.Comm(uid[0], rank, world, local_rank)

    lib = bsr.lib()
    oi = np.empty((Q, K), np.uint64)
    od = np.empty((Q, K), np.float32)
    oc = np.empty(Q, np.uint32)
    comm_h = comm._h if comm else None

    def step(nq=Q, qptr=None):
        st = lib.bsr_parallel_top_k_similarity_search(comm_h, index._h, qptr or qdev.data_ptr(), nq, K,
                                                       oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
        if st != 0:
            raise bsr.BsrError(st, lib.bsr_last_error().decode())

    # Clock settle: the same number of untimed searches on every rank (each search is a
    # collective for N > 1), sized on rank 0 from one search's time.
    step()
    t1 = time.perf_counter()
    step()
    n_settle = int(args.settle_ms * 1e-3 / max(time.perf_counter() - t1, 1e-5)) if args.settle_ms > 0 else 0
    if dist:
        nt = torch.tensor([n_settle], dtype=torch.int64)
        dist.broadcast(nt, src=0)
        n_settle = int(nt.item())
    for _ in range(n_settle):
        step()
    for _ in range(args.warmup):
        step()
    barrier()
    # Timed region: HIP events on the filter kernels only (the roofline's launch durations);
    # the per-stage breakdown comes from a separate profiled pass below.
    index.set_profile(1)
    index.profile(reset=True)
    stats_fb = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        stats_fb += index.last_stats().n_fallback
    barrier()
    elapsed = time.perf_counter() - t0
    prof = index.profile(reset=True)
    index.set_profile(2)
    n_stage = max(3, min(args.steps, 10))
    for _ in range(n_stage):
        step()
    prof_st = index.profile(reset=True)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    st = index.last_stats()

    # Self-query check of the reference's driver (src/main.rs:141-154): row 0 ranks first.
    self_ok = None
    if rank == 0:
        self_ok = bool(oi[0, 0] == 0 and od[0, 0] == 0.0)

    # p50 single-query latency (config 4 style path: exact HBM-bound scan), all ranks.
    # Latency without event recording; the kernel breakdown from a separate profiled pass.
    lat = []
    index.set_profile(0)
    for _ in range(args.p50_iters):
        barrier()
        t1 = time.perf_counter()
        step(1, qdev[1:2].data_ptr())
        lat.append((time.perf_counter() - t1) * 1e3)
    p50 = statistics.median(lat) if lat else None
    index.set_profile(2)
    index.profile(reset=True)
    for _ in range(max(3, min(args.p50_iters, 10))):
        step(1, qdev[1:2].data_ptr())
    prof_scan = index.profile(reset=True)

    out = None
    if rank == 0:
        launches = max(prof.gemm_emit_launches, 1)
        emit_ms = prof.gemm_emit_ms / launches
        flops = 2.0 * Q * n_local * D
        achieved = flops / (emit_ms * 1e-3) / 1e12 if emit_ms > 0 else None
        traffic = None
        peak = PEAK_I8_DENSE if args.filter == "i8" else PEAK_BF16_DENSE
        nk = (D + 63) // 64
        if args.filter == "i8":
            kname = f"k_filter_qs8<true, {nk}>" if nk % 2 == 0 and nk <= 12 else "k_filter<OpI8, true>"
        else:
            kname = "k_filter<OpBF16, true>"
        if os.path.exists(args.pmc_json):
            try:
                pm = json.load(open(args.pmc_json))
                if pm.get("rows") == n_local and pm.get("queries") == Q and pm.get("filter") == args.filter:
                    traffic = pm.get("hbm_bytes_per_launch")
            except Exception:
                traffic = None
        value = (Q * world if args.config == "c2" else Q) / (ms_per_step * 1e-3)
        # Batches of <= 16 queries on an int8 index run the skinny filter (csrc/index.cpp,
        # kSkinnyMaxQ): HBM-bound, its roofline is the int8 rows streamed once per launch.
        skinny = args.filter == "i8" and Q <= 16
        if skinny:
            kv = next((c for c in (4, 8, 12, 16) if nk <= c), None)
            kname = f"k_filter_skinny2<true, {kv}>" if kv else "k_filter_skinny<true>"
            sbytes = n_local * nk * 64
            sgbs = sbytes / (emit_ms * 1e-3) / 1e9 if emit_ms > 0 else None
            roof = {"bound": "hbm", "kernel": kname, "achieved": round(sgbs, 1) if sgbs else None,
                    "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": round(sgbs * 1e9 / PEAK_HBM, 4) if sgbs else None,
                    "traffic": traffic, "algorithmic_bytes_per_launch": sbytes, "avg_launch_ms": round(emit_ms, 5)}
        else:
            roof = {
                "bound": "mfma", "kernel": kname,
                "achieved": round(achieved, 2) if achieved else None,
                "peak": peak / 1e12, "unit": "TOP/s" if args.filter == "i8" else "TFLOP/s",
                "frac": round(achieved * 1e12 / peak, 4) if achieved else None,
                "frac_of_bf16_peak": round(achieved * 1e12 / PEAK_BF16_DENSE, 4) if achieved else None,
                "traffic": traffic,
                "algorithmic_flops_per_launch": flops,
                "avg_launch_ms": round(emit_ms, 5),
            }
        out = {
            "metric": "queries/sec + p50 latency, 768-d top-10 over N vectors @1/2/4/8 GPU",
            "value": round(value, 2),
            "unit": "queries/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.filter,
            "data": f"synthetic U(-1,1) {'bf16' if corpus_bf16 else 'f32'} corpus generated on device (seed 42), "
                    f"{Q} queries (seed 43, query 0 = row 0)",
            "config": {
                "workload": {"c2": "configs[1] per GPU", "c4": "configs[3] (single-query path)",
                             "c5": "configs[4] per-GPU shard"}[args.config] +
                            f": {n_local} x {D} {'bf16' if corpus_bf16 else 'f32'} rows per GPU ({n_total} total), "
                            f"{Q} batched queries, top-{K}" +
                            ("; value = queries x 1M-row shards / s" if args.config == "c2" else "; value = queries / s"),
                "rows_total": n_total, "rows_per_gpu": n_local, "queries": Q, "top_k": K, "dim": D,
                "parallelism": f"corpus sharded over {world} GPU(s) (interval_by_rank) + RCCL all-gather",
                "filter": ("int8 MFMA (v_mfma_i32_32x32x32_i8) candidates" if args.filter == "i8" else
                           "bf16 MFMA (v_mfma_f32_32x32x16_bf16) candidates") +
                          f", exact sequential-f32 rescore of k'={st.n_candidates} per query, certified (DESIGN.md §4)",
                "qps_over_full_corpus": round(Q / (ms_per_step * 1e-3), 2),
            },
            "p50_ms": round(p50, 4) if p50 is not None else None,
            "p50_config": f"1 query over {n_total} rows" + (
                " (int8 skinny filter, HBM-bound, + exact rescore)" if args.filter == "i8" else " (exact f32 scan, HBM-bound)"),
            "roofline": roof,
            "kernels_ms_per_step": {  # separate profiled pass of n_stage steps (every stage evented)
                "gemm_emit": round(prof_st.gemm_emit_ms / n_stage, 4),
                "gemm_sample": round(prof_st.gemm_sample_ms / n_stage, 4),
                "select": round(prof_st.select_ms / n_stage, 4),
                "rescore": round(prof_st.rescore_ms / n_stage, 4),
                "scan_fallback": round(prof_st.scan_ms / n_stage, 4),
                "local_search_total": round(prof_st.search_ms / n_stage, 4),
            },
            "p50_kernels_ms": {
                "filter_emit": round(prof_scan.gemm_emit_ms / max(prof_scan.gemm_emit_launches, 1), 4),
                "filter_sample": round(prof_scan.gemm_sample_ms / max(prof_scan.gemm_sample_launches, 1), 4),
                "exact_scan": round(prof_scan.scan_ms / max(prof_scan.scan_launches, 1), 4),
                "local_search_total": round(prof_scan.search_ms / max(prof_scan.searches, 1), 4)},
            "fallback_queries_per_step": stats_fb / args.steps,
            "candidates_per_query": st.n_candidates,
            "self_query_rank1": self_ok,
            "emitted_per_query": round(st.n_emitted / max(Q, 1), 1),
            "row_ebound": round(float(st.row_ebound), 6),
        }
        # HBM roofline of the single-query (p50) kernel: the int8 skinny filter reads the
        # int8 rows (N*ld bytes per query batch); the bf16 index uses the exact f32 scan
        # (N*ld*4 bytes).
        if args.filter == "i8":
            kms = prof_scan.gemm_emit_ms / max(prof_scan.gemm_emit_launches, 1)
            nk = (D + 63) // 64
            kv = next((c for c in (4, 8, 12, 16) if nk <= c), None)
            kbytes, kn = n_local * nk * 64, (f"k_filter_skinny2<true, {kv}>" if kv else "k_filter_skinny<true>")
        else:
            kms = prof_scan.scan_ms / max(prof_scan.scan_launches, 1)
            kbytes, kn = n_local * ((D + 63) // 64 * 64) * 4, "k_scan_exact<1,1>"
        if kms > 0:
            gbs = kbytes / (kms * 1e-3) / 1e9
            out["roofline_p50"] = {"bound": "hbm", "kernel": kn, "achieved": round(gbs, 1),
                                   "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": round(gbs * 1e9 / PEAK_HBM, 4),
                                   "bytes_per_launch": kbytes, "avg_launch_ms": round(kms, 4)}

    # Parity spot-check + CPU baseline (rank 0, N=1 only): the oracle on the same corpus.
    if rank == 0 and world == 1 and (args.verify or not args.no_cpu_baseline):
        import oracle
        rows_h = index.get_many()
        q_h = qdev.cpu().numpy()
        if args.verify:
            nv = min(args.verify, Q)
            step()  # refresh oi/od for the full batch
            wi, wd, wc = oracle.parallel_top_k(rows_h, q_h[:nv], K, size=min(16, os.cpu_count() or 1),
                                               threads=min(16, os.cpu_count() or 1))
            out["parity_spot_check"] = {
                "queries": nv,
                "indices_equal": bool(np.array_equal(oi[:nv], wi)),
                "distance_bits_equal": bool(np.array_equal(od[:nv].view(np.uint32), wd.view(np.uint32))),
            }
        if not args.no_cpu_baseline:
            threads = max(1, min(16, os.cpu_count() or 1))
            t1 = time.perf_counter()
            oracle.parallel_top_k(rows_h, q_h[1:2], K, size=threads, threads=threads)
            one = time.perf_counter() - t1
            nq_cpu = max(1, min(Q, int(args.cpu_seconds / max(one, 1e-3))))
            t1 = time.perf_counter()
            oracle.parallel_top_k(rows_h, q_h[:nq_cpu], K, size=threads, threads=threads)
            cpu_t = time.perf_counter() - t1
            out["cpu_baseline"] = {
                "value": round(nq_cpu / cpu_t, 4), "unit": "queries/s", "cores": threads, "kind": "port",
                "sample": f"{nq_cpu} of the {Q} queries over the same {n_local}-row corpus, "
                          f"{threads} rank threads (mpiexec analogue), oracle/bsr_oracle.c",
            }
        else:
            out["cpu_baseline"] = None
    if rank == 0:
        print(json.dumps(out), flush=True)
    barrier()
    if comm:
        comm.close()
    index.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
