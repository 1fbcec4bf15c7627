"""Benchmark: batched exact cosine top-k search (better-search-rag-rust's search hot path).

Default workload (BASELINE.json configs[2], strong scaling): one synthetic corpus of 10M
768-d U(-1,1) f32 rows (seed 42, generated on the devices), sharded over the N GPUs with the
reference's interval_by_rank; 1000 queries (query 0 = corpus row 0, the reference's
self-query), top-10.  One step = parallel_top_k_similarity_search for the whole batch:
the local search on every GPU (int8 MFMA candidate filter + exact f32 rescore of the
candidates, certified), the RCCL all-gather of the partial lists and the root's merge.
`value` = queries/s over the whole 10M corpus (the same total work at every N).  At N = 1
this is the north-star shape (batched 10M); the same run also reports configs[1] (the first
1M rows, 1000 queries) and the single-query p50 over the full corpus (configs[3]).

Usage: python bench.py [--gpus N --steps K --warmup W]
  N > 1: launched by torch.distributed.run (one rank per GPU), or, without WORLD_SIZE in
  the environment, bench.py starts the N rank processes itself (before any GPU call).
  --comm host: the exchange over gloo instead of RCCL (ranks may then share a GPU: a
  multi-rank rehearsal on a one-GPU box).
  --comm loopback --gpus N: ONE process timing rank 0's step of an N-rank run on one GPU, every
  all-gather emulated by a device kernel where ncclAllGather sits (bsr_comm_init_loopback), its
  contributions replayed from a recording of a real N-rank run of the same batch (made first,
  over the host transport with N rank processes on the one GPU; --replay FILE reuses one).  Not a
  scaling measurement: the collectives' own latency is not in it.
"""
import argparse
import json
import os
import socket
import statistics
import subprocess
import sys
import tempfile
import threading
import time
from datetime import timedelta

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "better-search-rag-rust_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

PEAK_BF16_DENSE = 2.5e15   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, spec)
PEAK_I8_DENSE = 5.0e15     # MI355X dense int8 MFMA: 2x the bf16 rate per clock (same guide)
PEAK_HBM = 8.0e12          # MI355X HBM3E (spec)
CPU_SHARE = 16             # host cores of one GPU's share on the box (nproc shows the machine)

CONFIGS = {
    # name: (rows in the corpus, queries, top-k, corpus dtype, sharding, label)
    "c1": (20_000, 32, 10, "f32", "strong",
           "configs[0]: JabRef stand-in, 20k x 768 f32 rows in the reference's parquet store "
           "(global.parquet), 32 queries, top-10, 1 GPU; parquet decode timed separately"),
    "c3": (10_000_000, 1000, 10, "f32", "strong",
           "configs[2]: 10M x 768 f32 corpus sharded over the N GPUs, 1000 batched queries, top-10"),
    "c2": (1_000_000, 1000, 10, "f32", "strong",
           "configs[1]: 1M x 768 f32 corpus (sharded over the N GPUs), 1000 batched queries, top-10"),
    "c4": (10_000_000, 1, 10, "f32", "strong",
           "configs[3]: 10M x 768 f32 corpus, single queries (p50 path), top-10"),
    "c5": (6_250_000, 4096, 100, "bf16", "weak",
           "configs[4] per-GPU shard: 6.25M x 768 bf16 rows per GPU (50M over 8), 4096 queries, top-100"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", choices=sorted(CONFIGS), default="c3")
    ap.add_argument("--rows", type=int, default=None, help="override the corpus rows (tests)")
    ap.add_argument("--queries", type=int, default=None)
    ap.add_argument("--k", type=int, default=None)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--comm", choices=["rccl", "host", "loopback"], default="rccl")
    ap.add_argument("--replay", default=None, help="--comm loopback: a recording made by --record-gathers")
    ap.add_argument("--record-gathers", default=None,
                    help="--comm host, rank 0: record the first search's all-gathers to this .npz")
    ap.add_argument("--record-only", action="store_true", help="with --record-gathers: stop after recording")
    ap.add_argument("--p50-iters", type=int, default=100)
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="untimed searches before the warmup steps (setup): the GPU leaves its idle "
                         "clocks only after some ms of load, longer than a few warmup steps take")
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="per point of the CPU-baseline sweep")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-configs1", action="store_true", help="skip the configs[1] side measurement (N=1)")
    ap.add_argument("--verify", type=int, default=4, help="queries checked against the oracle on rank 0")
    ap.add_argument("--pmc-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--rank-timeout", type=float, default=1500.0,
                    help="N > 1 without torchrun: the whole run's deadline for the rank processes")
    ap.add_argument("--collective-timeout", type=float, default=300.0,
                    help="N > 1: deadline of each collective phase (setup, the step loops, barriers); a "
                         "rank past it exits non-zero instead of blocking in a collective")
    a = ap.parse_args()
    rows, q, k, dt, sc, label = CONFIGS[a.config]
    a.rows_total = a.rows if a.rows is not None else rows
    a.queries = a.queries if a.queries is not None else q
    a.k = a.k if a.k is not None else k
    a.corpus_dtype, a.scaling, a.label = dt, sc, label
    a.filter = "i8"  # the MFMA candidate filter's operand (the bf16 operand is retired)
    if a.config == "c4":
        a.p50_iters = max(a.p50_iters, 100)
    return a


def _error_line(args, msg, **extra):
    """The run's one JSON line when it fails: the metric named, no value."""
    out = {"metric": "queries/sec + p50 latency, 768-d top-10 over N vectors @1/2/4/8 GPU", "value": None,
           "unit": "queries/s", "n_gpus": args.gpus, "error": msg}
    out.update(extra)
    print(json.dumps(out), flush=True)


def spawn_ranks(args):
    """Start the N rank processes (one per GPU; nothing here touches the GPU) and watch them.
    Fail fast (metrics.rs:185-197: no rank may be left blocked): the first rank that exits
    non-zero -- or the run's deadline -- ends every other rank (rank 0 may be blocked in a
    collective with the dead one), and one JSON error line names the rank and its stderr tail."""
    n = args.gpus
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    logdir = tempfile.mkdtemp(prefix="bsr_bench_")
    procs, errs = [], []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        ef = open(os.path.join(logdir, f"rank{r}.stderr"), "w+b")
        errs.append(ef)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stderr=ef))
    t_end = time.monotonic() + args.rank_timeout
    failed = None
    while failed is None:
        codes = [p.poll() for p in procs]
        bad = [(r, c) for r, c in enumerate(codes) if c not in (None, 0)]
        if bad:
            failed = bad[0]
        elif all(c == 0 for c in codes):
            break
        elif time.monotonic() > t_end:
            failed = (next(r for r, c in enumerate(codes) if c is None), "timeout")
        else:
            time.sleep(0.1)
    if failed is not None:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_kill = time.monotonic() + 10
        for p in procs:
            try:
                p.wait(timeout=max(0.1, t_kill - time.monotonic()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    tails = []
    for r, ef in enumerate(errs):
        ef.seek(0)
        data = ef.read().decode(errors="replace")
        ef.close()
        sys.stderr.write(data)
        tails.append(data[-1500:])
    sys.stderr.flush()
    if failed is None:
        return 0
    r, c = failed
    what = f"rank {r} exited with status {c}" if c != "timeout" else \
        f"rank {r} still running after --rank-timeout {args.rank_timeout:.0f} s"
    _error_line(args, what + "; the other ranks were terminated", failed_rank=r, stderr_tail=tails[r])
    return c if isinstance(c, int) and c > 0 else 1


class Watchdog:
    """A rank's collective deadline: a phase that has not finished within its time (a peer died
    inside a collective, a hung transport) ends the process with status 124 and a message,
    instead of blocking forever (the launcher then ends the other ranks)."""

    def __init__(self, rank):
        self.rank, self.deadline, self.label = rank, None, ""
        self.lock = threading.Lock()
        threading.Thread(target=self._run, daemon=True).start()

    def arm(self, label, seconds):
        with self.lock:
            self.label, self.deadline = label, time.monotonic() + seconds

    def disarm(self):
        with self.lock:
            self.deadline = None

    def save(self):
        with self.lock:
            return self.label, self.deadline

    def restore(self, state):
        with self.lock:
            self.label, self.deadline = state

    def _run(self):
        while True:
            time.sleep(0.5)
            with self.lock:
                late = self.deadline is not None and time.monotonic() > self.deadline
                label = self.label
            if late:
                sys.stderr.write(f"bench.py rank {self.rank}: collective phase '{label}' passed its deadline "
                                 f"(--collective-timeout); exiting\n")
                sys.stderr.flush()
                os._exit(124)


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


LAUNCH_TIMING = ("HIP events recorded on the index's stream around each filter launch, over K searches "
                 "right after the timed region (kernel_timing_pass)")


def kernel_timing_pass(index, search, n):
    """The filter kernel's launch durations for the roofline: n more searches (search() runs
    one) right after the timed region, at profile level 1 -- HIP events recorded on the index's
    stream around each filter launch (the search launched directly, not graph-replayed).
    Event-record nodes inside a replayed graph time from the graph's start, and the events
    hipExtLaunchKernel binds to a launch start at its submission, on ROCm 7.2
    (profiles/r04m_event_timing.txt)."""
    index.set_profile(1)
    index.profile(reset=True)
    for _ in range(n):
        search()
    prof = index.profile(reset=True)
    index.set_profile(0)
    return prof


def run_c1(args):
    """configs[0] (the reference's own CPU/MPI plumbing case, JabRef ~20k chunks): the corpus
    lives in the reference's vector store (one parquet file, column "embeddings" of
    List(Float32), src/vectorstore/polars.rs) and reaches the GPU through the vector-store
    adapter (bsr_index_load_vstore: decode + H2D + quantisation), timed on its own as the
    reference's report would time the parquet read inside "similarity_search"
    (src/main.rs:114-134).  Then the 32-query batch is timed (K steps) and every query is
    checked against the oracle; the CPU baseline (oracle, P = 4 rank threads as configs[0]'s
    mpiexec -n 4, all 32 queries) and the CPU-side parquet decode are reported separately."""
    import tempfile
    import torch
    import bsr
    import oracle
    D, Q, K, N = args.dim, args.queries, args.k, args.rows_total
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    corpus = torch.empty((N, D), dtype=torch.float32, device=dev)
    bsr.synth_uniform(corpus.data_ptr(), 0, N, D, 42)
    qdev = torch.empty((Q, D), dtype=torch.float32, device=dev)
    bsr.synth_uniform(qdev.data_ptr(), 0, Q, D, 43)
    bsr.synth_uniform(qdev[0:1].data_ptr(), 0, 1, D, 42)
    torch.cuda.synchronize()
    rows_h, q_h = corpus.cpu().numpy(), qdev.cpu().numpy()
    del corpus
    with tempfile.TemporaryDirectory() as vdir:
        vs = bsr.get_global_vstore(vdir, True)
        vs.append_many(rows_h)
        vs.persist()
        vs.close()
        # GPU path: open the store (parquet read) + this rank's block into HBM
        t0 = time.perf_counter()
        vs = bsr.get_global_vstore(vdir, False)
        index = bsr.Index(D, max_k=64, device=0, flags=bsr.BSR_FLAG_PROFILE)
        bsr.load_index_from_vstore(index, vs, 0, 1)
        torch.cuda.synchronize()
        load_ms = (time.perf_counter() - t0) * 1e3
        # CPU path's decode of the same file (the reference's read_parquet + Vec<Vec<f32>>)
        t0 = time.perf_counter()
        vs2 = bsr.get_global_vstore(vdir, False)
        dec = vs2.get_many_array(None, dim=D)
        cpu_decode_ms = (time.perf_counter() - t0) * 1e3
        vs2.close()
        vs.close()
    assert np.array_equal(dec, rows_h)
    lib = bsr.lib()
    oi = np.empty((Q, K), np.uint64)
    od = np.empty((Q, K), np.float32)
    oc = np.empty(Q, np.uint32)

    def step(nq=Q, qptr=None):
        st = lib.bsr_parallel_top_k_similarity_search(None, index._h, qptr or qdev.data_ptr(), nq, K,
                                                       oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
        if st != 0:
            raise bsr.BsrError(st, lib.bsr_last_error().decode())

    index.set_profile(0)  # (settle, warmup and timed steps: the product path, graph replay)
    t_end = time.perf_counter() + args.settle_ms * 1e-3
    while time.perf_counter() < t_end:
        step()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / args.steps * 1e3
    res_i, res_d, res_c = oi.copy(), od.copy(), oc.copy()
    prof = kernel_timing_pass(index, step, args.steps)
    lat = []
    for _ in range(max(args.p50_iters, 20)):
        t1 = time.perf_counter()
        step(1, qdev[1:2].data_ptr())
        lat.append((time.perf_counter() - t1) * 1e3)
    wi, wd, wc = oracle.parallel_top_k(rows_h, q_h, K, size=4, threads=4)
    ok_i = bool(np.array_equal(res_c, wc) and np.array_equal(res_i, wi))
    ok_d = bool(np.array_equal(res_d.view(np.uint32), wd.view(np.uint32)))
    t1 = time.perf_counter()
    oracle.parallel_top_k(rows_h, q_h, K, size=4, threads=4)
    cpu_s = time.perf_counter() - t1
    ems = prof.gemm_emit_ms / max(prof.gemm_emit_launches, 1)
    out = {
        "metric": "queries/sec + p50 latency, 768-d top-10 over N vectors @1/2/4/8 GPU",
        "value": round(Q / (ms * 1e-3), 2), "unit": "queries/s", "n_gpus": 1, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "f32", "filter_dtype": "i8",
        "data": "synthetic U(-1,1) f32 rows (seed 42) written to the reference's parquet store, 32 queries "
                "(seed 43, query 0 = row 0), HBM-resident",
        "config": {"workload": args.label, "rows_total": N, "queries": Q, "top_k": K, "dim": D,
                   "parallelism": "1 GPU"},
        "parquet_load_ms": round(load_ms, 3),
        "parquet_load_note": "open global.parquet + decode + H2D + row norms + int8 operand (bsr_index_load_vstore); "
                             "once per store, outside the timed searches",
        "p50_ms": round(statistics.median(lat), 4),
        "filter_avg_launch_ms": round(ems, 5),
        "parity_all_queries": {"queries": Q, "indices_equal": ok_i, "distance_bits_equal": ok_d,
                               "method": "oracle/bsr_oracle.c, P = 4 rank blocks merged"},
        "roofline": None,
        "cpu_baseline": {"value": round(Q / cpu_s, 3), "unit": "queries/s", "cores": 4, "kind": "port",
                         "sample": f"all {Q} queries over the {N} rows, oracle with P = 4 rank threads "
                                   "(configs[0]'s mpiexec -n 4); parquet decode excluded, reported as decode_ms",
                         "decode_ms": round(cpu_decode_ms, 3), "nproc": os.cpu_count(), "cpu_model": cpu_model()},
    }
    print(json.dumps(out), flush=True)
    index.close()
    return 0 if (ok_i and ok_d) else 1


def record_for_loopback(args):
    """--comm loopback without --replay: record a real N-rank run's all-gathers first (N rank
    processes over the host transport on this GPU; nothing here touches the GPU)."""
    path = os.path.join(tempfile.mkdtemp(prefix="bsr_loopback_"), "gathers.npz")
    cmd = [sys.executable, os.path.abspath(__file__), "--comm", "host", "--gpus", str(args.gpus), "--config",
           args.config, "--record-gathers", path, "--record-only", "--dim", str(args.dim), "--queries",
           str(args.queries), "--k", str(args.k), "--settle-ms", "0", "--warmup", "0", "--steps", "1"]
    if args.rows is not None:
        cmd += ["--rows", str(args.rows)]
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE)
    if r.returncode != 0 or not os.path.exists(path):
        _error_line(args, f"recording the {args.gpus}-rank all-gathers failed (rc {r.returncode})")
        sys.exit(r.returncode or 1)
    return path


def skinny_kernel(nk):
    """The skinny filter's row-mode kernel for rows of nk 64-byte K slices (csrc/k_filter.hip
    launch_skinny: 768-byte rows take the LDS-DMA kernel unless BSR_SKINNY_GLDS=0)."""
    return "k_filter_skinny_glds" if nk == 12 and os.environ.get("BSR_SKINNY_GLDS", "1")[:1] != "0" else "k_filter_skinny2"


def main():
    args = parse()
    if args.config == "c1":
        sys.exit(run_c1(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    loop = args.comm == "loopback"
    if loop and world > 1:
        _error_line(args, "--comm loopback is one process (rank 0 of --gpus N); do not launch it with torchrun")
        sys.exit(2)
    if loop and args.gpus > 1 and not args.replay:
        args.replay = record_for_loopback(args)
    if "WORLD_SIZE" not in os.environ and args.gpus > 1 and not loop:
        sys.exit(spawn_ranks(args))
    P = args.gpus if loop else world  # ranks the corpus is sharded over (loopback: emulated)
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"warning: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE", file=sys.stderr)

    # (test hook of the fail-fast path: this rank fails before its first collective)
    if os.environ.get("BSR_BENCH_FAIL_RANK") == str(rank) and world > 1:
        sys.stderr.write(f"bench.py rank {rank}: failing on purpose (BSR_BENCH_FAIL_RANK)\n")
        sys.exit(3)

    import torch
    import bsr

    watchdog = Watchdog(rank) if world > 1 else None
    dist = None
    if world > 1:
        watchdog.arm("process group init", args.collective_timeout)
        import torch.distributed as dist
        # (gloo prints its connection report to stdout: keep stdout for the one JSON line)
        sys.stdout.flush()
        saved_fd = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)  # bootstrap, timing, host transport
        finally:
            os.dup2(saved_fd, 1)
            os.close(saved_fd)
        watchdog.disarm()
    ndev = torch.cuda.device_count()
    device = local_rank % max(ndev, 1)
    torch.cuda.set_device(device)
    dev = torch.device("cuda", device)

    def barrier(timeout=None):
        """Every rank here, or a named failure: gloo's monitored barrier reports the rank that
        did not arrive (the bootstrap group is gloo), under the collective deadline."""
        torch.cuda.synchronize()
        if dist:
            t = timeout or args.collective_timeout
            prev = watchdog.save()
            watchdog.arm("barrier", t + 30)
            dist.monitored_barrier(timeout=timedelta(seconds=t))
            watchdog.restore(prev)

    def armed(label):
        if watchdog:
            watchdog.arm(label, args.collective_timeout)

    D, Q, K = args.dim, args.queries, args.k
    n_total = args.rows_total * (P if args.scaling == "weak" else 1)
    iv = bsr.interval_by_rank(rank, P, n_total)
    start, n_local = iv.start_index, iv.get_count()

    # Corpus shard, generated on this GPU (never crosses PCIe), loaded into the index
    # (config 5: rounded to a bf16 corpus first; parity is on the widened bf16 values).
    fflag = 0
    corpus_bf16 = args.corpus_dtype == "bf16"
    index = bsr.Index(D, max_k=max(K, 64), device=device, flags=bsr.BSR_FLAG_PROFILE | fflag,
                      dtype=bsr.BSR_BF16 if corpus_bf16 else bsr.BSR_F32)
    shard = torch.empty((max(n_local, 1), D), dtype=torch.float32, device=dev)
    if n_local:
        bsr.synth_uniform(shard.data_ptr(), start, n_local, D, 42)
    if corpus_bf16:
        shard = shard.to(torch.bfloat16)
    torch.cuda.synchronize()
    index.load(shard[:n_local] if n_local else np.zeros((0, D), np.float32), start)
    # configs[1] side measurement (N = 1, default config): the first 1M rows of the corpus
    ix1 = None
    if world == 1 and args.config == "c3" and not args.no_configs1 and n_local >= 1_000_000:
        ix1 = bsr.Index(D, max_k=64, device=device, flags=bsr.BSR_FLAG_PROFILE | fflag)
        ix1.load(shard[:1_000_000], 0)
    del shard
    torch.cuda.empty_cache()

    # Queries: row 0 of the global corpus (self-query) + seed-43 rows; resident in HBM.
    qdev = torch.empty((Q, D), dtype=torch.float32, device=dev)
    bsr.synth_uniform(qdev.data_ptr(), 0, Q, D, 43)
    bsr.synth_uniform(qdev[0:1].data_ptr(), 0, 1, D, 42)
    if corpus_bf16:  # the corpus holds row 0's bf16 rounding: query 0 is that row exactly
        qdev[0:1] = qdev[0:1].to(torch.bfloat16).to(torch.float32)
    torch.cuda.synchronize()

    comm = None
    armed("communicator setup")
    lb_calls = 0
    if loop and P > 1:
        rec = np.load(args.replay)
        script = [rec[f"rec{i}"] for i in range(int(rec["n_rec"]))]
        lb_calls = len(script)
        comm = bsr.Comm.loopback(0, P, device, script)
    elif world > 1:
        if args.comm == "host":
            comm = bsr.Comm.host(dist.group.WORLD)
        else:
            uid = [bsr.Comm.unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = bsr.Comm(uid[0], rank, world, device)

    lib = bsr.lib()
    # the root's outputs in coherent pinned host memory: on the global-threshold path (N > 1) the
    # merge writes the rows there directly, as a Rust caller using bsr_host_alloc would have it
    oi = bsr.host_array((Q, K), np.uint64)
    od = bsr.host_array((Q, K), np.float32)
    oc = bsr.host_array(Q, np.uint32)
    comm_h = comm._h if comm else None

    def step(nq=Q, qptr=None, ix=index):
        st = lib.bsr_parallel_top_k_similarity_search(comm_h if ix is index else None, ix._h, qptr or qdev.data_ptr(),
                                                       nq, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
        if st != 0:
            raise bsr.BsrError(st, lib.bsr_last_error().decode())

    def bcast_int(v):
        if dist:
            t = torch.tensor([v], dtype=torch.int64)
            dist.broadcast(t, src=0)
            v = int(t.item())
        return v

    # Clock settle: the same number of untimed searches on every rank (each search is a
    # collective for N > 1), sized on rank 0 from one search's time -- at the timed region's
    # profile level, so that its searches (and their graph, warmed here) are the timed ones'.
    armed("settle + warmup steps")
    index.set_profile(0)  # (settle, warmup and timed steps: the product path, graph replay)
    if args.record_gathers and comm is not None and comm.transport == "host":
        comm.record = [] if rank == 0 else None
        step()
        n_rec = len(comm.record) if rank == 0 else 0
        if rank == 0:
            np.savez(args.record_gathers, n_rec=np.int32(n_rec), **{f"rec{i}": b for i, b in enumerate(comm.record)})
        comm.record = None
        if args.record_only:
            barrier()
            if rank == 0:
                print(json.dumps({"recorded": args.record_gathers, "calls": n_rec, "ranks": world}), flush=True)
            comm.close()
            index.close()
            dist.destroy_process_group()
            return
    step()
    t1 = time.perf_counter()
    step()
    n_settle = bcast_int(int(args.settle_ms * 1e-3 / max(time.perf_counter() - t1, 1e-5)) if args.settle_ms > 0 else 0)
    for _ in range(n_settle):
        step()
    for _ in range(args.warmup):
        step()
    barrier()
    # Timed region: exactly K searches between barriers (the product path: graph replay, no
    # events); the filter's launch durations come from the pass right after it.
    stats_fb = stats_rescued = 0
    barrier()
    armed("timed steps")
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
        ls = index.last_stats()
        stats_fb += ls.n_fallback
        stats_rescued += ls.n_rescued
    barrier()
    elapsed = time.perf_counter() - t0
    armed("kernel-timing, stage-profile, local-search and p50 passes")
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms_per_step = elapsed / args.steps * 1e3
    st = index.last_stats()
    res_i, res_d, res_c = oi.copy(), od.copy(), oc.copy()  # the last timed step's result (root)
    prof = kernel_timing_pass(index, step, args.steps)  # (every rank: each search is a collective)
    # per-stage breakdown from a separate profiled pass (every stage evented)
    index.set_profile(2)
    n_stage = max(3, min(args.steps, 10))
    for _ in range(n_stage):
        step()
    prof_st = index.profile(reset=True)

    # The same steps without the exchange (each rank's local search alone, bsr_local_top_k):
    # the step time's split into local search and exchange + root merge (N > 1).
    index.set_profile(0)
    for _ in range(2):
        lib.bsr_local_top_k(index._h, qdev.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        st_l = lib.bsr_local_top_k(index._h, qdev.data_ptr(), Q, K, oi.ctypes.data, od.ctypes.data, oc.ctypes.data)
        if st_l != 0:
            raise bsr.BsrError(st_l, lib.bsr_last_error().decode())
    local_s = time.perf_counter() - t0
    if dist:
        t = torch.tensor([local_s], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        local_s = float(t.item())
    local_ms = local_s / args.steps * 1e3

    # p50 single-query latency over the whole corpus (configs[3] path), all ranks.  Settled as the
    # batched steps are (--settle-ms of untimed single-query searches at the profile level of the
    # timed ones): right after the batched passes the chip still holds the clocks of int8 MFMA load,
    # and the HBM-bound skinny filter ran ~4% slower there than in a single-query run
    # (profiles/r06f_bench.json p50_kernels_ms_rank0 vs r06f_p50_top_ab.txt).
    lat = []
    index.set_profile(0)
    # (a count agreed by every rank: each search is a collective for N > 1)
    step(1, qdev[1:2].data_ptr())
    t1 = time.perf_counter()
    step(1, qdev[1:2].data_ptr())
    n_p50_settle = bcast_int(int(args.settle_ms * 1e-3 / max(time.perf_counter() - t1, 1e-5))
                             if args.settle_ms > 0 else 0)
    for _ in range(n_p50_settle):
        step(1, qdev[1:2].data_ptr())
    barrier()
    for _ in range(args.p50_iters):
        barrier()
        t1 = time.perf_counter()
        step(1, qdev[1:2].data_ptr())
        lat.append((time.perf_counter() - t1) * 1e3)
    p50 = statistics.median(lat) if lat else None
    p50_path = index.last_stats().search_path  # (BSR_PATH_SKINNY_TOP: the self-thresholded filter)
    index.set_profile(2)
    index.profile(reset=True)
    for _ in range(max(3, min(args.p50_iters, 10))):
        step(1, qdev[1:2].data_ptr())
    prof_scan = index.profile(reset=True)

    # configs[1] side measurement (N = 1): 1M rows, the same 1000 queries
    c1 = None
    if ix1 is not None:
        ix1.set_profile(0)
        for _ in range(max(args.warmup, 3) + 20):
            step(ix=ix1)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            step(ix=ix1)
        torch.cuda.synchronize()
        c1_ms = (time.perf_counter() - t1) / args.steps * 1e3
        p1 = kernel_timing_pass(ix1, lambda: step(ix=ix1), args.steps)
        e1 = p1.gemm_emit_ms / max(p1.gemm_emit_launches, 1)
        a1 = 2.0 * Q * 1_000_000 * D / (e1 * 1e-3) if e1 > 0 else None
        c1 = {"workload": "configs[1]: first 1M rows of the corpus, the same 1000 queries, top-10, 1 GPU",
              "value": round(Q / (c1_ms * 1e-3), 2), "unit": "queries/s", "ms_per_step": round(c1_ms, 4),
              "filter_avg_launch_ms": round(e1, 5),
              "filter_frac_of_i8_peak": round(a1 / PEAK_I8_DENSE, 4) if a1 and args.filter == "i8" else None}
        step()  # leave oi/od as the main index's
        ix1.close()
        ix1 = None

    out = None
    nk = (D + 63) // 64
    if rank == 0:
        launches = max(prof.gemm_emit_launches, 1)
        emit_ms = prof.gemm_emit_ms / launches
        # roofline.traffic: HBM bytes per launch from the committed PMC passes (not read in
        # this run: rocprofv3 --pmc runs are separate, MI355X_MICROARCH.md); the source is named
        traffic, traffic_src = None, None
        if os.path.exists(args.pmc_json):
            try:
                pm = json.load(open(args.pmc_json))
                for e in pm.get("entries", [pm]):
                    if e.get("rows") == n_local and e.get("queries") == Q and e.get("filter") == args.filter:
                        traffic = e.get("hbm_bytes_per_launch")
                        traffic_src = (f"from {os.path.relpath(args.pmc_json, ROOT)} (run {e.get('run') or pm.get('run', '?')}, "
                                       "FETCH_SIZE x 2 + WRITE_SIZE, separate rocprofv3 --pmc passes)")
            except (OSError, ValueError):
                traffic = None
        if args.filter == "i8" and Q <= 16:
            # <= 16 queries on an int8 index: the skinny filter (HBM-bound)
            kv = next((c for c in (4, 8, 12, 16) if nk <= c), None)
            kname = (f"{skinny_kernel(nk)}<{2 if st.search_path & bsr.BSR_PATH_SKINNY_TOP else 1}, {kv}>" if kv
                     else "k_filter_skinny<true>")
            sbytes = n_local * nk * 64
            gbs = sbytes / (emit_ms * 1e-3) / 1e9 if emit_ms > 0 else None
            roof = {"bound": "hbm", "kernel": kname, "achieved": round(gbs, 1) if gbs else None,
                    "peak": PEAK_HBM / 1e9, "unit": "GB/s", "frac": round(gbs * 1e9 / PEAK_HBM, 4) if gbs else None,
                    "traffic": traffic, "traffic_source": traffic_src, "algorithmic_bytes_per_launch": sbytes,
                    "avg_launch_ms": round(emit_ms, 5), "launch_timing": LAUNCH_TIMING}
        else:
            flops = 2.0 * Q * n_local * D
            achieved = flops / (emit_ms * 1e-3) / 1e12 if emit_ms > 0 else None
            peak = PEAK_I8_DENSE if args.filter == "i8" else PEAK_BF16_DENSE
            if args.filter == "i8":
                kname = f"k_filter_qs16<true, {nk}>" if nk % 2 == 0 and nk <= 12 else "k_filter<OpI8, true>"
            else:
                kname = "k_filter<OpBF16, true>"
            roof = {"bound": "mfma", "kernel": kname, "achieved": round(achieved, 2) if achieved else None,
                    "peak": peak / 1e12, "unit": "TOP/s" if args.filter == "i8" else "TFLOP/s",
                    "frac": round(achieved * 1e12 / peak, 4) if achieved else None, "traffic": traffic,
                    "traffic_source": traffic_src,
                    "algorithmic_ops_per_launch": flops, "avg_launch_ms": round(emit_ms, 5),
                    "launch_timing": LAUNCH_TIMING,
                    "note": "rank 0's shard; ops = 2 * queries * shard rows * dim (int8 multiply-adds)"}
        out = {
            "metric": "queries/sec + p50 latency, 768-d top-10 over N vectors @1/2/4/8 GPU",
            "value": round(Q / (ms_per_step * 1e-3), 2),
            "unit": "queries/s",
            "n_gpus": world,
            "loopback": None if not loop else {
                "ranks": P, "replayed_allgathers": comm.loopback_stats()[0] if comm else 0,
                "missed_allgathers": comm.loopback_stats()[1] if comm else 0, "recorded_calls_per_search": lb_calls,
                "note": (f"ONE process on one GPU timing rank 0's step of a {P}-rank run: its shard "
                         f"({n_local} rows), every all-gather one device kernel where ncclAllGather sits "
                         "(no host wait), the other ranks' contributions replayed from a real "
                         f"{P}-rank run of this batch (host transport). value = queries / this step: a "
                         "per-rank step projection without the collectives' latency, not a scaling "
                         "measurement")},
            "steps": args.steps,
            "warmup": args.warmup,
            "settle_ms": args.settle_ms,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "filter_dtype": args.filter,
            "data": f"synthetic U(-1,1) {'bf16' if corpus_bf16 else 'f32'} corpus generated on device (seed 42), "
                    f"{Q} queries (seed 43, query 0 = row 0), HBM-resident",
            "config": {
                "workload": args.label + ("" if args.rows is None else f" (rows overridden: {n_total})"),
                "rows_total": n_total, "rows_per_gpu_rank0": n_local, "queries": Q, "top_k": K, "dim": D,
                "parallelism": (f"corpus sharded over {world} GPU(s) (interval_by_rank)" +
                                ("" if world == 1 else f" + {args.comm.upper()} all-gather of the partial lists"
                                                       " + root merge")) if not loop else
                               f"rank 0 of {P} (interval_by_rank), loopback communicator: emulated all-gathers",
                "filter": "int8 MFMA (v_mfma_i32_16x16x64_i8) candidates, " + (
                    f"exact sequential-f32 rescore of k'={st.n_candidates} per query, certified (DESIGN.md §4)"
                    if st.n_candidates else
                    "emission threshold selected from every rank's sample (all-gathered), exact sequential-f32 "
                    "rescore of every emitted row, the merged lists certified on every rank (DESIGN.md §6)"),
            },
            "p50_ms": round(p50, 4) if p50 is not None else None,
            "p50_config": f"1 query over {n_total} rows on {world} GPU(s)" + (
                (" (int8 skinny filter keeping each workgroup's 4 best rows, HBM-bound, + exact rescore)"
                 if p50_path & bsr.BSR_PATH_SKINNY_TOP else " (int8 skinny filter, HBM-bound, + exact rescore)")
                if args.filter == "i8" else
                " (exact f32 scan, HBM-bound)"),
            "roofline": roof,
            "local_search_ms_per_step": round(local_ms, 4),
            "exchange_ms_per_step": round(ms_per_step - local_ms, 4) if world > 1 else None,
            "step_split_note": None if world == 1 else (
                "local_search_ms_per_step = the same K searches through bsr_local_top_k (each rank's standard "
                "local search with its own threshold, no exchange)" + (
                    "; the timed steps ran the global-threshold search, whose local work is smaller (fewer rows "
                    "emitted per rank), so exchange_ms_per_step understates the all-gathers + merge"
                    if not st.n_candidates else "")),
            "kernels_ms_per_step_rank0": {  # separate profiled pass of n_stage steps (every stage evented)
                "note": "a separate profiled pass after the timed region (direct launches, HIP events around "
                        "every stage, a D2H copy and stream wait per search): NOT the timed path, whose "
                        "ms_per_step replays a captured graph without events; local_search_total can exceed "
                        "ms_per_step",
                "filter_emit": round(prof_st.gemm_emit_ms / n_stage, 4),
                "filter_sample": round(prof_st.gemm_sample_ms / n_stage, 4),
                "select": round(prof_st.select_ms / n_stage, 4),
                "rescore": round(prof_st.rescore_ms / n_stage, 4),
                "scan_fallback": round(prof_st.scan_ms / n_stage, 4),
                "local_search_total": round(prof_st.search_ms / n_stage, 4)},
            "p50_kernels_ms_rank0": {
                "filter_emit": round(prof_scan.gemm_emit_ms / max(prof_scan.gemm_emit_launches, 1), 4),
                "filter_sample": round(prof_scan.gemm_sample_ms / max(prof_scan.gemm_sample_launches, 1), 4),
                "exact_scan": round(prof_scan.scan_ms / max(prof_scan.scan_launches, 1), 4),
                "local_search_total": round(prof_scan.search_ms / max(prof_scan.searches, 1), 4)},
            "fallback_queries_per_step_rank0": stats_fb / args.steps,
            "rescued_queries_per_step_rank0": stats_rescued / args.steps,
            "candidates_per_query": st.n_candidates,  # (0: global threshold, every emitted row rescored)
            "self_query_rank1": bool(res_i[0, 0] == 0 and res_d[0, 0] == 0.0),
            "emitted_per_query_rank0": round(st.n_emitted / max(Q, 1), 1),
            "row_ebound": round(float(st.row_ebound), 6),
        }
        if c1:
            out["configs1"] = c1
        kms = (prof_scan.gemm_emit_ms / max(prof_scan.gemm_emit_launches, 1) if args.filter == "i8" else
               prof_scan.scan_ms / max(prof_scan.scan_launches, 1))
        if kms > 0:
            if args.filter == "i8":
                kv = next((c for c in (4, 8, 12, 16) if nk <= c), None)
                mode = 2 if p50_path & bsr.BSR_PATH_SKINNY_TOP else 1  # (kSkTop / kSkEmit)
                kbytes, kn = n_local * nk * 64, (f"{skinny_kernel(nk)}<{mode}, {kv}>" if kv else "k_filter_skinny<true>")
            else:
                kbytes, kn = n_local * nk * 64 * 4, "k_scan_exact<1,1>"
            gbs = kbytes / (kms * 1e-3) / 1e9
            out["roofline_p50"] = {"bound": "hbm", "kernel": kn, "achieved": round(gbs, 1), "peak": PEAK_HBM / 1e9,
                                   "unit": "GB/s", "frac": round(gbs * 1e9 / PEAK_HBM, 4), "bytes_per_launch": kbytes,
                                   "avg_launch_ms": round(kms, 4)}

    # Parity spot-check on rank 0 at every N, against the oracle over the WHOLE corpus:
    # the corpus is regenerated 1M rows at a time on rank 0's GPU (the same counter-based
    # generator), each block's oracle lists merged as the reference merges rank blocks.
    # Then the CPU baseline (rank 0, N = 1).  Other ranks wait at the final barrier.
    if loop:
        args.no_cpu_baseline = True
    if rank == 0 and (args.verify or (world == 1 and not args.no_cpu_baseline)):
        import oracle
        q_h = qdev.cpu().numpy()
        chunk = 1_000_000
        buf = torch.empty((min(chunk, n_total), D), dtype=torch.float32, device=dev)

        def corpus_block(r0, n):
            bsr.synth_uniform(buf.data_ptr(), r0, n, D, 42)
            torch.cuda.synchronize()
            blk = buf[:n]
            if corpus_bf16:
                blk = blk.to(torch.bfloat16).to(torch.float32)
            return blk.cpu().numpy()

        threads = max(1, min(CPU_SHARE, os.cpu_count() or 1))
        first_block = None
        if args.verify:
            nv = min(args.verify, Q)
            t_v = time.perf_counter()
            parts_i, parts_d = [[] for _ in range(nv)], [[] for _ in range(nv)]
            for r0 in range(0, n_total, chunk):
                n = min(chunk, n_total - r0)
                rows_h = corpus_block(r0, n)
                if r0 == 0:
                    first_block = rows_h
                wi, wd, wc = oracle.parallel_top_k(rows_h, q_h[:nv], K, size=threads, threads=threads)
                for q in range(nv):
                    parts_i[q].append(wi[q, :wc[q]] + np.uint64(r0))
                    parts_d[q].append(wd[q, :wc[q]])
            ok_i = ok_d = True
            for q in range(nv):
                gi, gd = oracle.global_top_k(np.concatenate(parts_i[q]), np.concatenate(parts_d[q]), K)
                c = int(res_c[q])
                ok_i &= c == len(gi) and np.array_equal(res_i[q, :c], gi)
                ok_d &= c == len(gd) and np.array_equal(res_d[q, :c].view(np.uint32), gd.view(np.uint32))
            out["parity_spot_check"] = {
                "queries": nv, "rows": n_total, "indices_equal": bool(ok_i), "distance_bits_equal": bool(ok_d),
                "method": f"oracle (oracle/bsr_oracle.c) over the regenerated corpus in {chunk}-row blocks, "
                          f"merged with compute_global_top_k; {time.perf_counter() - t_v:.1f} s"}
        if world == 1 and not args.no_cpu_baseline:
            # P = 1, 2, 4, 8, 16 rank threads (the mpiexec analogue), each on a bounded sample:
            # the first 1M rows (the reference's per-row cost is linear in rows), queries
            # scaled per P to ~cpu_seconds; reported as queries/s over the full corpus.
            rows_s = first_block if first_block is not None else corpus_block(0, min(chunk, n_total))
            n_s = rows_s.shape[0]
            sweep = []
            for P in [p for p in (1, 2, 4, 8, 16) if p <= threads]:
                t1 = time.perf_counter()
                oracle.parallel_top_k(rows_s, q_h[1:2], K, size=P, threads=P)
                one = time.perf_counter() - t1
                nq_cpu = max(1, min(Q, int(args.cpu_seconds / max(one, 1e-3))))
                t1 = time.perf_counter()
                oracle.parallel_top_k(rows_s, q_h[:nq_cpu], K, size=P, threads=P)
                dt = time.perf_counter() - t1
                sweep.append({"P": P, "queries": nq_cpu, "seconds": round(dt, 3),
                              "qps_full_corpus": round(nq_cpu / dt * n_s / n_total, 4)})
            best = max(sweep, key=lambda s: s["qps_full_corpus"])
            out["cpu_baseline"] = {
                "value": best["qps_full_corpus"], "unit": "queries/s", "cores": best["P"], "kind": "port",
                "sample": f"oracle/bsr_oracle.c (the reference path restated: per-rank block scan + stable "
                          f"sort, rank-order gather, stable sort + dedupe) with P rank threads over the first "
                          f"{n_s} rows of the corpus, {best['queries']} queries at the best P; queries/s over "
                          f"{n_total} rows = measured x {n_s}/{n_total}",
                "sweep": sweep, "nproc": os.cpu_count(), "cpu_share": CPU_SHARE, "cpu_model": cpu_model()}
        elif world == 1:
            out["cpu_baseline"] = None
    if rank == 0:
        out.setdefault("cpu_baseline", None)  # N > 1: the baseline is measured at N = 1 only
        print(json.dumps(out), flush=True)
    if watchdog:
        watchdog.disarm()
    barrier(timeout=max(args.collective_timeout, 1200))  # (rank 0's spot-check and CPU sweep ran)
    if comm:
        comm.close()
    index.close()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
