"""bench.py's contract on the GPU (the driver parses its one JSON line every round): the
default workload at a reduced row count, configs[0] through the parquet store (`--config c1`)
and the N > 1 path (`--gpus 2 --comm host`: spawn, sharding, the library's exchange and the
root merge, the spot-check over the whole corpus) with two rank processes on the one GPU.
Each run is a child process; nothing here re-executes a GPU-initialised process."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUICK = ["--steps", "3", "--warmup", "1", "--settle-ms", "0", "--p50-iters", "2", "--no-cpu-baseline"]


def _bench(*args, timeout=240):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stdout[-2000:], r.stderr[-4000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout  # exactly one JSON line on stdout
    return json.loads(lines[0])


def _common(d, n_gpus, steps=3):
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert key in d, key
    assert d["n_gpus"] == n_gpus and d["steps"] == steps and d["warmup"] == 1
    assert d["value"] > 0 and d["ms_per_step"] > 0 and d["higher_is_better"] is True
    assert d["unit"] == "queries/s" and d["dtype"] == "f32" and d["scaling"] in ("strong", "weak")
    assert "workload" in d["config"]


def test_bench_default_workload_small(gpu):
    d = _bench("--rows", "300000", "--no-configs1", "--verify", "2", *QUICK)
    _common(d, 1)
    rf = d["roofline"]
    assert rf["bound"] == "mfma" and rf["unit"] == "TOP/s" and rf["peak"] == 5000.0
    assert 0 < rf["frac"] < 1 and abs(rf["achieved"] / rf["peak"] - rf["frac"]) < 1e-3
    assert rf["algorithmic_ops_per_launch"] == 2 * 1000 * 300000 * 768
    assert d["cpu_baseline"] is None  # --no-cpu-baseline
    sc = d["parity_spot_check"]
    assert sc["indices_equal"] and sc["distance_bits_equal"]
    assert d["fallback_queries_per_step_rank0"] == 0
    assert d["self_query_rank1"] is True


def test_bench_configs0_parquet_store(gpu):
    d = _bench("--config", "c1", *QUICK)
    _common(d, 1)
    p = d["parity_all_queries"]
    assert p["queries"] == 32 and p["indices_equal"] and p["distance_bits_equal"]
    assert d["parquet_load_ms"] > 0


def test_bench_two_ranks_host_transport(gpu):
    d = _bench("--gpus", "2", "--comm", "host", "--rows", "200000", "--verify", "2", *QUICK)
    _common(d, 2)
    assert "HOST all-gather" in d["config"]["parallelism"]
    assert d["exchange_ms_per_step"] is not None
    sc = d["parity_spot_check"]
    assert sc["indices_equal"] and sc["distance_bits_equal"]


def test_bench_loopback_rank_step(gpu):
    """bench.py --comm loopback --gpus 4: a recorded 4-rank host-transport run of the batch, then ONE
    process timing rank 0's step with every all-gather emulated on the device and replayed from
    that recording; its result is the 4-rank run's global top-k (spot-checked over the whole
    corpus), every all-gather of the timed searches replayed."""
    d = _bench("--comm", "loopback", "--gpus", "4", "--rows", "400000", "--verify", "2", *QUICK)
    _common(d, 1)
    lb = d["loopback"]
    assert lb["ranks"] == 4 and lb["recorded_calls_per_search"] == 3
    assert lb["missed_allgathers"] == 0 and lb["replayed_allgathers"] >= 3 * 3
    assert d["config"]["rows_per_gpu_rank0"] == 100000 and "loopback" in d["config"]["parallelism"]
    assert d["candidates_per_query"] == 0  # the global-threshold path
    sc = d["parity_spot_check"]
    assert sc["rows"] == 400000 and sc["indices_equal"] and sc["distance_bits_equal"]


def _failing_run(extra=(), timeout=60):
    """bench.py --gpus 2 with rank 1 failing on purpose (BSR_BENCH_FAIL_RANK): the launcher must
    end rank 0 -- blocked in a collective with the dead rank -- and report, within the time."""
    import time
    env = dict(os.environ, BSR_BENCH_FAIL_RANK="1")
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm", "host",
                        "--rows", "200000", *QUICK, *extra], cwd=ROOT, capture_output=True, text=True,
                       timeout=timeout, env=env)
    dt = time.monotonic() - t0
    assert r.returncode != 0 and dt < timeout, (r.returncode, dt)
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    d = json.loads(lines[-1])
    assert d["value"] is None and d["failed_rank"] == 1 and "rank 1 exited with status 3" in d["error"]
    assert "BSR_BENCH_FAIL_RANK" in d["stderr_tail"]
    return d


def test_bench_failing_rank_fails_fast(gpu):
    _failing_run()


def _two_gpus():
    try:
        import torch  # (counting devices does not initialise the GPU)
        return torch.cuda.device_count() >= 2
    except Exception:
        return False


# The RCCL transport needs one device per rank (RCCL refuses two ranks on one device): these run
# on a box with two or more GPUs and are skipped on the one-GPU box (the driver's 8-GPU scale run
# exercises the same path through bench.py --gpus N).
@pytest.mark.skipif(not _two_gpus(), reason="RCCL: one device per rank, needs >= 2 GPUs")
def test_bench_two_ranks_rccl(gpu):
    d = _bench("--gpus", "2", "--rows", "200000", "--verify", "2", *QUICK)
    _common(d, 2)
    assert "HOST" not in d["config"]["parallelism"]
    sc = d["parity_spot_check"]
    assert sc["indices_equal"] and sc["distance_bits_equal"]


@pytest.mark.skipif(not _two_gpus(), reason="RCCL: one device per rank, needs >= 2 GPUs")
def test_bench_failing_rank_fails_fast_rccl(gpu):
    import time
    env = dict(os.environ, BSR_BENCH_FAIL_RANK="1")
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--rows", "200000", *QUICK],
                       cwd=ROOT, capture_output=True, text=True, timeout=90, env=env)
    assert r.returncode != 0 and time.monotonic() - t0 < 90
    d = json.loads([ln for ln in r.stdout.splitlines() if ln.strip()][-1])
    assert d["value"] is None and d["failed_rank"] == 1
