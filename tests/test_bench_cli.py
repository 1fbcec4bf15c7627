"""bench.py's N > 1 launcher on CPU: a rank that dies must not leave the others blocked
(src/mpi_helpers/metrics.rs:185-197 -- no rank may be left waiting in a collective).  Rank 1
fails on purpose before its first collective (BSR_BENCH_FAIL_RANK); rank 0 is then waiting
for it in the process-group rendezvous.  The launcher must end rank 0, exit non-zero within
60 s and print one JSON error line naming rank 1 and its stderr tail.  No GPU is touched."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_failing_rank_fails_fast_cpu():
    env = dict(os.environ, BSR_BENCH_FAIL_RANK="1")
    t0 = time.monotonic()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--comm", "host",
                        "--rows", "1000", "--no-cpu-baseline"], cwd=ROOT, capture_output=True, text=True,
                       timeout=120, env=env)
    dt = time.monotonic() - t0
    assert r.returncode == 3 and dt < 60, (r.returncode, dt, r.stderr[-2000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["value"] is None and d["failed_rank"] == 1 and "rank 1 exited with status 3" in d["error"]
    assert "BSR_BENCH_FAIL_RANK" in d["stderr_tail"]
