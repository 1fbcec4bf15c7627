#!/bin/bash
# Round 3 (tooling): GPU suite, then the qs64 emit-filter A/B microbenchmark, then the bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03b
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -32 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/microbench/qs64_ab 1000000 1000 20 0.125 > "$O/qs64_ab_1m.txt" 2>&1
rc=$?; echo "ab 1M rc=$rc"; cat "$O/qs64_ab_1m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 tools/microbench/qs64_ab 10000000 1000 10 0.14 > "$O/qs64_ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; cat "$O/qs64_ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; head -c 800 "$O/bench.json"; [ $rc -eq 0 ] || exit $rc
echo done
