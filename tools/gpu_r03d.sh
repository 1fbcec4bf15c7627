#!/bin/bash
# Round 3 (tooling): emit-filter ablation A/B (1M and 10M rows), then the GPU suite.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p "$O"
timeout -k 10 150 tools/microbench/qs64_ab 1000000 1000 15 0.125 > "$O/ab_1m.txt" 2>&1
rc=$?; echo "ab 1M rc=$rc"; cat "$O/ab_1m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 tools/microbench/qs64_ab 10000000 1000 6 0.14 > "$O/ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; cat "$O/ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=25 > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -32 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
echo done
