#!/bin/bash
# Round 3, first pass (tooling): the whole GPU suite (new multi-rank, 50M configs[4], graph
# replay freshness tests), then the default bench.  Each GPU step under its own limit.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread --durations=20 > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; cat "$O/bench.json" | head -c 600; [ $rc -eq 0 ] || exit $rc
echo done
