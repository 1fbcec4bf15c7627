#!/bin/bash
# Round 3 (tooling): GPU suite (fused finalize), host-turnaround diagnostic at the 1.25M shard,
# benches at 10M and 1.25M.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/diag/host_turnaround.py 1250000 > "$O/turnaround_125.txt" 2>&1
rc=$?; echo "diag rc=$rc"; cat "$O/turnaround_125.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 2 --steps 30 > "$O/bench_125.json" 2> "$O/bench.err"
rc=$?; echo "bench 1.25M rc=$rc"; head -c 300 "$O/bench_125.json"; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$O/bench.json" 2>> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; head -c 300 "$O/bench.json"; echo; [ $rc -eq 0 ] || exit $rc
echo done
