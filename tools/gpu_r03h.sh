#!/bin/bash
# Round 3 (tooling): GPU suite, 1.25M-row kernel trace timeline, benches (10M, 1.25M, c5, c4).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tl125" -o run -- \
    python3 bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 0 --steps 30 --p50-iters 3 > "$O/bench_125_prof.json" 2> "$O/tl125.err"
rc=$?; echo "trace 1.25M rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$O/tl125" -name "*kernel_trace.csv" | head -1); python3 tools/diag/timeline.py "$f" 40 > "$O/timeline_125.txt"; cat "$O/timeline_125.txt"
timeout -k 10 300 python bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 2 --steps 30 > "$O/bench_125.json" 2> "$O/bench.err"
rc=$?; echo "bench 1.25M rc=$rc"; head -c 300 "$O/bench_125.json"; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --verify 2 --no-cpu-baseline --no-configs1 > "$O/bench_c5.json" 2>> "$O/bench.err"
rc=$?; echo "bench c5 rc=$rc"; head -c 300 "$O/bench_c5.json"; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --verify 2 --no-cpu-baseline --no-configs1 > "$O/bench_c4.json" 2>> "$O/bench.err"
rc=$?; echo "bench c4 rc=$rc"; head -c 300 "$O/bench_c4.json"; echo; [ $rc -eq 0 ] || exit $rc
echo done
