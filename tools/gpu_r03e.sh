#!/bin/bash
# Round 3 (tooling): product (static DMA schedule) vs lab copies at 10M, GPU suite, bench,
# rocprof kernel stats of the bench and a 1.25M-row (8-GPU shard) bench + kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p "$O"
timeout -k 10 150 tools/microbench/qs64_ab 1000000 1000 10 0.125 > "$O/ab_1m.txt" 2>&1
rc=$?; echo "ab 1M rc=$rc"; cat "$O/ab_1m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 tools/microbench/qs64_ab 10000000 1000 6 0.14 > "$O/ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; cat "$O/ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; head -c 1500 "$O/bench.json"; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 2 --steps 30 > "$O/bench_125.json" 2>> "$O/bench.err"
rc=$?; echo "bench 1.25M rc=$rc"; head -c 600 "$O/bench_125.json"; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tl125" -o run -- \
    python3 bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 0 --steps 30 --p50-iters 3 > "$O/bench_125_prof.json" 2> "$O/tl125.err"
rc=$?; echo "trace 1.25M rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$O/tl125" -name "*kernel_trace.csv" | head -1); python3 tools/diag/timeline.py "$f" 40 > "$O/timeline_125.txt"; cat "$O/timeline_125.txt"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 --no-configs1 > "$O/bench_prof.json" 2> "$O/prof.err"
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1); head -12 "$f"
echo done
