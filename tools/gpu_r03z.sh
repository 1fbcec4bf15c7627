#!/bin/bash
# Round 3 (tooling): GPU suite after the two-wave query prep and the one-read tau selection;
# rescore phase stamps; 1.25M timeline; default bench.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p "$O"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread --durations=15 > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -20 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc
for rows in 1250000 10000000; do
  BSR_LIB=tools/ab/libbsr_stamps.so timeout -k 10 240 python tools/diag/rescore_stamps.py $rows > "$O/stamps_$rows.txt" 2>&1
  rc=$?; echo "stamps $rows rc=$rc"; cat "$O/stamps_$rows.txt"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/tl125" -o run -- \
    python3 bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 1 --steps 30 --p50-iters 3 > "$O/bench_125_prof.json" 2> "$O/tl.err"
rc=$?; echo "trace 1.25M rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find "$O/tl125" -name "*kernel_trace.csv" | head -1)
python3 tools/diag/timeline.py "$f" 20 > "$O/timeline_125.txt"; python3 tools/diag/gaps.py "$f" 100 >> "$O/timeline_125.txt"; cat "$O/timeline_125.txt"
f=$(find "$O/tl125" -name "*kernel_stats.csv" | head -1); grep -E "rows_to_i8|row_norms" "$f"
timeout -k 10 300 python bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 2 --steps 30 > "$O/bench_125.json" 2> "$O/bench.err"
rc=$?; echo "bench 1.25M rc=$rc"; head -c 300 "$O/bench_125.json"; echo; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > "$O/bench.json" 2>> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; head -c 300 "$O/bench.json"; echo; [ $rc -eq 0 ] || exit $rc
echo done
