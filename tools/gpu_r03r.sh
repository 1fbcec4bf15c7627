#!/bin/bash
# Round 3 (tooling): result readback through a copy kernel into mapped coherent host memory
# (BSR_READBACK_KERNEL=1) vs the D2H copy node, at the 1.25M-row shard: parity tests, kernel
# traces (per-transition gaps), bench lines, host turnaround.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p "$O"
BSR_READBACK_KERNEL=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multirank.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/pytest_rk.log" 2>&1
rc=$?; echo "pytest rk rc=$rc"; tail -3 "$O/pytest_rk.log"; [ $rc -eq 0 ] || exit $rc
for v in 0 1; do
  if [ $v = 1 ]; then export BSR_READBACK_KERNEL=1; else unset BSR_READBACK_KERNEL; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tl$v" -o run -- \
      python3 bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 0 --steps 30 --p50-iters 3 > "$O/bench_prof_$v.json" 2> "$O/tl$v.err"
  rc=$?; echo "trace $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find "$O/tl$v" -name "*kernel_trace.csv" | head -1)
  python3 tools/diag/timeline.py "$f" 40 > "$O/timeline_$v.txt"; python3 tools/diag/gaps.py "$f" 100 >> "$O/timeline_$v.txt"; cat "$O/timeline_$v.txt"
  timeout -k 10 300 python bench.py --rows 1250000 --no-cpu-baseline --no-configs1 --verify 2 --steps 30 > "$O/bench_125_$v.json" 2>> "$O/bench.err"
  rc=$?; echo "bench $v rc=$rc"; head -c 250 "$O/bench_125_$v.json"; echo; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python tools/diag/host_turnaround.py > "$O/turnaround_$v.txt" 2>&1
  rc=$?; echo "turnaround $v rc=$rc"; cat "$O/turnaround_$v.txt"; [ $rc -eq 0 ] || exit $rc
done
echo done
