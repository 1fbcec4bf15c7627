#!/bin/bash
# Round 3 (tooling): rescore prefetch depth (chunks of 64 rows x 64 floats in flight per wave,
# lab toggle BSR_RESCORE_P = 2 / 3 / 4) at the 1.25M and 10M shards: parity, kernel traces.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p "$O"
BSR_RESCORE_P=4 timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > "$O/pytest_p4.log" 2>&1
rc=$?; echo "pytest p4 rc=$rc"; tail -2 "$O/pytest_p4.log"; [ $rc -eq 0 ] || exit $rc
for rows in 1250000 10000000; do
for p in 2 3 4; do
  export BSR_RESCORE_P=$p
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$O/tl_${rows}_$p" -o run -- \
      python3 bench.py --rows $rows --no-cpu-baseline --no-configs1 --verify 1 --steps 30 --p50-iters 3 > "$O/bench_${rows}_$p.json" 2> "$O/tl.err"
  rc=$?; echo "trace $rows P=$p rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find "$O/tl_${rows}_$p" -name "*kernel_trace.csv" | head -1)
  python3 tools/diag/timeline.py "$f" 20 > "$O/timeline_${rows}_$p.txt"; grep -E "rescore|span|turnaround" "$O/timeline_${rows}_$p.txt"
  head -c 200 "$O/bench_${rows}_$p.json"; echo
done
done
echo done
