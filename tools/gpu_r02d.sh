#!/bin/bash
# round-2 pass after a kernel change: microbench A/B (cross-checked), GPU parity, default bench,
# rocprof kernel stats.  Each GPU step has its own time limit; a failure ends the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/${1:-r02d}; mkdir -p $O
timeout -k 10 120 ./tools/microbench/ring_ab 1000000 1000 20 0.125 > $O/ring_ab.txt 2>&1; rc=$?; echo "ab rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 --no-configs1 > $O/bench_prof.json 2> $O/prof.err; rc=$?; echo "stats rc=$rc"
