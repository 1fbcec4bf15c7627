#!/bin/bash
# Standard measurement pass on the GPU box (tooling): filter microbenchmark, GPU parity
# tests, bench (int8 and bf16 filters), rocprofv3 kernel stats and the PMC HBM-traffic
# passes of the bench command.  Every GPU step has its own time limit; a crash or time
# limit (exit status other than 0/1) ends the script.
# usage: bash tools/gpu_round.sh TAG
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

timeout -k 10 180 ./tools/microbench/gemm_ablate 1000000 1000 10 > "$O/gemm_ablate.txt" 2>&1
rc=$?; echo "microbench rc=$rc"; ok $rc || exit $rc

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; ok $rc || exit $rc

timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --filter bf16 --no-cpu-baseline --verify 2 > "$O/bench_bf16.json" 2>> "$O/bench.err"
rc=$?; echo "bench bf16 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --verify 2 --no-cpu-baseline > "$O/bench_c5.json" 2>> "$O/bench.err"
rc=$?; echo "bench c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --verify 2 --no-cpu-baseline > "$O/bench_c4.json" 2>> "$O/bench.err"
rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 > "$O/bench_prof.json" 2> "$O/prof.err"
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc

for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $c --output-format csv -d "$O/pmc_$c" -o run -- \
        python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 --p50-iters 2 > /dev/null 2>> "$O/prof.err"
    rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_traffic.py "$O/pmc_FETCH_SIZE" "$O/pmc_WRITE_SIZE" 1000000 1000 i8 "$O/pmc_traffic.json"
echo done
