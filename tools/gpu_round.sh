#!/bin/bash
# Standard measurement pass on the GPU box (tooling): GPU parity tests, the default bench
# (configs[2] corpus 10M x 1000, with the configs[1] side line), the configs[3] / configs[4]
# benches, configs[1] and the 1.25M-row shard of an 8-GPU run, then rocprofv3 kernel stats of the default bench.
# Every GPU step has its own time limit; a crash or time limit ends the script.
# (The PMC passes are tools/gpu_r02p.sh; the filter A/B microbenchmark tools/microbench.)
# usage: bash tools/gpu_round.sh TAG
TAG=${1:-run}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"

timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 400 python bench.py > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c4 --steps 5 --warmup 2 --verify 2 --no-cpu-baseline --no-configs1 > "$O/bench_c4.json" 2>> "$O/bench.err"
rc=$?; echo "bench c4 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --verify 2 --no-cpu-baseline --no-configs1 > "$O/bench_c5.json" 2>> "$O/bench.err"
rc=$?; echo "bench c5 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c1 --steps 50 --warmup 5 > "$O/bench_c1.json" 2>> "$O/bench.err"
rc=$?; echo "bench c1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 3 --verify 2 --no-cpu-baseline --no-configs1 > "$O/bench_c2.json" 2>> "$O/bench.err"
rc=$?; echo "bench c2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --rows 1250000 --steps 30 --warmup 3 --verify 2 --no-cpu-baseline --no-configs1 > "$O/bench_125.json" 2>> "$O/bench.err"
rc=$?; echo "bench 1.25M rc=$rc"; [ $rc -eq 0 ] || exit $rc

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 --no-configs1 > "$O/bench_prof.json" 2> "$O/prof.err"
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo done
