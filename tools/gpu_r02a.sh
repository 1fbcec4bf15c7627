cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r02a; mkdir -p $O
timeout -k 10 120 ./tools/microbench/gemm_ablate 1000000 1000 4 "S2" > $O/ablate.txt 2>&1; echo "ablate rc=$?"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 > $O/bench_prof.json 2> $O/prof.err; rc=$?; echo "stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc1 -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --verify 0 --p50-iters 2 > $O/pmc1.json 2>> $O/prof.err; rc=$?; echo "pmc1 rc=$rc"
