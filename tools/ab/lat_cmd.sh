cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
O=gpurun_out/lat; mkdir -p $O
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --verify 2 --p50-iters 100 > $O/bench.json 2> $O/err.txt || exit $?
timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline --verify 1 > $O/bench_c4.json 2>> $O/err.txt || exit $?
echo done
