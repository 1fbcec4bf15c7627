cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
O=gpurun_out/settle; mkdir -p $O
timeout -k 10 300 python bench.py --settle-ms 0 --no-cpu-baseline > $O/bench_settle0.json 2> $O/err.txt || exit $?
timeout -k 10 300 python bench.py > $O/bench.json 2>> $O/err.txt || exit $?
echo done
