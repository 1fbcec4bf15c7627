cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
O=gpurun_out/r02f; mkdir -p $O
for d in 8 16 12; do
BSR_KS_DIV=$d timeout -k 10 300 python bench.py --no-cpu-baseline --verify 2 > $O/bench_ks$d.json 2> $O/bench_ks$d.err; rc=$?; echo "ks$d rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
BSR_KS_DIV=16 timeout -k 10 300 python bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline --verify 2 --p50-iters 3 > $O/bench_c5_ks16.json 2> $O/bench_c5.err; echo "c5 rc=$?"
