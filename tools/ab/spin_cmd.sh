cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
O=gpurun_out/spin; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --verify 0 --p50-iters 100"
for r in 1 2; do
  BSR_LIB=tools/ab/libbsr_head.so timeout -k 10 200 $B > $O/head_$r.json 2>>$O/err.txt || exit $?
  timeout -k 10 200 $B > $O/spin_$r.json 2>>$O/err.txt || exit $?
done
echo done
