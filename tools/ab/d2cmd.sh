cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
mkdir -p gpurun_out/d2
timeout -k 10 180 ./tools/microbench/gemm_ablate 1000000 1000 10 2 > gpurun_out/d2/ablate.txt 2>&1 || exit $?
BSR_LIB=tools/ab/libbsr_d2.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/d2/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/d2/pytest.log; [ $rc -eq 0 ] || exit $rc
bash tools/ab/ab_run.sh new d2
