#!/bin/bash
# Round 3 (tooling): LDS-DMA skinny filter v3 (p50 path) -- parity with the v3 builds, then a
# bench p50 A/B on one box: HEAD (skinny2) vs v3 ring 24 / ahead 20 and ring 32 / ahead 28.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03rr
mkdir -p "$O"
for v in s3_24 s3_32; do
  BSR_LIB=tools/ab/libbsr_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "small_batches or graph_replay" -x -q --timeout 240 --timeout-method thread > "$O/pytest_$v.log" 2>&1
  rc=$?; echo "pytest $v rc=$rc"; tail -2 "$O/pytest_$v.log"; [ $rc -eq 0 ] || exit $rc
done
BSR_LIB=tools/ab/libbsr_s3_32.so timeout -k 10 400 python -u -m pytest tests/test_gpu_full_size.py -k "configs3" -x -q --timeout 380 --timeout-method thread > "$O/pytest_c3_s3_32.log" 2>&1
rc=$?; echo "pytest configs3 s3_32 rc=$rc"; tail -2 "$O/pytest_c3_s3_32.log"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in head s3_24 s3_32; do
    if [ $v = head ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
    BSR_LIB=$L timeout -k 10 200 python bench.py --steps 3 --p50-iters 60 --no-cpu-baseline --no-configs1 --verify 0 > "$O/b_${v}_$r.json" 2>> "$O/err.txt"
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', $r, 'p50', d['p50_ms'], 'skinny', d['roofline_p50']['avg_launch_ms'], d['roofline_p50']['frac'], 'q/s', d['value'])"
  done
done
echo done
