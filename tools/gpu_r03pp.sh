#!/bin/bash
# Round 3 (tooling): non-temporal loads -- the emit filter's row-stream DMA (harness A/B) and
# the skinny (p50) filter's A fragments (bench A/B: HEAD vs tools/ab/libbsr_snt.so).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03pp
mkdir -p "$O"
timeout -k 10 240 tools/microbench/qs64_ab 10000000 1000 10 0.14 > "$O/ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; grep -E "IDENTICAL|DIFFER|median" "$O/ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tools/microbench/qs64_ab 1250000 1000 20 0.125 > "$O/ab_125.txt" 2>&1
rc=$?; echo "ab 1.25M rc=$rc"; grep -E "IDENTICAL|DIFFER|median" "$O/ab_125.txt"; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in head snt; do
    if [ $v = head ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
    BSR_LIB=$L timeout -k 10 200 python bench.py --steps 3 --p50-iters 60 --no-cpu-baseline --no-configs1 --verify 0 > "$O/b_${v}_$r.json" 2>> "$O/err.txt"
    rc=$?; [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
    python -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v', $r, 'p50', d['p50_ms'], 'skinny', d['roofline_p50']['avg_launch_ms'], d['roofline_p50']['frac'], 'q/s', d['value'])"
  done
done
echo done
