#!/bin/bash
# Round 3 (tooling): dynamic tail gated on shard size -- A/B vs the tail on every shard
# (tools/ab/libbsr_tailall.so), bench at 1M and 1.25M rows, interleaved, 3 rounds.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03oo
mkdir -p "$O"
for r in 1 2 3; do
  for rows in 1000000 1250000; do
    for v in gated tailall; do
      if [ $v = gated ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
      BSR_LIB=$L timeout -k 10 200 python bench.py --rows $rows --steps 40 --no-cpu-baseline --no-configs1 --verify 0 --p50-iters 3 > "$O/b_${v}_${rows}_$r.json" 2>> "$O/err.txt"
      rc=$?; [ $rc -eq 0 ] || { echo "bench $v $rows rc=$rc"; exit $rc; }
      python -c "import json;d=json.load(open('$O/b_${v}_${rows}_$r.json'));print('$v', $rows, $r, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
    done
  done
done
echo done
