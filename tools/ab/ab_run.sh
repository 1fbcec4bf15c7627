#!/bin/bash
# A/B on one box (tooling): bench.py with alternative builds of libbsr.so (tools/ab/libbsr_<name>.so;
# "new" = the tree's build), interleaved, two rounds.  usage: bash tools/ab/ab_run.sh old ps new
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
O=gpurun_out/ab; rm -rf $O; mkdir -p $O
B="python bench.py --steps 30 --warmup 5 --no-cpu-baseline --verify 0 --p50-iters 5"
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = new ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
    BSR_LIB=$L timeout -k 10 200 $B > $O/bench_${v}_$r.json 2>>$O/err.txt || exit $?
  done
done
echo done
