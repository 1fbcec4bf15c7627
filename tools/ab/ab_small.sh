#!/bin/bash
# A/B on one box (tooling): bench.py at the 8-GPU shard size (1.25M rows x 1000 queries), where
# the per-batch small kernels weigh most, with alternative builds of libbsr.so
# (tools/ab/libbsr_<name>.so; "new" = the tree's build), interleaved, two rounds.
# usage: bash tools/ab/ab_small.sh old new
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
O=gpurun_out/ab_small; rm -rf $O; mkdir -p $O
B="python bench.py --config c2 --rows 1250000 --steps 50 --warmup 5 --no-cpu-baseline --verify 2 --p50-iters 10"
for r in 1 2; do
  for v in "$@"; do
    if [ "$v" = new ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
    BSR_LIB=$L timeout -k 10 200 $B > $O/bench_${v}_$r.json 2>>$O/err.txt || exit $?
    python3 -c "import json; d=json.load(open('$O/bench_${v}_$r.json')); print('$v', $r, d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['p50_ms'], d['kernels_ms_per_step_rank0'], d['parity_spot_check']['indices_equal'])"
  done
done
echo done
