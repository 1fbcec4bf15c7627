#!/bin/bash
# Round 3 (tooling): multi-rank rehearsal at HEAD on one GPU (host transport over gloo): the
# spawn, sharding, exchange, device root merge and the N > 1 spot-check; the timings are not
# a scaling measurement (the ranks' persistent filters serialise on the shared GPU).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03vv
mkdir -p "$O"
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --comm host --steps 10 --warmup 2 --verify 2 --no-cpu-baseline > "$O/bench_n$n.json" 2> "$O/bench_n$n.err"
  rc=$?; echo "bench N=$n rc=$rc"; head -c 600 "$O/bench_n$n.json"; echo; [ $rc -eq 0 ] || exit $rc
done
echo done
