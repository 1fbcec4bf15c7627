#!/bin/bash
# Round 3 (tooling): configs[4] shard-5 diagnostic (round-2 library = qs16 emit filter, then
# the tree's = qs64), then the qs64 emit-filter A/B microbenchmark.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p "$O"
BSR_LIB=tools/ab/libbsr_r02.so timeout -k 10 300 python -u tools/diag/c4_shard5.py 5 > "$O/diag_r02lib.txt" 2>&1
rc=$?; echo "diag r02 rc=$rc"; cat "$O/diag_r02lib.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 tools/microbench/qs64_ab 1000000 1000 20 0.125 > "$O/qs64_ab_1m.txt" 2>&1
rc=$?; echo "ab 1M rc=$rc"; cat "$O/qs64_ab_1m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 180 tools/microbench/qs64_ab 10000000 1000 10 0.14 > "$O/qs64_ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; cat "$O/qs64_ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/diag/c4_shard5.py 5 > "$O/diag_tree.txt" 2>&1
rc=$?; echo "diag tree rc=$rc"; cat "$O/diag_tree.txt"; [ $rc -eq 0 ] || exit $rc
echo done
