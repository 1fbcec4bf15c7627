#!/bin/bash
# Round 3 (tooling): one barrier per 3 slices (ring of 9-10 slots) vs the product's per-2, A/B.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p "$O"
timeout -k 10 240 tools/microbench/qs64_ab 10000000 1000 8 0.14 > "$O/ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; cat "$O/ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tools/microbench/qs64_ab 1250000 1000 15 0.125 > "$O/ab_125.txt" 2>&1
rc=$?; echo "ab 1.25M rc=$rc"; cat "$O/ab_125.txt"; [ $rc -eq 0 ] || exit $rc
