#!/bin/bash
# Round 3 (tooling): the row stream DMA issued by waves 0-3 only (VAR 64) -- harness A/B at 10M and 1.25M.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03xx
mkdir -p "$O"
timeout -k 10 240 tools/microbench/qs64_ab 10000000 1000 10 0.14 > "$O/ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; grep -E "IDENTICAL|DIFFER|median" "$O/ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tools/microbench/qs64_ab 1250000 1000 20 0.125 > "$O/ab_125.txt" 2>&1
rc=$?; echo "ab 1.25M rc=$rc"; grep -E "IDENTICAL|DIFFER|median" "$O/ab_125.txt"; [ $rc -eq 0 ] || exit $rc
echo done
