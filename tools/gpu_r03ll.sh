#!/bin/bash
# Round 3 (tooling): barrier after the epilogue (VAR 8) -- harness A/B, stamp split of VAR 8.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03ll
mkdir -p "$O"
timeout -k 10 240 tools/microbench/qs64_ab 10000000 1000 10 0.14 > "$O/ab_10m.txt" 2>&1
rc=$?; echo "ab 10M rc=$rc"; grep -E "IDENTICAL|DIFFER|median" "$O/ab_10m.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 150 tools/microbench/qs64_ab 1250000 1000 20 0.125 > "$O/ab_125.txt" 2>&1
rc=$?; echo "ab 1.25M rc=$rc"; grep -E "IDENTICAL|DIFFER|median" "$O/ab_125.txt"; [ $rc -eq 0 ] || exit $rc
for rows in 10000000 1250000; do
  BSR_LIB=tools/ab/libbsr_fstamps.so timeout -k 10 240 python tools/diag/filter_stamps.py $rows > "$O/stamps_$rows.txt" 2>&1
  rc=$?; echo "stamps $rows rc=$rc"; grep -v amdgpu.ids "$O/stamps_$rows.txt"; [ $rc -eq 0 ] || exit $rc
done
echo done
