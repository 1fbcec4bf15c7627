#!/bin/bash
# Round 3 (tooling): per-workgroup timing of the persistent emit filter (lab build).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03bb
mkdir -p "$O"
for rows in 10000000 1250000; do
  BSR_LIB=tools/ab/libbsr_counters.so timeout -k 10 240 python tools/diag/filter_wg_balance.py $rows > "$O/wg_$rows.txt" 2>&1
  rc=$?; echo "wg $rows rc=$rc"; cat "$O/wg_$rows.txt"; [ $rc -eq 0 ] || exit $rc
done
