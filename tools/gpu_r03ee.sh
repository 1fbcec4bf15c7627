#!/bin/bash
# Round 3 (tooling): dynamic tail at the 1.25M shard -- per-workgroup times and tile counts.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03ee
mkdir -p "$O"
for rows in 1250000 10000000; do
  BSR_LIB=tools/ab/libbsr_counters.so timeout -k 10 240 python tools/diag/filter_wg_balance.py $rows > "$O/wg_$rows.txt" 2>&1
  rc=$?; echo "wg $rows rc=$rc"; grep -E "launch 9|by XCD|tiles" "$O/wg_$rows.txt"; [ $rc -eq 0 ] || exit $rc
done
