#!/bin/bash
# Round 3 (tooling): does the slow-XCD pattern of the emit filter follow the XCD or its tiles?
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03cc
mkdir -p "$O"
for x in 0 1 2 0; do
  BSR_LIB=tools/ab/libbsr_counters.so timeout -k 10 240 python tools/diag/filter_wg_balance.py 10000000 $x > "$O/wg_x$x.txt" 2>&1
  rc=$?; echo "xor $x rc=$rc"; grep -E "launches|by XCD|launch 9" "$O/wg_x$x.txt"; [ $rc -eq 0 ] || exit $rc
done
