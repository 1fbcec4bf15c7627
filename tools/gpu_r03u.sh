#!/bin/bash
# Round 3 (tooling): phase timestamps of the one-wave-per-query rescore (lab build).
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p "$O"
for rows in 1250000 10000000; do
  BSR_LIB=tools/ab/libbsr_stamps.so timeout -k 10 240 python tools/diag/rescore_stamps.py $rows > "$O/stamps_$rows.txt" 2>&1
  rc=$?; echo "stamps $rows rc=$rc"; cat "$O/stamps_$rows.txt"; [ $rc -eq 0 ] || exit $rc
done
