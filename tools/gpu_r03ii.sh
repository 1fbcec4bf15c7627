#!/bin/bash
# Round 3 (tooling): stamp split of the emit filter with the DMA wait timed apart from the barrier.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03ii
mkdir -p "$O"
for rows in 10000000 1250000; do
  BSR_LIB=tools/ab/libbsr_fstamps.so timeout -k 10 240 python tools/diag/filter_stamps.py $rows > "$O/stamps_$rows.txt" 2>&1
  rc=$?; echo "stamps $rows rc=$rc"; grep -v amdgpu.ids "$O/stamps_$rows.txt"; [ $rc -eq 0 ] || exit $rc
done
echo done
