#!/bin/bash
# Round 3 (tooling): stamp split of the level-1 variants (VAR 1 progressive maxima inside the last
# slice, VAR 4 tree) against the product (VAR 0), 10M rows -- does level 1 get shorter?
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03ww
mkdir -p "$O"
for v in 0 1 4; do
  BSR_LIB=tools/ab/libbsr_fst_v$v.so timeout -k 10 240 python tools/diag/filter_stamps.py 10000000 > "$O/stamps_v$v.txt" 2>&1
  rc=$?; echo "stamps VAR $v rc=$rc"; grep -E "level-1|level-2 epi|kt=1|other barriers|loop cycles" "$O/stamps_v$v.txt"; [ $rc -eq 0 ] || exit $rc
done
echo done
