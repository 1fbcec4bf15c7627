#!/bin/bash
# Round 3 (tooling): instruction-cache counters of the emit filter (is the epilogue's ~10 cycles
# per instruction instruction fetch?).  Lists the counters, then one --pmc pass over the harness.
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/r03ss
mkdir -p "$O"
timeout -k 10 60 rocprofv3 -L > "$O/counters.txt" 2>&1
rc=$?; echo "list rc=$rc"; grep -oE "SQC_[A-Z_]*|SQ_IFETCH[A-Z_]*|SQ_INSTS_[A-Z_]*" "$O/counters.txt" | sort -u | tr '\n' ' '; echo
C=""
for c in SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE; do
  grep -q "\b$c\b" "$O/counters.txt" && C="$C $c"
done
echo "counters:$C"
[ -n "$C" ] || exit 0
timeout -s KILL 120 rocprofv3 --pmc $C SQ_IFETCH SQ_WAVES -d "$O/p1" -o run --output-format csv -- tools/microbench/qs64_ab 10000000 1000 2 0.14 > "$O/p1.log" 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 "$O/p1.log"
echo done
