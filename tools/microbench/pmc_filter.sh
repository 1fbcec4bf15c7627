#!/bin/bash
# PMC passes over the filter microbenchmark (tooling).  Each pass is its own rocprofv3 run
# (counters only with --kernel-trace-free --pmc; never combined with trace domains).
# usage: bash tools/microbench/pmc_filter.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
B=./tools/microbench/gemm_ablate
O=${1:-gpurun_out/pmc_filter}
mkdir -p "$O"; rm -f "$O/summary.txt"
for var in "i8 tau=inf" "i8 tau=0.125" "i8 no-DMA" "i8 DMA-only"; do
i=0
tag=$(echo "$var" | tr ' =.' '___')
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
            "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU" \
            "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  mkdir -p "$O/$tag"; timeout -k 10 120 rocprofv3 --pmc $pass -d "$O/$tag/p$i" -o run --output-format csv -- $B 1000000 1000 3 "$var" > "$O/$tag/p$i.log" 2>&1
  rc=$?; echo "$var pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
echo "== $var" >> "$O/summary.txt"
python3 tools/microbench/pmc_summary.py "$O/$tag" >> "$O/summary.txt"
done
cat "$O/summary.txt"
