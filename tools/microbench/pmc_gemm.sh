#!/bin/bash
# PMC passes over the filter microbenchmark (tooling).  Each pass is its own rocprofv3 run.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B=./tools/microbench/gemm_ablate
O=gpurun_out/pmc_gemm
mkdir -p $O
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
            "SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_MFMA SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS" \
            "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $pass -d $O/p$i -o run --output-format csv -- $B 1000000 1000 1e9 > $O/p$i.log 2>&1
done
echo done
