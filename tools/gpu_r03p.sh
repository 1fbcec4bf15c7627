#!/bin/bash
# PMC evidence for the product filter kernel (k_filter_qs16) through bench.py (tooling):
# kernel stats, two SQ passes, one GRBM pass, then FETCH_SIZE / WRITE_SIZE per shard size
# (10M and 1.25M rows = the rank shards at N=1 and 8), after a lookahead-depth A/B of the filter.  One counter group per
# rocprofv3 run, each under its own time limit; any failure ends the script.
# usage: bash tools/gpu_r03p.sh TAG
TAG=${1:-r03p}
export PMC_RUN="round 3 ($TAG)"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 --p50-iters 2"
timeout -k 10 150 tools/microbench/qs64_ab 10000000 1000 6 0.14 > "$O/ab_10m_ahead.txt" 2>&1
rc=$?; echo "ab rc=$rc"; cat "$O/ab_10m_ahead.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
    python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --verify 0 > "$O/bench_prof.json" 2> "$O/prof.err"
rc=$?; echo "rocprof stats rc=$rc"; [ $rc -eq 0 ] || exit $rc
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA" \
            "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $pass --output-format csv -d "$O/sq/p$i" -o run -- $B --no-configs1 > /dev/null 2>> "$O/pmc.err"
    rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/microbench/pmc_summary.py "$O/sq" > "$O/pmc_summary.txt"
for rows in 10000000 1250000; do
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d "$O/t$rows/$c" -o run -- $B --no-configs1 --rows $rows > /dev/null 2>> "$O/pmc.err"
        rc=$?; echo "pmc $rows $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 tools/pmc_traffic.py "$O/t$rows/FETCH_SIZE" "$O/t$rows/WRITE_SIZE" $rows 1000 i8 "$O/pmc_traffic.json"
done
timeout -k 10 300 python3 bench.py --pmc-json "$O/pmc_traffic.json" > "$O/bench.json" 2> "$O/bench.err"
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
echo done
