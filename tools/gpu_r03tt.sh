#!/bin/bash
# Round 3 (tooling): HBM traffic of the emit filter at HEAD (FETCH_SIZE / WRITE_SIZE passes, one
# counter per rocprofv3 run) for the rank shards at N = 1, 2, 4, 8 (10M, 5M, 2.5M, 1.25M rows),
# merged into a copy of profiles/pmc_traffic.json, then one SQ/GRBM pass at 10M.
TAG=r03tt
export PMC_RUN="round 3 ($TAG, HEAD with the dynamic tail)"
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
cp profiles/pmc_traffic.json "$O/pmc_traffic.json"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 --p50-iters 2 --no-configs1"
for rows in 10000000 5000000 2500000 1250000; do
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 240 rocprofv3 --pmc $c --output-format csv -d "$O/t$rows/$c" -o run -- $B --rows $rows > /dev/null 2>> "$O/pmc.err"
        rc=$?; echo "pmc $rows $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    python3 tools/pmc_traffic.py "$O/t$rows/FETCH_SIZE" "$O/t$rows/WRITE_SIZE" $rows 1000 i8 "$O/pmc_traffic.json" || exit 1
done
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA" \
            "GRBM_GUI_ACTIVE GRBM_COUNT"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $pass --output-format csv -d "$O/sq/p$i" -o run -- $B > /dev/null 2>> "$O/pmc.err"
    rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/microbench/pmc_summary.py "$O/sq" > "$O/pmc_summary.txt"
grep -A20 "qs16<true" "$O/pmc_summary.txt" | head -22
echo done
