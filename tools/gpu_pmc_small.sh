#!/bin/bash
# PMC passes over the bench for the small per-batch kernels (tooling): two SQ counter groups,
# each its own rocprofv3 run under its own time limit.  usage: bash tools/gpu_pmc_small.sh TAG
TAG=${1:-pmc_small}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
B="python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --verify 0 --p50-iters 2 --no-configs1"
i=0
for pass in "SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA" \
            "SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE"; do
    i=$((i+1))
    timeout -k 10 240 rocprofv3 --pmc $pass --output-format csv -d "$O/p$i" -o run -- $B > /dev/null 2>> "$O/pmc.err"
    rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 - "$O" <<'PY' > "$O/summary.txt"
import collections, csv, glob, sys
d = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "")
        vals[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
for name in sorted(vals):
    print(name)
    for c in sorted(vals[name]):
        v = vals[name][c]
        print(f"   {c:32s} {sum(v) / len(v):14.6g}")
PY
echo done
