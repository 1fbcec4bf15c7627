#!/bin/bash
# GPU-box measurement passes (tooling), one launcher for every round's runs.
#   usage: bash tools/gpu_round.sh TAG STEP [STEP ...]      (default steps: tests bench)
# Steps (each GPU command under its own time limit; the first failure ends the script):
#   tests       pytest -m gpu (the whole GPU suite)
#   bench       the default bench (configs[2] corpus 10M x 1000 + the configs[1] side line)
#   configs     configs[0] (c1, parquet store), configs[1] (c2), configs[3] (c4), configs[4] (c5)
#   r125        the 1.25M-row shard of an 8-GPU split (the per-rank step of the scale curve)
#   prof        rocprofv3 kernel stats of the default bench
#   timeline    rocprofv3 kernel trace of the 1.25M shard -> per-batch kernel/gap timeline
#   apitrace    rocprofv3 HIP API + kernel trace of the 1.25M shard (the host's share of the turnaround)
#   pmc         HBM traffic (FETCH_SIZE, WRITE_SIZE) at 10M / 5M / 2.5M / 1.25M rows into a copy of
#               profiles/pmc_traffic.json, then one SQ/GRBM pass at 10M
#   pmcsmall    two SQ passes (issue, LDS, waits) over the default bench
#   rehearsal   --gpus 2, 4 and 8 over the host transport on the one GPU (spawn, exchange, root merge)
#   mr          the multi-rank GPU tests alone (tests/test_gpu_multirank.py)
#   rehprof     rocprofv3 kernel stats of the --gpus 8 host rehearsal (every rank process traced)
#   stamps      s_memtime phase split of the emit filter (make lab-fstamps) at 10M and 1.25M
#   counters    emission-epilogue event counts + per-workgroup balance (make lab-counters)
#   (the lab binaries these steps run are built here beforehand -- make -C tools/microbench filter_ab
#    filter_hist ... -- and are git-ignored; the tree holds their sources only)
#   fab         tools/microbench/filter_ab (product vs variants of the emit filter) at 10M and 1.25M
#   fabshard    filter_ab at the rank shards of N = 2, 4, 8 (5M, 2.5M, 1.25M rows) at the global threshold's
#               emission rate (tau 0.1473: ~256 rows per query over the 10M corpus, 256/N per rank)
#   fabpmc      FETCH_SIZE of each filter_ab variant at 10M and 1.25M (HBM traffic per launch)
#   hist        tools/microbench/filter_hist (the product vs the emit filter at earlier commits) at 1M,
#               1.25M (local-threshold rate) and 1.25M at the global threshold's rate (round 5)
#   loopback    bench.py --comm loopback --gpus 8: rank 0's step of an 8-rank run on one GPU (the all-gathers
#               emulated where ncclAllGather sits, replayed from a recorded 8-rank host-transport run)
#   looprec     record an 8-rank host-transport run's all-gathers ($O/loop8.npz) for the loopback steps below
#   rstamps     phase stamps of the global-threshold rescore (lab-stamps build; after looprec)
#   looptl      rocprofv3 kernel trace of the loopback step (replaying looprec) -> per-search timeline
#   loopapi     rocprofv3 HIP API + kernel trace of the loopback step -> the host's calls between searches
#   abloop:A,B  the loopback step with alternative libbsr builds (tools/ab/libbsr_<A>.so; "new" = tree)
#   mpub        tools/microbench/merge_pub with and without the host-row writers' system-scope release
#   mrfull      the full-size 8-rank global-threshold tests (configs[2], configs[4])
#   ab:A,B,...  bench.py A/B of alternative libbsr builds (tools/ab/libbsr_<A>.so; "new" = tree),
#               interleaved, two rounds; ab125:A,B,... the same at the 1.25M-row shard; abc2 / abc5:
#               configs[1] (1M x 1000) / the configs[4] shard (6.25M bf16 x 4096, top-100)
#   p50ab       p50 with the tiny-batch rescore on / off (BSR_RESCORE_KP), interleaved
#   p50lib:A,B  p50 of one query over 10M rows per libbsr build, interleaved
#   p50rs       the single-query rescore events (tools/diag/p50_rescore.py), kp on / off
#   p50st       the tiny-batch rescore's lab stamps + a kernel timeline of single-query searches at 2M rows
#               (P50ROWS=10000000: the self-thresholded path)
#   seltau      tools/microbench/seltau_ab: k_select_tau_m vs k_select_tau, bit for bit
#   gldstests   the single-query / small-batch tests with k_filter_skinny2 at 768-wide rows (BSR_SKINNY_GLDS=0)
#   p50glds     p50 A/B of the LDS-DMA skinny filter against k_filter_skinny2 at 10M (self-thresholded and
#               thresholded) and 1.25M (thresholded)
#   p50api      the host's HIP API calls between single-query searches (rocprofv3 --hip-trace, tools/diag/api_gap.py)
#   scstamps    the second chance's phases at 10M x 1000 (tools/diag/second_chance_stamps.py, lab-stamps build)
#   kpab        the first rescore pass at 10M x 1000: one wave per query vs the tiny-batch kernel (BSR_RESCORE_KP=2)
#   seltauab    tau0's selection at 10M x 1000: the 4-wave kernel vs the 16-wave one (BSR_SELECT_TAU_M=2)
#   c3fb        the configs[3] searches' stats under the tiny-batch A/B switches (tools/diag/c3_fallback.py)
#   rescue1     the single-query rescue case under the same switches (tools/diag/rescue1.py)
#   abflat      the loopback step with the dealt-rows global-threshold rescore on / off (after looprec)
#   histmid     filter_hist at the 5M / 2.5M rank shards (N = 2 / 4) at the global threshold's rate
#   smoke       __graft_entry__.smoke() (the driver's round-end check)
#   mrall       every multi-rank GPU test (tests/test_gpu_multirank.py, the full-size ones included)
TAG=${1:-run}
shift
STEPS=${*:-tests bench}
cd "${GRAFT_REPO_ROOT:-/root/repo}" || exit 9
export TMPDIR=/tmp
O=gpurun_out/$TAG
mkdir -p "$O"
NOB="--no-cpu-baseline --no-configs1"

run() {  # run SECONDS LABEL OUTFILE CMD...: one GPU step, its limit, its status
    local t=$1 label=$2 out=$3
    shift 3
    timeout -k 10 "$t" "$@" > "$out" 2>> "$O/err.txt"
    local rc=$?
    echo "$label rc=$rc"
    [ $rc -eq 0 ] || exit $rc
}

for step in $STEPS; do
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1
      rc=$?; echo "pytest rc=$rc"; tail -3 "$O/pytest_gpu.log"; [ $rc -eq 0 ] || exit $rc ;;
    bench)
      run 400 bench "$O/bench.json" python bench.py; head -c 400 "$O/bench.json"; echo ;;
    configs)
      run 300 "bench c1" "$O/bench_c1.json" python bench.py --config c1 --steps 50 --warmup 5
      run 300 "bench c2" "$O/bench_c2.json" python bench.py --config c2 --steps 20 --warmup 3 --verify 2 $NOB
      run 300 "bench c4" "$O/bench_c4.json" python bench.py --config c4 --steps 5 --warmup 2 --verify 2 $NOB
      run 300 "bench c5" "$O/bench_c5.json" python bench.py --config c5 --steps 5 --warmup 2 --verify 2 $NOB ;;
    p50ab)
      # the tiny-batch rescore (k_rescore_kp) against the one-wave kernel, same process build,
      # interleaved: p50 of one query over the default corpus and its kernels
      for r in 1 2; do
        for v in 1 0; do
          BSR_RESCORE_KP=$v run 200 "p50 kp=$v $r" "$O/p50ab_${v}_$r.json" python bench.py --steps 3 --warmup 2 \
              --verify 0 --p50-iters 200 $NOB
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('kp', sys.argv[2], d['p50_ms'], d.get('p50_kernels_ms_rank0'))" \
              "$O/p50ab_${v}_$r.json" "$v"
        done
      done ;;
    p50top)
      # round 6: the self-thresholded single-query path on / off, interleaved in one process
      run 400 "p50top" "$O/p50top.txt" python3 tools/diag/p50_top_ab.py 10000000 3 200 ${P50MODES:-1,0}; cat "$O/p50top.txt" ;;
    p50glds)
      # round 6: the LDS-DMA skinny filter (BSR_SKINNY_GLDS=1) against k_filter_skinny2 (=0), interleaved:
      # the self-thresholded path at 10M rows and the thresholded path at the 1.25M-row rank shard
      run 400 "p50glds 10M" "$O/p50glds_10m.txt" python3 tools/diag/p50_top_ab.py 10000000 3 200 1,1g,0,0g
      cat "$O/p50glds_10m.txt"
      run 300 "p50glds 1.25M" "$O/p50glds_125.txt" python3 tools/diag/p50_top_ab.py 1250000 3 300 0,0g
      cat "$O/p50glds_125.txt" ;;
    p50gldslib:*)
      # the same A/B with another libbsr build (tools/ab/libbsr_<NAME>.so), e.g. the default-policy DMA
      L="${step#*:}"
      BSR_LIB=tools/ab/libbsr_$L.so run 400 "p50glds $L 10M" "$O/p50glds_${L}_10m.txt" python3 tools/diag/p50_top_ab.py 10000000 3 200 1,1g
      cat "$O/p50glds_${L}_10m.txt" ;;
    gldstests)
      BSR_SKINNY_GLDS=0 timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
          tests/test_gpu_tiny_top.py tests/test_gpu_parity.py -k "tiny or small_batches or rescue or golden" \
          > "$O/gldstests.log" 2>&1
      rc=$?; echo "glds tests rc=$rc"; tail -3 "$O/gldstests.log"; [ $rc -eq 0 ] || exit $rc ;;
    c4ab)
      # round 6: the configs[3] bench (p50 over 10M rows) with the self-thresholded path on / off, interleaved
      for r in 1 2; do
        for v in 1 0; do
          BSR_SKINNY_TOP=$v run 300 "c4 top=$v $r" "$O/c4ab_${v}_$r.json" python bench.py --config c4 --steps 5 --warmup 2 \
              --verify 1 $NOB
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('top', sys.argv[2], d['p50_ms'], d.get('p50_kernels_ms_rank0'))" \
              "$O/c4ab_${v}_$r.json" "$v"
        done
      done ;;
    mergeab)
      # round 6: the loopback step (rank 0 of 8, replaying $O/loop8.npz from looprec) with the merge's
      # first-occurrence filter forced (BSR_MERGE_HASH=1) or skipped for disjoint rank lists, interleaved
      for r in 1 2; do
        for v in 0 1; do
          BSR_MERGE_HASH=$v run 300 "mergeab hash=$v $r" "$O/mergeab_${v}_$r.json" python bench.py --comm loopback --gpus 8 \
              --replay "$O/loop8.npz" --steps 100 --warmup 5 --verify 1 --no-cpu-baseline
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('hash', sys.argv[2], d['ms_per_step'], d['loopback']['missed_allgathers'])" \
              "$O/mergeab_${v}_$r.json" "$v"
        done
      done ;;
    toptests)
      # round 6: the new collective and single-query tests alone
      timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
        tests/test_gpu_tiny_top.py tests/test_gpu_multirank.py::test_rccl_forced_collectives_single_rank \
        tests/test_gpu_multirank.py::test_rccl_forced_collectives_configs2_shard \
        tests/test_gpu_multirank.py::test_parallel_search_phase_a_faults \
        "tests/test_gpu_parity.py::test_published_rescue_and_fallback_rows" > "$O/toptests.log" 2>&1
      rc=$?; echo "toptests rc=$rc"; tail -25 "$O/toptests.log"; [ $rc -eq 0 ] || exit $rc ;;
    p50rs)
      # the single-query rescore kernels, kp on / off, two rounds (tools/diag/p50_rescore.py)
      for r in 1 2; do
        for v in 1 0; do
          for nq in 1 16; do
            BSR_RESCORE_KP=$v timeout -k 10 200 python3 tools/diag/p50_rescore.py 2000000 $nq >> "$O/p50rs.txt" 2>> "$O/err.txt" || exit 1
          done
        done
      done
      cat "$O/p50rs.txt" ;;
    p50st)
      # the single query's rescore phases (lab stamps) and its kernel timeline (rocprof trace)
      BSR_LIB=tools/ab/libbsr_stamps.so BSR_READ_STAMPS=1 timeout -k 10 200 python3 tools/diag/p50_rescore.py ${P50ROWS:-2000000} 1 \
          > "$O/p50_stamps.txt" 2>> "$O/err.txt" || exit 1
      cat "$O/p50_stamps.txt"
      run 300 "p50 trace" "$O/p50_trace.txt" rocprofv3 --kernel-trace --output-format csv -d "$O/tlp50" -o run -- \
          python3 tools/diag/p50_rescore.py ${P50ROWS:-2000000} 1
      f=$(find "$O/tlp50" -name "*kernel_trace.csv" | head -1)
      python3 tools/diag/timeline.py "$f" 40 > "$O/timeline_p50.txt"; tail -30 "$O/timeline_p50.txt" ;;
    p50lib:*)
      # p50 of one query over the default corpus, per library (new = the tree's), interleaved
      for r in 1 2; do
        for v in $(echo "${step#*:}" | tr , ' '); do
          if [ "$v" = new ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
          BSR_LIB=$L run 200 "p50 $v $r" "$O/p50lib_${v}_$r.json" python bench.py --steps 3 --warmup 2 \
              --verify 0 --p50-iters 200 $NOB
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('p50', sys.argv[2], d['p50_ms'], d.get('p50_kernels_ms_rank0'))" \
              "$O/p50lib_${v}_$r.json" "$v"
        done
      done ;;
    c3fb)
      # the configs[3] searches' stats under the tiny-batch A/B variables (tools/diag/c3_fallback.py)
      for e in "" "BSR_SELECT_TAU_M=0" "BSR_SOLO_PUB=0" "BSR_SELECT_TAU_M=0 BSR_SOLO_PUB=0"; do
        env $e timeout -k 10 200 python3 tools/diag/c3_fallback.py >> "$O/c3fb.txt" 2>> "$O/err.txt" || exit 1
      done
      cat "$O/c3fb.txt" ;;
    seltau)
      timeout -k 10 60 tools/microbench/seltau_ab > "$O/seltau.txt" 2>&1; rc=$?; cat "$O/seltau.txt"; [ $rc -eq 0 ] || exit $rc
      timeout -k 10 60 tools/microbench/seltau_time > "$O/seltau_time.txt" 2>&1; rc=$?; cat "$O/seltau_time.txt"; [ $rc -eq 0 ] || exit $rc ;;
    rescue1)
      for e in "" "BSR_SOLO_PUB=0" "BSR_SELECT_TAU_M=0" "BSR_RESCORE_KP=0" "BSR_SOLO_PUB=0 BSR_SELECT_TAU_M=0 BSR_RESCORE_KP=0"; do
        for nq in 1 2; do
          env $e timeout -k 10 120 python3 tools/diag/rescue1.py $nq >> "$O/rescue1.txt" 2>> "$O/err.txt" || exit 1
        done
      done
      cat "$O/rescue1.txt" ;;
    abflat)
      # the loopback step with the dealt-rows global-threshold rescore on / off (BSR_GT_FLAT), interleaved
      for r in 1 2; do
        for v in 1 0; do
          BSR_GT_FLAT=$v run 300 "abflat $v $r" "$O/abflat_${v}_$r.json" python bench.py --comm loopback --gpus 8 \
              --replay "$O/loop8.npz" --steps 50 --warmup 5 --verify 4 --p50-iters 5 $NOB
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_ms_per_step_rank0']; print('flat', sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['emitted_per_query_rank0'], k['rescore'], d['loopback']['missed_allgathers'], d.get('parity_spot_check'))" \
              "$O/abflat_${v}_$r.json" "$v"
        done
      done ;;
    mrall)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > "$O/pytest_mrall.log" 2>&1
      rc=$?; echo "pytest mrall rc=$rc"; tail -3 "$O/pytest_mrall.log"; [ $rc -eq 0 ] || exit $rc ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > "$O/smoke.txt" 2>&1
      rc=$?; tail -2 "$O/smoke.txt"; [ $rc -eq 0 ] || exit $rc ;;
    histmid)
      # the emit filter builds at the N = 2 / N = 4 rank shards at the global threshold's rate
      run 300 "filter_hist 5M gtau" "$O/hist_5m_g.txt" tools/microbench/filter_hist 5000000 1000 12 0.1473
      run 300 "filter_hist 2.5M gtau" "$O/hist_25m_g.txt" tools/microbench/filter_hist 2500000 1000 15 0.1473
      grep -h -E "median|DIFFER" "$O"/hist_*.txt ;;
    r125)
      run 300 "bench 1.25M" "$O/bench_125.json" python bench.py --rows 1250000 --steps 30 --warmup 3 --verify 2 $NOB
      head -c 400 "$O/bench_125.json"; echo ;;
    p50api)
      # the host's share of the single-query search: HIP API calls between one search's last kernel
      # and the next one's query prep (rocprofv3 HIP API + kernel trace of tools/diag/p50_rescore.py)
      run 300 "p50 api trace" "$O/p50api.txt" rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$O/p50api" \
          -o run -- python3 tools/diag/p50_rescore.py ${P50ROWS:-10000000} 1
      python3 tools/diag/api_gap.py "$O/p50api" "k_rescore<1, 8, 2, 1>" > "$O/api_gap_p50.txt"; cat "$O/api_gap_p50.txt" ;;
    scstamps)
      # the second chance's phases at 10M x 1000 (lab stamps build, made beforehand)
      BSR_LIB=tools/ab/libbsr_stamps.so run 300 "second-chance stamps" "$O/sc_stamps.txt" \
          python3 tools/diag/second_chance_stamps.py 10000000
      cat "$O/sc_stamps.txt" ;;
    kpab)
      # the first rescore pass at 10M x 1000: the one-wave-per-query kernel (the product) against the
      # tiny-batch kernel for every batch size (BSR_RESCORE_KP=2, lab), rocprof averages, interleaved
      for r in 1 2; do
        for v in 1 2; do
          BSR_RESCORE_KP=$v run 300 "kp $v round $r" "$O/kpab_${v}_$r.json" rocprofv3 --kernel-trace --stats \
              --output-format csv -d "$O/kpab_${v}_$r" -o run -- python3 bench.py --steps 10 --warmup 3 --verify 2 $NOB
          python3 tools/diag/kstats.py "$O/kpab_${v}_$r" "$O/kpab_${v}_$r.json" rescore
        done
      done ;;
    seltauab)
      # tau0's selection at 10M x 1000 (9766 values per query): the 4-wave kernel (BSR_SELECT_TAU_M=1,
      # the product) against the 16-wave kernel (=2), rocprof averages, two interleaved rounds;
      # the spot check (--verify 2) confirms identical results
      for r in 1 2; do
        for v in 1 2; do
          BSR_SELECT_TAU_M=$v run 300 "seltau $v round $r" "$O/seltau_${v}_$r.json" rocprofv3 --kernel-trace --stats \
              --output-format csv -d "$O/seltau_${v}_$r" -o run -- python3 bench.py --steps 10 --warmup 3 --verify 2 $NOB
          f=$(find "$O/seltau_${v}_$r" -name "*kernel_stats.csv" | head -1)
          echo "M=$v round $r: $(grep -h -E 'k_select_tau|k_filter_qs16<false' "$f" | cut -d, -f1,2,4 | tr '\n' ' ')"
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('  q/s', d['value'], 'spot', d.get('parity_spot_check',{}).get('indices_equal'), d.get('parity_spot_check',{}).get('distance_bits_equal'))" "$O/seltau_${v}_$r.json"
        done
      done ;;
    prof)
      run 300 "rocprof stats" "$O/bench_prof.json" rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
          python3 bench.py --steps 10 --warmup 3 --verify 0 $NOB
      f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -12 "$f" ;;
    timeline)
      run 300 "trace 1.25M" "$O/bench_125_prof.json" rocprofv3 --kernel-trace --output-format csv -d "$O/tl125" -o run -- \
          python3 bench.py --rows 1250000 --verify 0 --steps 30 --p50-iters 3 $NOB
      f=$(find "$O/tl125" -name "*kernel_trace.csv" | head -1)
      python3 tools/diag/timeline.py "$f" 40 > "$O/timeline_125.txt"; tail -30 "$O/timeline_125.txt" ;;
    apitrace)
      run 300 "hip trace 1.25M" "$O/bench_125_api.json" rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$O/api125" -o run -- \
          python3 bench.py --rows 1250000 --verify 0 --steps 30 --p50-iters 3 $NOB
      find "$O/api125" -name "*.csv" | head -5 ;;
    pmc)
      export PMC_RUN="$TAG"
      cp profiles/pmc_traffic.json "$O/pmc_traffic.json"
      B="python3 bench.py --steps 3 --warmup 1 --verify 0 --p50-iters 2 $NOB"
      for rows in 10000000 5000000 2500000 1250000; do
        for c in FETCH_SIZE WRITE_SIZE; do
          run 240 "pmc $rows $c" /dev/null rocprofv3 --pmc $c --output-format csv -d "$O/t$rows/$c" -o run -- $B --rows $rows
        done
        python3 tools/pmc_traffic.py "$O/t$rows/FETCH_SIZE" "$O/t$rows/WRITE_SIZE" $rows 1000 i8 "$O/pmc_traffic.json" || exit 1
      done
      run 240 "pmc sq" /dev/null rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
          SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --output-format csv -d "$O/sq/p1" -o run -- $B
      run 240 "pmc grbm" /dev/null rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$O/sq/p2" -o run -- $B
      python3 tools/microbench/pmc_summary.py "$O/sq" > "$O/pmc_summary.txt"
      grep -A20 "qs16<true" "$O/pmc_summary.txt" | head -22 ;;
    pmcsmall)
      B="python3 bench.py --steps 3 --warmup 1 --verify 0 --p50-iters 2 $NOB"
      run 240 "pmc small 1" /dev/null rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
          SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA --output-format csv -d "$O/ps/p1" -o run -- $B
      run 240 "pmc small 2" /dev/null rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VALU \
          SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d "$O/ps/p2" -o run -- $B
      python3 tools/microbench/pmc_summary.py "$O/ps" > "$O/pmc_small_summary.txt" ;;
    rehearsal)
      for n in 2 4 8; do
        run 400 "bench N=$n host" "$O/bench_n$n.json" python bench.py --gpus $n --comm host --steps 10 --warmup 2 --verify 2 \
            --no-cpu-baseline
        head -c 600 "$O/bench_n$n.json"; echo
      done ;;
    rehprof)
      run 600 "rehearsal N=8 rocprof" "$O/bench_n8_prof.json" rocprofv3 --kernel-trace --stats --output-format csv \
          -d "$O/rehprof" -o run -- python3 bench.py --gpus 8 --comm host --steps 10 --warmup 2 --verify 0 --no-cpu-baseline \
          --p50-iters 3
      find "$O/rehprof" -name "*kernel_stats.csv" | head -3 ;;
    hist)
      run 200 "filter_hist 1M" "$O/hist_1m.txt" tools/microbench/filter_hist 1000000 1000 25 0.1253
      run 200 "filter_hist 1.25M" "$O/hist_125.txt" tools/microbench/filter_hist 1250000 1000 25 0.1284
      run 200 "filter_hist 1.25M gtau" "$O/hist_125g.txt" tools/microbench/filter_hist 1250000 1000 25 0.1462
      run 300 "filter_hist 10M" "$O/hist_10m.txt" tools/microbench/filter_hist 10000000 1000 9 0.1473
      grep -h -E "median|DIFFER" "$O"/hist_*.txt ;;
    loopback)
      run 600 "loopback N=8" "$O/bench_loop8.json" python bench.py --comm loopback --gpus 8 --steps 50 --warmup 5 \
          --verify 4 --no-cpu-baseline
      head -c 700 "$O/bench_loop8.json"; echo ;;
    looprec)
      run 600 "loopback record" "$O/loop_rec.json" python bench.py --comm host --gpus 8 --record-gathers "$O/loop8.npz" \
          --record-only --settle-ms 0 --warmup 0 --steps 1
      cat "$O/loop_rec.json" ;;
    abloop:*)
      for r in 1 2; do
        for v in $(echo "${step#*:}" | tr , ' '); do
          if [ "$v" = new ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
          BSR_LIB=$L run 300 "abloop $v $r" "$O/abloop_${v}_$r.json" python bench.py --comm loopback --gpus 8 \
              --replay "$O/loop8.npz" --steps 50 --warmup 5 --verify 0 --p50-iters 5 $NOB
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); k=d['kernels_ms_per_step_rank0']; print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['emitted_per_query_rank0'], k['rescore'], d['loopback']['missed_allgathers'])" \
              "$O/abloop_${v}_$r.json" "$v"
        done
      done ;;
    rstamps)
      BSR_LIB=tools/ab/libbsr_stamps.so run 300 "rescore stamps gtau" "$O/rstamps_gtau.txt" python tools/diag/rescore_stamps_gtau.py "$O/loop8.npz"
      grep -v amdgpu.ids "$O/rstamps_gtau.txt" ;;
    loopapi)
      run 300 "loopback api trace" "$O/bench_loop8_api.json" rocprofv3 --hip-trace --kernel-trace --output-format csv -d "$O/apiloop" -o run -- \
          python3 bench.py --comm loopback --gpus 8 --replay "$O/loop8.npz" --verify 0 --steps 30 --p50-iters 3 $NOB
      python3 tools/diag/api_gap.py "$O/apiloop" > "$O/api_gap_loop8.txt"; cat "$O/api_gap_loop8.txt" ;;
    looptl)
      run 300 "loopback trace" "$O/bench_loop8_prof.json" rocprofv3 --kernel-trace --output-format csv -d "$O/tlloop" -o run -- \
          python3 bench.py --comm loopback --gpus 8 --replay "$O/loop8.npz" --verify 0 --steps 30 --p50-iters 3 --settle-ms 0 $NOB
      f=$(find "$O/tlloop" -name "*kernel_trace.csv" | head -1)
      python3 tools/diag/timeline.py "$f" 40 > "$O/timeline_loop8.txt"; tail -30 "$O/timeline_loop8.txt" ;;
    mpub)
      run 120 "merge_pub" "$O/merge_pub.txt" tools/microbench/merge_pub 300
      run 120 "merge_pub no sysrel" "$O/merge_pub_nosysrel.txt" tools/microbench/merge_pub_nosysrel 300
      cat "$O/merge_pub.txt" "$O/merge_pub_nosysrel.txt" ;;
    mrfull)
      timeout -k 10 1100 python -u -m pytest tests/test_gpu_multirank.py -x -v -s -k full_size --timeout 540 --timeout-method thread > "$O/pytest_mrfull.log" 2>&1
      rc=$?; echo "pytest mrfull rc=$rc"; grep -E "emitted per query|PASS|FAIL|Error|passed|failed" "$O/pytest_mrfull.log" | tail -12; [ $rc -eq 0 ] || exit $rc ;;
    mr)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_multirank.py -x -v -k "not full_size" --timeout 200 --timeout-method thread > "$O/pytest_mr.log" 2>&1
      rc=$?; echo "pytest mr rc=$rc"; tail -12 "$O/pytest_mr.log"; [ $rc -eq 0 ] || exit $rc ;;
    stamps)
      for rows in 10000000 1250000; do
        BSR_LIB=tools/ab/libbsr_fstamps.so run 240 "stamps $rows" "$O/stamps_$rows.txt" python tools/diag/filter_stamps.py $rows
        grep -v amdgpu.ids "$O/stamps_$rows.txt"
      done ;;
    counters)
      for rows in 10000000 1250000; do
        BSR_LIB=tools/ab/libbsr_counters.so run 240 "counters $rows" "$O/counters_$rows.txt" python tools/diag/filter_counters.py $rows
        cat "$O/counters_$rows.txt"
        BSR_LIB=tools/ab/libbsr_counters.so run 240 "wg balance $rows" "$O/wg_$rows.txt" python tools/diag/filter_wg_balance.py $rows
        cat "$O/wg_$rows.txt"
      done ;;
    fab)
      run 300 "filter_ab 10M" "$O/fab_10m.txt" tools/microbench/filter_ab 10000000 1000 10 0.1473; cat "$O/fab_10m.txt"
      run 200 "filter_ab 1.25M" "$O/fab_125.txt" tools/microbench/filter_ab 1250000 1000 30 0.1284; cat "$O/fab_125.txt" ;;
    fabshard)
      for rows in 5000000 2500000 1250000; do
        run 300 "filter_ab $rows" "$O/fab_$rows.txt" tools/microbench/filter_ab $rows 1000 20 0.1473
        grep -E "emitted|median" "$O/fab_$rows.txt"
      done ;;
    fabpmc)
      for rows in 10000000 1250000; do
        run 300 "filter_ab pmc $rows" /dev/null rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/fabpmc_$rows" -o run -- \
            tools/microbench/filter_ab $rows 1000 2 0.1473
        python3 tools/microbench/pmc_summary.py "$O/fabpmc_$rows" > "$O/fabpmc_$rows.txt"; grep -A2 "qs16" "$O/fabpmc_$rows.txt"
      done ;;
    ab:*|ab125:*|abc2:*|abc5:*)
      extra=""
      case "${step%%:*}" in
        ab125) extra="--rows 1250000 --steps 50" ;;
        abc2) extra="--config c2 --steps 30" ;;
        abc5) extra="--config c5 --steps 5 --warmup 2" ;;
      esac
      for r in 1 2; do
        for v in $(echo "${step#*:}" | tr , ' '); do
          if [ "$v" = new ]; then L=""; else L="tools/ab/libbsr_$v.so"; fi
          BSR_LIB=$L run 200 "${step%%:*} $v $r" "$O/${step%%:*}_${v}_$r.json" python bench.py --steps 30 --warmup 5 \
              --verify 0 --p50-iters 5 $NOB $extra
          python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'], d['emitted_per_query_rank0'])" \
              "$O/${step%%:*}_${v}_$r.json" "$v"
        done
      done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
