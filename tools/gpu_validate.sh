#!/bin/bash
# One parameterised GPU-box session (replaces the per-round one-off scripts r03_gpu_*, r04_final*):
#   STEPS  (space-separated, run in this order; any failure ends the script)
#     tests    pytest -m gpu over $TESTS (default: the whole suite)
#     smoke    __graft_entry__.smoke()
#     bench    python bench.py $BENCH_ARGS                       -> $OUT/bench.json
#     trace    rocprofv3 --kernel-trace --stats of the same bench   -> $OUT/trace/
#     timed    kernel trace of the headline's timed launches only   -> $OUT/trace_timed/
#     traffic  PMC FETCH_SIZE / WRITE_SIZE passes per workload      -> $OUT/traffic_*/
#     issue    PMC issue / wait / memory-path passes over $PMC_ARGS -> $OUT/pmc_*/
#     rehearse $RANKS-rank (default 2) gloo rehearsal of bench.py on the one card, the ranks started by bench.py --gpus N
#              itself (no WORLD_SIZE: its child torch.distributed.run)  -> $OUT/rehearsal.json
#     ab       tools/ab_libs.sh $AB_WL $AB_STEPS $AB_LIBS (AB_ARGS: extra bench arguments) -> $OUT/ab.txt
#   TAG    output directory gpurun_out/$TAG
# Every GPU step has its own time limit; the first failure (test failure included) stops the session.
set -u
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=${TAG:-r06}
OUT=$R/gpurun_out/$TAG
STEPS=${STEPS:-"tests smoke bench trace"}
TESTS=${TESTS:-tests}
BENCH_ARGS=${BENCH_ARGS:-}
PMC_ARGS=${PMC_ARGS:-"--precision f16"}
PMC_KERNEL=${PMC_KERNEL:-rollout_pp}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
cd "$R"
stop() { echo "stopping after $1 (rc=$2)"; exit "$2"; }
LITE="--no-cpu-baseline --dropin-calls 0 --no-small-k --no-f16 --no-cfg2 --no-extra --no-scale"

pmc_pass() {  # name, bench args, counters...
  local name=$1 args=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 $LITE $args > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pmc $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; stop "pmc $name" $rc; }
}

for step in $STEPS; do
  case $step in
    tests)
      timeout -k 10 1100 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread $TESTS \
          > "$OUT/pytest.log" 2>&1 || { tail -40 "$OUT/pytest.log"; stop tests 1; }
      tail -1 "$OUT/pytest.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || stop smoke $?
      cat "$OUT/smoke.log" ;;
    bench)
      timeout -k 10 600 python bench.py $BENCH_ARGS > "$OUT/bench.json" 2> "$OUT/bench.err" || stop bench $?
      echo "bench: $(head -c 300 "$OUT/bench.json")" ;;
    trace)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- \
          python3 bench.py $BENCH_ARGS > "$OUT/trace_bench.json" 2> "$OUT/trace_bench.err" || stop trace $? ;;
    timed)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_timed" -o run -- \
          python3 bench.py --steps 50 --warmup 5 $LITE $BENCH_ARGS > "$OUT/trace_timed.json" 2>&1 || stop timed $? ;;
    traffic)
      for wl in ${TRAFFIC_WL:-cfg3:split cfg3:f16 cfg2:split ns_shard:split cfg4_shard:split cfg5:split}; do
        w=${wl%%:*}; p=${wl##*:}
        pmc_pass "traffic_${w}_${p}_fetch" "--workload $w --precision $p" FETCH_SIZE
        pmc_pass "traffic_${w}_${p}_write" "--workload $w --precision $p" WRITE_SIZE
      done
      # (the FETCH_SIZE calibration: cfg3 with its f64 action tensor read from HBM)
      pmc_pass "traffic_cfg3_split_hbm_fetch" "--workload cfg3 --precision split --actions hbm" FETCH_SIZE
      python3 "$R/tools/traffic_json.py" "$OUT" "$OUT/traffic_per_launch.json" ;;
    issue)
      pmc_pass pmc_a "$PMC_ARGS" GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY \
          SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC
      pmc_pass pmc_b "$PMC_ARGS" SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU \
          SQ_INSTS_VALU_TRANS_F32 SQ_WAIT_INST_ANY SQ_WAIT_ANY
      pmc_pass pmc_c "$PMC_ARGS" SQ_VALU_MFMA_COEXEC_CYCLES SQ_ACTIVE_INST_VALU2 SQ_INST_CYCLES_VMEM_RD \
          SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT
      pmc_pass pmc_d "$PMC_ARGS" GRBM_GUI_ACTIVE TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum \
          TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum
      python3 "$R/tools/pmc_issue.py" "$OUT" "$PMC_KERNEL" ${PMC_CANDSTEPS:-1310720} > "$OUT/pmc_summary.txt" 2>&1 || true
      cat "$OUT/pmc_summary.txt" ;;
    rehearse)
      BCMPC_DIST_BACKEND=gloo BCMPC_BENCH_DEVICE=0 timeout -k 10 400 python bench.py --gpus ${RANKS:-2} --steps 5 \
          --warmup 1 --no-cpu-baseline $BENCH_ARGS > "$OUT/rehearsal.json" 2> "$OUT/rehearsal.err" || stop rehearse $?
      tail -c 600 "$OUT/rehearsal.json" ;;
    ab)
      ROUNDS=${ROUNDS:-2} AB_ARGS=${AB_ARGS:-} bash tools/ab_libs.sh ${AB_WL:-cfg3} ${AB_STEPS:-30} $AB_LIBS \
          > "$OUT/ab.txt" 2>&1 || { cat "$OUT/ab.txt"; stop ab 1; }
      cat "$OUT/ab.txt" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
