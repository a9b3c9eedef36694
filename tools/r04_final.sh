#!/bin/bash
# round 4 validation at head: the whole GPU suite, smoke(), the default bench line, rocprofv3 of the same
# command, and the pipelined f16 kernel's PMC (head counters + HBM traffic)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/r04_pmc_f16
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests \
  > gpurun_out/r04_final_pytest.log 2>&1 || { tail -40 gpurun_out/r04_final_pytest.log; exit 1; }
tail -1 gpurun_out/r04_final_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r04_final_bench.json 2> gpurun_out/r04_final_bench.err || exit 1
echo bench done
cd /tmp
pass() {  # name, bench args, counters...
  local name=$1 args=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/r04_pmc_f16/$name" -o run -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --dropin-calls 0 --no-small-k --no-f16 --no-cfg2 $args \
      > "$R/gpurun_out/r04_pmc_f16/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
pass p1_pp "--precision f16" GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU
pass p4_pp "--precision f16" TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum
pass fetch_pp "--precision f16" FETCH_SIZE
pass write_pp "--precision f16" WRITE_SIZE
cd "$R"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04_prof_final" -o run -- \
    python3 bench.py > gpurun_out/r04_final_bench_prof.json 2> gpurun_out/r04_final_bench_prof.err
echo "prof rc=$?"
