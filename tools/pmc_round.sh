#!/bin/bash
# PMC passes for the default kernel: SQ utilisation + HBM traffic (hbm vs device-RNG actions).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/pmc2
mkdir -p "$OUT"
pass() {  # name, bench args, counters...
  local name=$1 args=$2; shift 2
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline $args > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
pass sq_cfg3 "" GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU
pass fetch_hbm "" FETCH_SIZE
pass fetch_dev "--actions device" FETCH_SIZE
pass write_hbm "" WRITE_SIZE
pass sq_cfg2 "--workload cfg2" GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU
