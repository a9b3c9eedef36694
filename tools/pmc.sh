#!/bin/bash
# rocprofv3 PMC passes (each in its own run, --pmc only) over a short bench.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc
mkdir -p "$OUT"
i=0
while read -r counters; do
  [ -z "$counters" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $counters --output-format csv -d "$OUT/p$i" -o run -- \
      python3 "$R/bench.py" --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline ${BENCH_ARGS:-} > "$OUT/p$i.log" 2>&1
  rc=$?
  echo "pass $i ($counters) rc=$rc"
  [ $rc -ne 0 ] && { tail -5 "$OUT/p$i.log"; exit $rc; }
done <<LIST
${PASSES:-GRBM_GUI_ACTIVE GRBM_COUNT SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES
FETCH_SIZE
WRITE_SIZE
SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR SQ_WAVES}
LIST
