#!/bin/bash
# PMC passes for the L2 -> CU weight-stream question (one rocprofv3 --pmc run per pass, each under a KILL timeout):
# MFMA busy / waits, L1 -> L2 read requests, L2 hits / misses, for the workloads in $WLS.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/pmc_l2
mkdir -p "$OUT"
for wl in ${WLS:-cfg3 cfg5_pass}; do
  i=0
  for counters in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
                  "GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
                  "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d "$OUT/${wl}_p$i" -o run -- \
        python3 "$R/bench.py" --workload $wl --steps 3 --warmup 1 --no-cpu-baseline --no-small-k --dropin-calls 0 \
        > "$OUT/${wl}_p$i.log" 2>&1
    rc=$?
    echo "$wl pass $i ($counters) rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$OUT/${wl}_p$i.log"; exit $rc; }
  done
done
