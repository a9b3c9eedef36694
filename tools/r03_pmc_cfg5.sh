#!/bin/bash
# the cfg5 pass's weight stream under PMC, per library variant in $VARS (build/variants/,
# "tree" = the in-tree build): MFMA busy, L1 -> L2 read requests (128 B), L2 hit / miss.  One rocprofv3
# --pmc run per pass under a KILL timeout; summary by tools/pmc_summary.py.
set -u
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/r03_pmc_cfg5
mkdir -p "$OUT"
for v in ${VARS:-tree}; do
  if [ "$v" = tree ]; then L=$R/bc_mpc_amd/libbcmpc.so; else L=$R/build/variants/libbcmpc_$v.so; fi
  i=0
  for counters in "GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES" \
                  "GRBM_GUI_ACTIVE TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
                  "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum"; do
    i=$((i+1))
    BCMPC_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $counters --output-format csv -d "$OUT/${v}_p$i" -o run -- \
        python3 "$R/bench.py" --workload cfg5_pass --steps 3 --warmup 1 --no-cpu-baseline --no-small-k --dropin-calls 0 \
        > "$OUT/${v}_p$i.log" 2>&1
    rc=$?
    echo "$v pass $i rc=$rc"
    [ $rc -ne 0 ] && { tail -5 "$OUT/${v}_p$i.log"; exit $rc; }
  done
done
python3 "$R/tools/pmc_summary.py" "$OUT" rollout_x3 > "$OUT/summary.txt" && cat "$OUT/summary.txt"
