#!/bin/bash
# round 4: HBM traffic per launch of the head kernels (FETCH_SIZE / WRITE_SIZE, one counter per pass) and a
# kernel-trace summary of the timed launches only (no drop-in / small-K / f16 / cfg2 launches in the run)
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/r04_traffic
mkdir -p "$OUT"
B="--steps 3 --warmup 1 --no-cpu-baseline --dropin-calls 0 --no-small-k --no-f16 --no-cfg2"
pass() {
  local name=$1 args=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/bench.py" $B $args > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
pass fetch_hbm "--precision split --actions hbm" FETCH_SIZE
pass fetch_dev "--precision split --actions device" FETCH_SIZE
pass write_dev "--precision split --actions device" WRITE_SIZE
pass f16_fetch_dev "--precision f16 --actions device" FETCH_SIZE
pass f16_write_dev "--precision f16 --actions device" WRITE_SIZE
pass cfg2_fetch_dev "--workload cfg2 --precision split --actions device" FETCH_SIZE
pass cfg2_write_dev "--workload cfg2 --precision split --actions device" WRITE_SIZE
# the timed launches alone: 5 warmup + 50 timed get_action launches, nothing else of the bench
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_timed" -o run -- \
    python3 "$R/bench.py" --steps 50 --warmup 5 --no-cpu-baseline --dropin-calls 0 --no-small-k --no-f16 --no-cfg2 \
    > "$OUT/trace_timed.log" 2>&1
echo "trace_timed rc=$?"
