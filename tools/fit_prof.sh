#!/bin/bash
# Fused vs per-op fit iteration: bench_fit wall time for both, then a kernel-trace of the fused run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_fit.py --cpu-iters 1 > gpurun_out/fit_fused.log 2>&1 || exit $?
BCMPC_FIT_FUSED=0 timeout -k 10 120 python tools/bench_fit.py --cpu-iters 1 > gpurun_out/fit_perop.log 2>&1 || exit $?
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/fitprof -o fit -- \
    python tools/bench_fit.py --cpu-iters 1 --reps 2 > gpurun_out/fit_prof.log 2>&1 || exit $?
tail -1 gpurun_out/fit_fused.log; tail -1 gpurun_out/fit_perop.log
find gpurun_out/fitprof -name '*kernel_stats.csv' -exec cat {} \;
