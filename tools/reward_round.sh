#!/bin/bash
# Parity tests (all GPU tests) + A/B of the group layouts on several workloads.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
    rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
    case $rc in 0|1) ;; *) exit $rc ;; esac
fi
for wl in ${WORKLOADS:-cfg3 cfg3_reward cfg3_polrew runsh_recipe}; do
    for k in ${KERNELS:-group4 group8}; do
        BENCH_ARGS="--workload $wl" KERNELS=$k bash tools/ab_kernels.sh | sed "s/^/$wl /" || exit $?
    done
done
