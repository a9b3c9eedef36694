#!/bin/bash
# GPU box: the NumPy-stream drop-in tests, then the drop-in latency bench (serial vs jump-ahead draw).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -q -s -p no:cacheprovider --timeout 120 \
    --timeout-method thread -k "dropin" > gpurun_out/pytest_dropin.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_dropin.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/bench_dropin.py > gpurun_out/bench_dropin.log 2>&1 || exit $?
cat gpurun_out/bench_dropin.log
