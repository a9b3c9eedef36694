#!/bin/bash
# split-kernel session: parity (-k split) on the in-tree lib, then A/B of build/variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_cem.py -x -q -s --timeout 120 \
      --timeout-method thread -p no:cacheprovider -k "${TESTK:-split}" > gpurun_out/x3_pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed" gpurun_out/x3_pytest.log | tail -2
  [ $rc -le 1 ] || exit $rc
fi
BENCH_ARGS="--precision split ${BENCH_ARGS:-}" STEPS=${STEPS:-20} bash tools/ab_variants.sh
