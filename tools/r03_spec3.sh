#!/bin/bash
# round 3: speculative draw beside the rollout (slab engines) -- tests, then A/B at cfg1 and cfg3
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -v -s --timeout 200 --timeout-method thread tests/test_gpu_mt.py \
  tests/test_gpu_parity.py tests/test_gpu_workloads.py -k "speculative or device_draw or stream or dropin or cfg4 or failed" \
  > gpurun_out/r03_spec3_tests.log 2>&1 || exit 1
: > gpurun_out/r03_spec3_ab.txt
for r in 1 2; do
  for sp in 0 1; do
    for wl in cfg2 cfg3; do
      echo "speculate=$sp run=$r $wl" >> gpurun_out/r03_spec3_ab.txt
      BCMPC_MT_SPECULATE=$sp timeout -k 10 200 python tools/dropin_breakdown.py $wl 100 \
        >> gpurun_out/r03_spec3_ab.txt 2>/dev/null || exit 1
    done
  done
done
