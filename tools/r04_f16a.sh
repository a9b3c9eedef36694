#!/bin/bash
# round 4: single-pass f16 layouts (hi-only slab: NC=8 / two 4-wave groups per CU) -- tests, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_f16.py \
  > gpurun_out/r04_f16a_tests.log 2>&1 || exit $?
for lay in "4,4" "4,8"; do
  BCMPC_F16_NC=${lay%,*} BCMPC_F16_NW=${lay#*,} timeout -k 10 200 python -u -m pytest -x -v -s --timeout 120 \
    --timeout-method thread tests/test_gpu_f16.py -k "full_size" > gpurun_out/r04_f16a_tests_$lay.log 2>&1 || exit $?
done
timeout -k 10 300 python -u tools/f16_ab.py --rounds 2 0,0 4,8 8,8 4,4 > gpurun_out/r04_f16a_ab.jsonl 2>&1
