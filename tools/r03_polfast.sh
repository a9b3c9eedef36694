#!/bin/bash
# round 3: the policy controller's repeat-call fast path -- tests, then the small-K lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -m gpu -v -s --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "fast_path or dropin" > gpurun_out/r03_polfast_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f16 --dropin-calls 0 \
  > gpurun_out/r03_polfast_bench.json 2>/dev/null
