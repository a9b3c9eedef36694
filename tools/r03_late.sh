#!/bin/bash
# round 3: late pre-draw hits (the team kernel waits for the worker's rows word) -- tests, then A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -m gpu -v -s --timeout 200 --timeout-method thread tests/test_gpu_mt.py \
  tests/test_gpu_dropin_soak.py tests/test_gpu_parity.py -k "predraw or late or soak or dropin or fast_path or zero_copy" \
  > gpurun_out/r03_late_tests.log 2>&1 || exit 1
: > gpurun_out/r03_late_ab.txt
for r in 1 2; do
  for late in 0 1; do
    echo "late=$late run=$r" >> gpurun_out/r03_late_ab.txt
    BCMPC_MT_PREDRAW_LATE=$late timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 \
      >> gpurun_out/r03_late_ab.txt 2>/dev/null || exit 1
  done
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f16 --dropin-calls 0 \
  > gpurun_out/r03_late_bench.json 2>/dev/null
