#!/bin/bash
# round 3: zero-copy rows cost in-kernel, then the pre-draw device-copy A/B (BCMPC_MT_PREDRAW_DEV), ppo_defaults
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r03_devcopy_ab.txt
: > $out
timeout -k 10 200 python tools/zc_kernel_time.py ppo_defaults 300 2>/dev/null >> $out || exit 1
BCMPC_MT_PREDRAW_DEV=1 timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 120 --timeout-method thread \
  tests/test_gpu_dropin_soak.py tests/test_gpu_mt.py >> $out 2>&1 || exit 1
for i in 1 2; do
  for dv in 0 1; do
    echo "dev=$dv run=$i" >> $out
    BCMPC_MT_PREDRAW_DEV=$dv timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 2>/dev/null >> $out || exit 1
  done
done
