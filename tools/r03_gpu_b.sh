#!/bin/bash
# round 3: pre-draw parity, reward-model fit timing + rocprofv3 summary, drop-in breakdown
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_mt.py \
  > gpurun_out/r03_mt.log 2>&1 &&
bash tools/r03_fit_bench.sh
