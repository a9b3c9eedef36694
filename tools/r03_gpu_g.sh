#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_mt.py tests/test_gpu_reward.py tests/test_gpu_parity.py -k "mt or dropin or stream or policy" > gpurun_out/r03_g.log 2>&1 &&
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dropin-calls 10 > gpurun_out/r03_smallk.json 2> gpurun_out/r03_smallk.err
