#!/bin/bash
# round 3: the policy controllers' batched seed stream -- every policy / reward / MCTS / multi-rank GPU test,
# then the small-K bench lines
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -v -s --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_reward.py tests/test_gpu_mcts.py tests/test_gpu_multirank.py tests/test_gpu_team_progress.py \
  tests/test_gpu_mt.py -k "policy or reward or mcts or polrew or ranks or stochastic or progress or fast_path" \
  > gpurun_out/r03_seedstream_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f16 --dropin-calls 0 \
  > gpurun_out/r03_seedstream_bench.json 2>/dev/null
