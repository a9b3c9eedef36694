#!/bin/bash
# round 3: the team kernel's fused argmin tail -- team tests, then the small-K lines with the tail on / off (A/B/A/B)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_team.py \
  tests/test_gpu_team_progress.py tests/test_gpu_dropin_soak.py tests/test_gpu_mt.py tests/test_gpu_reward.py \
  tests/test_gpu_mcts.py tests/test_gpu_multirank.py > gpurun_out/r03_team_fused_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -m gpu -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "team" >> gpurun_out/r03_team_fused_tests.log 2>&1 || exit 1
out=gpurun_out/r03_team_fused_ab.txt
: > $out
for i in 1 2; do
  for f in 0 1; do
    echo "team_fused=$f run=$i" >> $out
    BCMPC_TEAM_FUSED_ARGMIN=$f timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-f16 \
      --dropin-calls 0 2>/dev/null >> $out || exit 1
  done
done
