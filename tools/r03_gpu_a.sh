#!/bin/bash
# round 3: team kernel with the reference's control configurations (policy over relu+LN, LN reward net)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread \
  tests/test_gpu_reward.py tests/test_gpu_team.py "$@" > gpurun_out/r03_a.log 2>&1
