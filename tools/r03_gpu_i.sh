#!/bin/bash
# round 3: the drop-in fast-path tests, the drop-in breakdown (ppo_defaults), then the whole GPU suite
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread tests/test_gpu_parity.py \
  -k "dropin or fast_path" > gpurun_out/r03_fastpath_tests.log 2>&1 &&
timeout -k 10 300 python tools/dropin_breakdown.py ppo_defaults 400 > gpurun_out/r03_dropin_breakdown_fast.json 2>&1 &&
timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests \
  > gpurun_out/r03_full.log 2>&1
