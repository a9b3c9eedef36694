#!/bin/bash
# Team kernel with the fused policy / reward net: its tests, then the run.sh recipe A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_reward.py tests/test_gpu_parity.py tests/test_gpu_team.py \
    -k "team" -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_team_pr.log 2>&1
rc=$?; grep -E "PASS|FAIL|ERROR|max\|" gpurun_out/pytest_team_pr.log | tail -40; [ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_team_pr.log; exit $rc; }
SKIP_TESTS=1 WLS="runsh_recipe" STEPS=100 bash tools/team_round.sh
