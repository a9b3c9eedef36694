#!/bin/bash
# round 4: the advisor fixes (reward fit aliasing, seed unread, team ordering, late hits under a
# communicator) and the collective give-up path
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v -s --timeout 150 --timeout-method thread \
  tests/test_gpu_comm.py tests/test_gpu_multirank.py tests/test_gpu_team_progress.py tests/test_gpu_fit.py \
  tests/test_gpu_f16.py tests/test_gpu_dropin_soak.py "$@" > gpurun_out/r04_gpu_a.log 2>&1
rc=$?; tail -5 gpurun_out/r04_gpu_a.log; exit $rc
