#!/bin/bash
# round 4: the next call's rows drawn from the launch on (early pre-draw post) + the team engines' 2^18 host
# bound: NumPy-stream / drop-in tests, then the drop-in A/B (old bound 2^16 = device draw for cfg1)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 150 --timeout-method thread tests/test_gpu_mt.py \
  tests/test_gpu_dropin_soak.py tests/test_gpu_team_progress.py tests/test_gpu_team.py tests/test_gpu_reward.py \
  > gpurun_out/r04_gpu_c_tests.log 2>&1 || { tail -40 gpurun_out/r04_gpu_c_tests.log; exit 1; }
tail -2 gpurun_out/r04_gpu_c_tests.log
timeout -k 10 400 python -u tools/dropin_zc_ab.py --rounds 2 "new:" "zc16:BCMPC_MT_ZC_WORDS=65536" > gpurun_out/r04_dropin_zc_ab.jsonl 2>&1
cat gpurun_out/r04_dropin_zc_ab.jsonl
