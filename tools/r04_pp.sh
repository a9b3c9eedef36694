#!/bin/bash
# round 4: the two-group pipelined single-pass kernel (rollout_pp): tests, then A/B against the other layouts
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_f16.py -k "pp" \
  > gpurun_out/r04_pp_tests.log 2>&1 || { tail -30 gpurun_out/r04_pp_tests.log; exit 1; }
tail -3 gpurun_out/r04_pp_tests.log
timeout -k 10 300 python -u tools/f16_ab.py --rounds 2 0,0 4,8 4,4 pp > gpurun_out/r04_pp_ab.jsonl 2>&1
