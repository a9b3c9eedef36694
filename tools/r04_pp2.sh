#!/bin/bash
# round 4: the pipelined single-pass kernel -- tests, stamps, A/B
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_f16.py -k "pp" \
  > gpurun_out/r04_pp_tests.log 2>&1 || { tail -30 gpurun_out/r04_pp_tests.log; exit 1; }
tail -2 gpurun_out/r04_pp_tests.log
BCMPC_LIB=$PWD/build/variants/libbcmpc_stamp.so BCMPC_X3_STAMPS=1 timeout -k 10 120 \
  python -u tools/f16_ab.py --rounds 1 --steps 3 --warmup 1 pp > gpurun_out/r04_pp_stamps.log 2>&1 || exit 1
grep "x3 stamps" gpurun_out/r04_pp_stamps.log | tail -2
timeout -k 10 300 python -u tools/f16_ab.py --rounds 2 4,4 pp > gpurun_out/r04_pp_ab.jsonl 2>&1
