#!/bin/bash
# round 4: PP wave priorities (C segment ahead of the MFMA segment) -- tests, stamps, A/B vs variants
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v -s --timeout 120 --timeout-method thread tests/test_gpu_f16.py -k "pp" \
  > gpurun_out/r04_ppprio_tests.log 2>&1 || { tail -30 gpurun_out/r04_ppprio_tests.log; exit 1; }
tail -2 gpurun_out/r04_ppprio_tests.log
BCMPC_LIB=$PWD/build/variants/libbcmpc_stamp.so BCMPC_X3_STAMPS=1 timeout -k 10 120 \
  python -u tools/f16_ab.py --rounds 1 --steps 3 --warmup 1 pp > gpurun_out/r04_ppprio_stamps.log 2>&1 || exit 1
grep "x3 stamps" gpurun_out/r04_ppprio_stamps.log | tail -2
for r in 0 1; do
  for v in default prio0 prio1 prioME pg1d4 pg1d5 pg1d6; do
    if [ $v = default ]; then L=""; else L=$PWD/build/variants/libbcmpc_$v.so; fi
    BCMPC_LIB=$L timeout -k 10 200 python -u tools/f16_ab.py --rounds 1 pp 2>/dev/null | sed "s/^{/{\"lib\": \"$v\", /" \
      >> gpurun_out/r04_ppprio_ab.jsonl || exit 1
  done
done
cat gpurun_out/r04_ppprio_ab.jsonl
