#!/bin/bash
set -o pipefail
rm -f gpurun_out/r04_p2sched_ab.jsonl
for r in 0 1; do
  for v in default p2_iterative-maxocc p2_iterative-minreg p2_max-occupancy; do
    if [ $v = default ]; then L=""; else L=$PWD/build/variants/libbcmpc_$v.so; fi
    BCMPC_LIB=$L timeout -k 10 200 python -u tools/f16_ab.py --rounds 1 pp 2>/dev/null | sed "s/^{/{\"lib\": \"$v\", /" >> gpurun_out/r04_p2sched_ab.jsonl || exit 1
  done
done
cat gpurun_out/r04_p2sched_ab.jsonl
