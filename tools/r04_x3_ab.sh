#!/bin/bash
# round 4: a rollout_x3 change against build/variants/libbcmpc_x3old.so (the previous commit's kernel source):
# the split-kernel parity tests, then cfg3 / cfg2 A/B, two alternating rounds
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_workloads.py tests/test_gpu_f16.py > gpurun_out/r04_x3_ab_tests.log 2>&1 || { tail -30 gpurun_out/r04_x3_ab_tests.log; exit 1; }
tail -1 gpurun_out/r04_x3_ab_tests.log
rm -f gpurun_out/r04_x3_ab.jsonl
for r in 0 1; do
  for v in new ${VARIANTS:-x3old}; do
    if [ $v = new ]; then L=""; else L=$PWD/build/variants/libbcmpc_$v.so; fi
    for wl in cfg3 cfg2; do
      BCMPC_LIB=$L timeout -k 10 300 python bench.py --workload $wl --steps 40 --warmup 5 --no-cpu-baseline --no-small-k \
        --no-f16 --no-cfg2 --dropin-calls 0 2>/dev/null | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(json.dumps({'lib': '$v', 'round': $r, 'wl': '$wl', 'p50_ms': round(d['p50_ms'], 4), 'kernel_ms': round(d['kernel_ms_avg'], 4), 'frac': round(d['roofline']['frac'], 4)}))
" >> gpurun_out/r04_x3_ab.jsonl || exit 1
    done
  done
done
cat gpurun_out/r04_x3_ab.jsonl
