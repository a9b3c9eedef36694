#!/bin/bash
# round 4: branch-free owner phase at hidden 1024 (X3_BF_MAXHP=1024 variant) -- cfg5 / cfg5_pass A/B
set -o pipefail
rm -f gpurun_out/r04_bf1024_ab.jsonl
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_cem.py > gpurun_out/r04_bf1024_tests.log 2>&1; tail -1 gpurun_out/r04_bf1024_tests.log
for r in 0 1; do
  for v in new bf1024; do
    if [ $v = new ]; then L=""; else L=$PWD/build/variants/libbcmpc_$v.so; fi
    for wl in cfg5_pass cfg5; do
      BCMPC_LIB=$L timeout -k 10 300 python bench.py --workload $wl --steps 5 --warmup 1 --no-cpu-baseline --no-small-k \
        --no-f16 --no-cfg2 --dropin-calls 0 2>/dev/null | python -c "
import json,sys
d=json.loads(sys.stdin.read().strip().splitlines()[-1])
print(json.dumps({'lib': '$v', 'round': $r, 'wl': '$wl', 'p50_ms': round(d['p50_ms'], 3), 'kernel_ms': round(d['kernel_ms_avg'], 3), 'frac': round(d['roofline']['frac'], 4)}))
" >> gpurun_out/r04_bf1024_ab.jsonl || exit 1
    done
  done
done
cat gpurun_out/r04_bf1024_ab.jsonl
