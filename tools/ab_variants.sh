#!/bin/bash
# A/B the libbcmpc variants in build/variants on one GPU (bench only, no CPU baseline).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${VARIANTS:-build/variants/libbcmpc_*.so}; do
  name=$(basename "$lib" .so)
  BCMPC_LIB=$PWD/$lib timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$name.log 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 gpurun_out/ab_$name.log; exit $rc; fi
  python - "$name" gpurun_out/ab_$name.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().split('\n')[-1])
print(f"{sys.argv[1]:24s} value={d['value']:.4g} kernel_ms={d['kernel_ms_avg']:.3f} frac={d['roofline']['frac']:.3f} p50={d['p50_ms']:.3f}")
PY
done
