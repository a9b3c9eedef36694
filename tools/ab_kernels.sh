#!/bin/bash
# A/B the kernel layouts (BCMPC_KERNEL) and optional library variants on one GPU.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab_$name.log 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name rc=$rc"; tail -3 gpurun_out/ab_$name.log; exit $rc; fi
  python - "$name" gpurun_out/ab_$name.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().split('\n')[-1])
print(f"{sys.argv[1]:28s} value={d['value']:.4g} kernel_ms={d['kernel_ms_avg']:.3f} frac={d['roofline']['frac']:.3f} p50={d['p50_ms']:.3f}")
PY
}
for k in ${KERNELS:-solo group2 group4}; do run "$k" BCMPC_KERNEL=$k; done
for lib in ${VARIANTS:-}; do
  for k in ${VKERNELS:-group4}; do run "$(basename $lib .so)_$k" BCMPC_LIB=$PWD/$lib BCMPC_KERNEL=$k; done
done
