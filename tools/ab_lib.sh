#!/bin/bash
# A/B one workload between the in-tree library and a variant (BCMPC_LIB=$1), alternating runs.
# usage: tools/ab_lib.sh build/libbcmpc_x.so workload [steps]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
V=$1; WL=$2; N=${3:-200}
for r in 1 2; do
  for lib in base "$V"; do
    if [ "$lib" = base ]; then unset BCMPC_LIB; else export BCMPC_LIB=$PWD/$lib; fi
    timeout -k 10 200 python bench.py --workload "$WL" --steps "$N" --warmup 20 --no-cpu-baseline --dropin-calls 0 \
        > gpurun_out/ab_$r.log 2>&1 || { echo "$lib failed"; tail -5 gpurun_out/ab_$r.log; exit 1; }
    python - "$lib" gpurun_out/ab_$r.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print(f"{sys.argv[1]:32s} p50 {d['p50_ms']:.4f} ms  kernel {d['kernel_ms_avg']:.4f} ms  value {d['value']:.4g}")
PY
  done
done
