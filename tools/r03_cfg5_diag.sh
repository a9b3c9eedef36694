#!/bin/bash
# cfg5 pass timing with diagnostic weight streams (results wrong; timing only): in-tree build vs
# L1-resident weights (smallw), hi-only fragments (hionly: half the bytes), no weight loads (noloads).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VARS:-nw8 smallw hionly noloads}; do
    BCMPC_LIB=$PWD/build/variants/libbcmpc_$v.so timeout -k 10 300 python bench.py --workload cfg5_pass --steps 5 --warmup 2 \
        --no-cpu-baseline > gpurun_out/cfg5_d_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v bench rc=$rc"; tail -3 gpurun_out/cfg5_d_$v.log; exit $rc; }
    python - "$v" gpurun_out/cfg5_d_$v.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().split('\n')[-1])
print(f"{sys.argv[1]:10s} kernel_ms={d['kernel_ms_avg']:.3f} frac_equiv={d['roofline']['frac']:.3f}")
PY
  done
done
