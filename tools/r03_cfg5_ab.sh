#!/bin/bash
# cfg5 (3x1024) split-kernel geometry A/B: 1024-wide parity tests per variant, then cfg5_pass A/B/A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in ${VARS:-nw8 nw16 nw16g2}; do
  L=$PWD/build/variants/libbcmpc_$v.so
  BCMPC_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_workloads.py -m gpu -q -x \
      -k "1024 or cfg5" -p no:cacheprovider --timeout 200 --timeout-method thread > gpurun_out/cfg5_t_$v.log 2>&1
  rc=$?; echo "$v tests rc=$rc: $(tail -1 gpurun_out/cfg5_t_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in ${VARS:-nw8 nw16 nw16g2}; do
    BCMPC_LIB=$PWD/build/variants/libbcmpc_$v.so timeout -k 10 300 python bench.py --workload cfg5_pass --steps 5 --warmup 2 \
        --no-cpu-baseline > gpurun_out/cfg5_b_$v.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "$v bench rc=$rc"; tail -3 gpurun_out/cfg5_b_$v.log; exit $rc; }
    python - "$v" gpurun_out/cfg5_b_$v.log <<'PY'
import json,sys
d=json.loads(open(sys.argv[2]).read().strip().split('\n')[-1])
print(f"{sys.argv[1]:10s} value={d['value']:.4g} kernel_ms={d['kernel_ms_avg']:.3f} frac={d['roofline']['frac']:.3f} kernel={d.get('kernel')}")
PY
  done
done
