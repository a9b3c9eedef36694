#!/bin/bash
# Bench a list of workloads (WLS) at the given precision (PREC, default auto); one line each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WLS:-cfg2 cfg3 cfg4_shard cfg5}; do
  timeout -k 10 300 python bench.py --workload "$wl" --precision "${PREC:-auto}" --steps ${STEPS:-10} --warmup 2 \
      --no-cpu-baseline ${BENCH_ARGS:-} > "gpurun_out/wl_$wl.log" 2>&1
  rc=$?
  if [ $rc -ne 0 ]; then echo "$wl rc=$rc"; tail -3 "gpurun_out/wl_$wl.log"; exit $rc; fi
  python - "$wl" "gpurun_out/wl_$wl.log" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().split('\n')[-1])
print(f"{sys.argv[1]:12s} {d['dtype'][:20]:20s} value={d['value']:.4g} kernel_ms={d['kernel_ms_avg']:.3f} "
      f"frac={d['roofline']['frac']:.3f} p50={d['p50_ms']:.3f} kernel={d['roofline']['kernel'][:40]}")
PY
done
