#!/bin/bash
# Drop-in (NumPy stream) p50 per workload: the device MT draw vs the host draw (BCMPC_MT_PATH=host).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WLS:-ppo_defaults cfg1 cfg2 cfg3}; do
  for path in device host; do
    if [ $path = host ]; then export BCMPC_MT_PATH=host; else unset BCMPC_MT_PATH; fi
    timeout -k 10 200 python bench.py --workload "$wl" --steps 50 --warmup 5 --no-cpu-baseline --dropin-calls 100 \
        > gpurun_out/dp_${wl}_${path}.log 2>&1 || { echo "$wl $path failed"; tail -3 gpurun_out/dp_${wl}_${path}.log; exit 1; }
    python - "$wl" "$path" gpurun_out/dp_${wl}_${path}.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[3]) if x.startswith("{")][-1])
print(f"{sys.argv[1]:14s} {sys.argv[2]:7s} get_action p50 {d['p50_ms']:.4f} ms  drop-in p50 {d['dropin_parity_p50_ms']:.4f} ms")
PY
  done
done
