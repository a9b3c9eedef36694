#!/bin/bash
# Synchronous get_action completion: spin on the argmin's mapped done word (default) against a
# stream synchronisation (BCMPC_SYNC=stream), small-K workloads, A/B/A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WLS:-ppo_defaults cfg1 runsh_recipe}; do
    for sync in spin stream spin stream; do
        BCMPC_SYNC=$sync timeout -k 10 120 python bench.py --workload $wl --steps ${STEPS:-300} --warmup 20 \
            --no-cpu-baseline --dropin-calls ${DROPIN:-50} > gpurun_out/sync_${wl}_$sync.log 2>&1 || { tail -5 gpurun_out/sync_${wl}_$sync.log; exit 1; }
        python - "$wl" "$sync" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/sync_{sys.argv[1]}_{sys.argv[2]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[1]:14s} {sys.argv[2]:6s} p50_ms {d['p50_ms']:.4f} kernel_ms {d['kernel_ms_avg']:.4f} "
      f"dropin_p50 {d.get('dropin_parity_p50_ms')} kernel {d['roofline'].get('kernel')}")
PY
    done
done
