#!/bin/bash
# Round 6: the north_star's per-GPU shard sizes on one card (K = 65536 / N for N = 1, 2, 4, 8), lean bench lines
# (prewarm, 10 warmup, 100 timed steps): the inputs of DESIGN.md §7's projected strong-scaling curve.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for wl in cfg3 cfg4_shard k16384 ns_shard; do
    timeout -k 10 200 python bench.py --workload $wl --steps 100 --warmup 10 --no-cpu-baseline --no-small-k --no-cfg2 \
        --no-f16 --no-extra --no-scale --dropin-calls 0 > gpurun_out/shard_sweep.log 2>&1 || { tail -5 gpurun_out/shard_sweep.log; exit 1; }
    python - $wl <<'PY'
import json, sys
d = json.loads([x for x in open("gpurun_out/shard_sweep.log") if x.startswith("{")][-1])
print(f"{sys.argv[1]:11s} K {d['config']['K_per_gpu']:6d}  p50 {d['p50_ms']:.4f} ms  ms/step {d['ms_per_step']:.4f}  kernel {d['kernel_ms_avg']:.4f} ms  "
      f"value {d['value']:.4g}  frac {d['roofline']['frac']:.3f}  {d['roofline']['kernel'][:40]}", flush=True)
PY
  done
done
