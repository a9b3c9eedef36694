#!/bin/bash
# A/B one library under several environment settings, alternating rounds (same session, same box).
# usage: tools/ab_env.sh workload steps "NAME=VAL ..." "NAME=VAL ..." ...   ("-" = no extra variables)
#   env: ROUNDS (default 2), AB_ARGS (extra bench.py arguments)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WL=$1; N=$2; shift 2
for r in $(seq 1 ${ROUNDS:-2}); do
  for vars in "$@"; do
    ev=""; [ "$vars" != "-" ] && ev="$vars"
    env $ev timeout -k 10 200 python bench.py --workload "$WL" --steps "$N" --warmup 5 --no-cpu-baseline \
        --no-small-k --no-cfg2 --no-f16 --no-extra --dropin-calls 0 ${AB_ARGS:-} > gpurun_out/ab_env.log 2>&1 \
        || { echo "[$vars] failed"; tail -5 gpurun_out/ab_env.log; exit 1; }
    python - "$vars" gpurun_out/ab_env.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print(f"{sys.argv[1]:28s} p50 {d['p50_ms']:.4f} ms  kernel {d['kernel_ms_avg']:.4f} ms  value {d['value']:.4g}  "
      f"frac {d['roofline']['frac']:.3f}  {d['roofline']['kernel'][:60]}", flush=True)
PY
  done
done
