#!/bin/bash
# A/B several library builds (BCMPC_LIB) on one workload, alternating rounds; "tree" = the in-tree library.
# usage: tools/ab_libs.sh workload steps lib1 lib2 ...   (env ROUNDS, default 2; KERNEL: BCMPC_KERNEL;
#        AB_ARGS: extra bench.py arguments, e.g. "--precision f16"; AB_SMALLK=1: the small-K lines too,
#        their p50 / kernel ms printed)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
WL=$1; N=$2; shift 2
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "$@"; do
    if [ "$lib" = tree ]; then unset BCMPC_LIB; else export BCMPC_LIB=$PWD/$lib; fi
    env ${KERNEL:+BCMPC_KERNEL=$KERNEL} timeout -k 10 200 python bench.py --workload "$WL" --steps "$N" --warmup 10 \
        --no-cpu-baseline $([ -n "${AB_SMALLK:-}" ] || echo --no-small-k) --no-cfg2 --no-f16 --no-extra --dropin-calls 0 ${AB_ARGS:-} > gpurun_out/ab_libs.log 2>&1 \
        || { echo "$lib failed"; tail -5 gpurun_out/ab_libs.log; exit 1; }
    python - "$lib" gpurun_out/ab_libs.log <<'PY'
import json, sys
d = json.loads([x for x in open(sys.argv[2]) if x.startswith("{")][-1])
print(f"{sys.argv[1]:36s} p50 {d['p50_ms']:.4f} ms  kernel {d['kernel_ms_avg']:.4f} ms  value {d['value']:.4g}", flush=True)
for k, v in (d.get("small_k") or {}).items():
    print(f"    {k:18s} p50 {v['p50_ms'] * 1e3:7.2f} us  kernel {v['kernel_ms'] * 1e3:7.2f} us  drop-in {v.get('dropin_parity_p50_ms', 0) * 1e3:7.2f} us", flush=True)
PY
  done
done
