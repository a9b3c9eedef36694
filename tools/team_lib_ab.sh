#!/bin/bash
# A/B of team-kernel variant libraries (LIBS: base = in-tree, else build/variants/libbcmpc_<name>.so)
# on small-K workloads (WLS), after the team tests on each library.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for lib in ${LIBS:-base}; do
    if [ $lib = base ]; then L=$PWD/bc_mpc_amd/libbcmpc.so; else L=$PWD/build/variants/libbcmpc_$lib.so; fi
    BCMPC_LIB=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_team.py tests/test_gpu_parity.py -k "team" -x -q \
        -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_ab_$lib.log 2>&1
    rc=$?; echo "$lib: $(tail -1 gpurun_out/pytest_ab_$lib.log)"; [ $rc -eq 0 ] || exit $rc
done
for wl in ${WLS:-ppo_defaults}; do
  for lib in ${LIBS:-base} ${LIBS:-base}; do
    if [ $lib = base ]; then L=$PWD/bc_mpc_amd/libbcmpc.so; else L=$PWD/build/variants/libbcmpc_$lib.so; fi
    BCMPC_LIB=$L timeout -k 10 120 python bench.py --workload $wl --steps 300 --warmup 20 --no-cpu-baseline \
        --no-small-k --dropin-calls 0 > gpurun_out/libab_$lib.log 2>&1 || { tail -5 gpurun_out/libab_$lib.log; exit 1; }
    python - "$wl" "$lib" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/libab_{sys.argv[2]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[1]:14s} {sys.argv[2]:8s} p50_ms {d['p50_ms']:.4f} kernel_ms {d['kernel_ms_avg']:.4f}")
PY
  done
done
