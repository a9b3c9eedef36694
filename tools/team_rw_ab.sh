#!/bin/bash
# Reward-net team layouts (TEAM_RW_NWV 4 in-tree vs 8 variant) on the run.sh recipe, A/B/A/B, after
# the policy / reward team tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_reward.py tests/test_gpu_parity.py tests/test_gpu_team.py \
    -k "team" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_team_pr.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_team_pr.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" gpurun_out/pytest_team_pr.log | head; exit $rc; }
for lib in ${LIBS:-base rw8 base rw8}; do
    if [ $lib = base ]; then L=$PWD/bc_mpc_amd/libbcmpc.so; else L=$PWD/build/variants/libbcmpc_$lib.so; fi
    BCMPC_LIB=$L timeout -k 10 120 python bench.py --workload runsh_recipe --steps 100 --warmup 10 --no-cpu-baseline \
        --dropin-calls 0 > gpurun_out/rwab_$lib.log 2>&1 || { tail -5 gpurun_out/rwab_$lib.log; exit 1; }
    python - "$lib" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/rwab_{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(f"runsh {sys.argv[1]:6s} p50_ms {d['p50_ms']:.4f} kernel_ms {d['kernel_ms_avg']:.4f}")
PY
done
BCMPC_LIB=$PWD/build/variants/libbcmpc_tstamp.so BCMPC_X3_STAMPS=1 timeout -k 10 120 python bench.py --workload runsh_recipe \
    --steps 3 --warmup 2 --no-cpu-baseline --dropin-calls 0 > gpurun_out/tstamp_runsh.log 2>&1 && grep "team stamps" gpurun_out/tstamp_runsh.log | tail -1
