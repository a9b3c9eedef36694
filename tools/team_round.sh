#!/bin/bash
# Team kernel (rollout_team.hip) on the box: its tests + the parity fixtures, then the small-K
# workloads with the team kernel (auto) against the slab kernel (BCMPC_TEAM=0), p50 and kernel time.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 400 python -u -m pytest tests/test_gpu_team.py tests/test_gpu_parity.py -k "team or dropin" -x -v \
        -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_team.log 2>&1
    rc=$?; grep -E "PASS|FAIL|ERROR|SKIP|max\|" gpurun_out/pytest_team.log | tail -60; [ $rc -eq 0 ] || exit $rc
fi
for wl in ${WLS:-ppo_defaults cfg1 cfg2}; do
    for team in 1 0 1 0; do
        BCMPC_TEAM=$team timeout -k 10 120 python bench.py --workload $wl --steps ${STEPS:-200} --warmup 20 \
            --no-cpu-baseline --dropin-calls 0 > gpurun_out/bench_${wl}_team$team.log 2>&1 || { tail -5 gpurun_out/bench_${wl}_team$team.log; exit 1; }
        python - "$wl" "$team" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/bench_{sys.argv[1]}_team{sys.argv[2]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(f"{sys.argv[1]:14s} team={sys.argv[2]} p50_ms {d['p50_ms']:.4f} kernel_ms {d['kernel_ms_avg']:.4f} "
      f"value {d['value']:.3e} kernel {d['roofline'].get('kernel')}")
PY
    done
done
