#!/bin/bash
# Phase stamps of the team kernel (TEAM_STAMP variant, tools/team_variants.sh "tstamp:-DTEAM_STAMP=1")
# for the small-K workloads, one stamped get_action each after warm-up.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in ${WLS:-ppo_defaults cfg1}; do
    echo "== $wl"
    BCMPC_LIB=$PWD/build/variants/libbcmpc_tstamp.so BCMPC_X3_STAMPS=1 timeout -k 10 120 python bench.py --workload $wl \
        --steps 3 --warmup 2 --no-cpu-baseline --no-small-k --dropin-calls 0 > gpurun_out/tstamp_$wl.log 2>&1 || { tail -5 gpurun_out/tstamp_$wl.log; exit 1; }
    grep "team stamps" gpurun_out/tstamp_$wl.log | tail -2
done
