#!/bin/bash
# round 4: where the team exchange goes -- TEAM_STAMP=3 realtime probes (member skew, hand-off latency)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$PWD}"
mkdir -p gpurun_out/r04_team_xchg2
for spec in "runsh_recipe:8" "cfg1:4"; do
  wl=${spec%%:*}; T=${spec#*:}
  rm -f gpurun_out/r04_team_xchg2/$wl.bin
  BCMPC_LIB=$PWD/build/variants/libbcmpc_rt3.so BCMPC_X3_STAMPS=1 BCMPC_STAMP_DUMP=$PWD/gpurun_out/r04_team_xchg2/$wl.bin \
    timeout -k 10 120 python bench.py --workload $wl --steps 3 --warmup 2 --no-cpu-baseline --no-small-k --dropin-calls 0 \
    > gpurun_out/r04_team_xchg2/$wl.log 2>&1 || { tail -5 gpurun_out/r04_team_xchg2/$wl.log; exit 1; }
  echo "== $wl"; grep "team stamps" gpurun_out/r04_team_xchg2/$wl.log | tail -1
  python tools/team_xchg_stamps.py gpurun_out/r04_team_xchg2/$wl.bin $T || exit 1
done
