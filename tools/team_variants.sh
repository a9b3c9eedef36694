#!/bin/bash
# Build A/B or diagnostic variants of the team kernel (rollout_team.hip) into
# build/variants/libbcmpc_<name>.so (selected at run time via BCMPC_LIB).
# usage: tools/team_variants.sh "name:-DFLAG=1 ..." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -DBCMPC_DIAG_VARIANT"
make -s -j8 ARCH=gfx950 >/dev/null
OBJS="build/rollout.o build/rollout_grp.o build/rollout_x3.o build/rollout_x3_plain.o build/cem.o build/fit.o build/mt19937.o build/mt_jump.o build/mt_device.o build/comm.o"
# capi.cpp is rebuilt with each variant's flags: the host weight packing and the kernel must agree on the
# compile-time switches they share (TEAM_DEFER: the output layer packed for the deferred LayerNorm or not)
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( $H ${TEAMSCHED:--mllvm -amdgpu-sched-strategy=iterative-ilp} $flags -c bc_mpc_amd/csrc/rollout_team.hip -o build/variants/rollout_team_$name.o &&
    $H $flags -x hip -c bc_mpc_amd/csrc/capi.cpp -o build/variants/capi_team_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/variants/libbcmpc_$name.so $OBJS \
        build/variants/capi_team_$name.o build/variants/rollout_team_$name.o -ldl ) &
done
wait
ls build/variants/*.so
