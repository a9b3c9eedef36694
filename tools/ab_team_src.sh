#!/bin/bash
# Build a team-kernel variant from another SOURCE file (e.g. an older revision of rollout_team.hip) into
# build/variants/libbcmpc_<name>.so (selected at run time via BCMPC_LIB).
# usage: tools/ab_team_src.sh name path/to/rollout_team_variant.hip
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
name=$1; src=$2
make -s -j8 ARCH=gfx950 >/dev/null
cp "$src" bc_mpc_amd/csrc/rollout_team_variant_tmp.hip
OBJS="build/rollout.o build/rollout_grp.o build/rollout_x3.o build/rollout_x3_plain.o build/rollout_rr.o build/cem.o build/fit.o build/capi.o build/mt19937.o build/mt_jump.o build/mt_device.o build/comm.o"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
    -c bc_mpc_amd/csrc/rollout_team_variant_tmp.hip -o build/variants/rollout_team_$name.o
rm -f bc_mpc_amd/csrc/rollout_team_variant_tmp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/variants/libbcmpc_$name.so $OBJS build/variants/rollout_team_$name.o -ldl
ls -la build/variants/libbcmpc_$name.so
