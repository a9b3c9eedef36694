#!/bin/bash
# Build A/B variants of libbcmpc.so into build/variants/ (selected at run time via BCMPC_LIB).
# usage: tools/build_variants.sh "name:-DFLAG=1 ..." ...
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize"
$H -x hip -c bc_mpc_amd/csrc/capi.cpp -o build/variants/capi.o
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  ( $H $flags -c bc_mpc_amd/csrc/rollout.hip -o build/variants/rollout_$name.o &&
    $H $flags -c bc_mpc_amd/csrc/rollout_grp.hip -o build/variants/rollout_grp_$name.o &&
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/variants/libbcmpc_$name.so \
        build/variants/rollout_$name.o build/variants/rollout_grp_$name.o build/variants/capi.o ) &
done
wait
ls build/variants/*.so
