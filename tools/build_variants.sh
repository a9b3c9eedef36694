#!/bin/bash
# Build A/B variants of libbcmpc.so into build/variants/ (selected at run time via BCMPC_LIB).
# usage: tools/build_variants.sh [-x] "name:-DFLAG=1 ..." ...
#   default: flags apply to rollout.hip + rollout_grp.hip (f32 kernels)
#   -x     : flags apply to rollout_x3.hip only, built for one width / NC ($X3W, default 512; $X3NC, default 4)
#   -p     : flags apply to both units of rollout_x3.hip (X3_PART=1 / 2, every width and NC, the
#            production schedulers), linked with the in-tree build's other objects
set -e
cd "$(dirname "$0")/.."
mkdir -p build/variants
H="/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize -DBCMPC_DIAG_VARIANT"
X3=0
if [ "${1:-}" = "-x" ]; then X3=1; shift; fi
if [ "${1:-}" = "-p" ]; then X3=2; shift; fi
make -s -j8 ARCH=gfx950 >/dev/null
$H -x hip -c bc_mpc_amd/csrc/capi.cpp -o build/variants/capi.o
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  src=bc_mpc_amd/csrc/rollout_x3.hip
  if [[ "$name" == *@* ]]; then     # name@gitref: the split kernel source at that revision
    ref=${name#*@}; name=${name%%@*}
    git show "$ref":bc_mpc_amd/csrc/rollout_x3.hip > bc_mpc_amd/csrc/_x3_$name.hip
    src=bc_mpc_amd/csrc/_x3_$name.hip
  fi
  if [ $X3 = 2 ]; then
    ( $H -mllvm -amdgpu-sched-strategy=iterative-ilp -DX3_PART=1 $flags -c $src -o build/variants/rollout_x3_plain_$name.o &&
      $H -mllvm -amdgpu-sched-strategy=max-ilp -DX3_PART=2 $flags -c $src -o build/variants/rollout_x3_$name.o &&
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/variants/libbcmpc_$name.so \
          build/rollout.o build/rollout_grp.o build/cem.o build/fit.o build/mt19937.o build/mt_jump.o build/mt_device.o build/comm.o build/rollout_team.o build/variants/rollout_x3_$name.o build/variants/rollout_x3_plain_$name.o build/variants/capi.o -ldl ) &
  elif [ $X3 = 1 ]; then
    ( $H -DX3_ONLY=${X3W:-512} -DX3_ONLY_NC=${X3NC:-4} $flags -c $src -o build/variants/rollout_x3_$name.o &&
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/variants/libbcmpc_$name.so \
          build/rollout.o build/rollout_grp.o build/cem.o build/fit.o build/mt19937.o build/mt_jump.o build/mt_device.o build/comm.o build/rollout_team.o build/variants/rollout_x3_$name.o build/variants/capi.o -ldl ) &
  else
    ( $H $flags -c bc_mpc_amd/csrc/rollout.hip -o build/variants/rollout_$name.o &&
      $H $flags -c bc_mpc_amd/csrc/rollout_grp.hip -o build/variants/rollout_grp_$name.o &&
      /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o build/variants/libbcmpc_$name.so \
          build/variants/rollout_$name.o build/variants/rollout_grp_$name.o build/cem.o build/fit.o build/mt19937.o build/mt_jump.o build/mt_device.o build/comm.o build/rollout_x3.o build/rollout_x3_plain.o build/rollout_team.o \
          build/variants/capi.o -ldl ) &
  fi
done
wait
rm -f bc_mpc_amd/csrc/_x3_*.hip
ls build/variants/*.so
