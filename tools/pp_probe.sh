#!/bin/bash
# Register / spill report for rollout_pp<512> under extra flags (e.g. -DPP_D=3).
# usage: tools/pp_probe.sh [hipcc flags...]
set -e
cd "$(dirname "$0")/.."
f=$(mktemp /tmp/ppprobe_XXXX.hip)
{ echo '#define X3_PROBE 1'; echo '#include "'$PWD'/bc_mpc_amd/csrc/rollout_x3.hip"'
  echo "template __global__ void bcmpc::rollout_pp<512, ${PP_FOLD:-true}>(const bcmpc::RolloutArgs);"; } > $f
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
  ${X3SCHED:--mllvm -amdgpu-sched-strategy=max-ilp} "$@" --cuda-device-only -c $f -o /tmp/ppprobe.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs:|Spill|Occupancy" | \
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' | paste - - - - - - | sed 's/Function Name: _ZN5bcmpc10//'
rm -f $f
