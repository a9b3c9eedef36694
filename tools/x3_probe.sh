#!/bin/bash
# Register / spill report for single rollout_x3 instantiations (no launchers, seconds per build).
# usage: tools/x3_probe.sh "HP,NC,NW,PHP,RW,AK,F1" ... [-- extra hipcc flags]
set -e
cd "$(dirname "$0")/.."
insts=(); extra=()
while [ $# -gt 0 ]; do
  if [ "$1" = "--" ]; then shift; extra=("$@"); break; fi
  insts+=("$1"); shift
done
f=$(mktemp /tmp/x3probe_XXXX.hip)
{
  echo '#define X3_PROBE 1'
  echo '#include "'$PWD'/bc_mpc_amd/csrc/rollout_x3.hip"'
  for i in "${insts[@]}"; do
    IFS=, read hp nc nw php rw ak f1 <<< "$i"
    echo "template __global__ void bcmpc::rollout_x3<$hp,$nc,$nw,$php,$rw,$ak,$f1>(const bcmpc::RolloutArgs);"
  done
} > $f
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -fno-slp-vectorize \
  ${X3SCHED:--mllvm -amdgpu-sched-strategy=max-ilp} "${extra[@]}" --cuda-device-only -c $f -o /tmp/x3probe.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|AGPRs:|Spill|Occupancy" | \
  sed -e 's/.*remark: *//' -e 's/ \[-Rpass.*//' | paste - - - - - - | sed 's/_ZN5bcmpc10rollout_x3I//'
rm -f $f
