#!/bin/bash
# round 3: pre-draw handshake A/B (spin 0 = condition variable only, default 200 us spin), alternating, ppo_defaults
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/r03_spin_ab.txt
: > $out
for i in 1 2; do
  for sp in 0 200; do
    echo "spin_us=$sp run=$i" >> $out
    BCMPC_MT_PREDRAW_SPIN_US=$sp timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 2>/dev/null >> $out || exit 1
  done
done
