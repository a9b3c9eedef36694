#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 > gpurun_out/r03_dropin_breakdown.json 2>&1 &&
BCMPC_MT_PREDRAW=0 timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 >> gpurun_out/r03_dropin_breakdown.json 2>&1
