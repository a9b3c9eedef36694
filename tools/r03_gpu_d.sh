#!/bin/bash
# round 3: small-K bench lines + team phase stamps of the LN reward / policy nets
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dropin-calls 10 > gpurun_out/r03_smallk.json 2> gpurun_out/r03_smallk.err &&
WLS="runsh_recipe runsh_noln ppo_mpc_default ppo_defaults" bash tools/team_stamps.sh > gpurun_out/r03_team_stamps.txt 2>&1
