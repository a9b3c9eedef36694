#!/bin/bash
# round 3: small-K bench lines, team A/B (current vs the pre-forward-progress kernel), team stamps
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --dropin-calls 10 > gpurun_out/r03_smallk.json 2> gpurun_out/r03_smallk.err &&
timeout -k 10 300 python tools/ab_smallk.py default,build/variants/libbcmpc_old47.so > gpurun_out/r03_ab_team.txt 2>&1 &&
WLS="runsh_recipe runsh_noln ppo_mpc_default" bash tools/team_stamps.sh > gpurun_out/r03_team_stamps.txt 2>&1
