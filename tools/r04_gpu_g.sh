#!/bin/bash
set -o pipefail
bash tools/r04_team_ab.sh || exit 1
WLS="ppo_defaults cfg1 runsh_recipe ppo_mpc_default" bash tools/team_stamps.sh > gpurun_out/r04_team_stamps.txt 2>&1 || exit 1
cat gpurun_out/r04_team_stamps.txt
