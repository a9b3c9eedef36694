#!/bin/bash
# round 3: reward-model fit timing (run.sh's model) + rocprofv3 kernel summary of the same command
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python tools/bench_fit.py --reward 1 --hidden 500 --ln 1 > gpurun_out/r03_fit_reward.json 2> gpurun_out/r03_fit_reward.err &&
timeout -k 10 300 python tools/bench_fit.py --reward 1 --hidden 500 --ln 0 > gpurun_out/r03_fit_reward_noln.json 2>> gpurun_out/r03_fit_reward.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fit -o fit -- python tools/bench_fit.py --reward 1 --hidden 500 --ln 1 --reps 2 --cpu-iters 2 > gpurun_out/r03_fit_reward_prof.log 2>&1 &&
timeout -k 10 200 python tools/dropin_breakdown.py ppo_defaults 400 > gpurun_out/r03_dropin_breakdown.json 2>&1 &&
timeout -k 10 200 python tools/dropin_breakdown.py cfg1 200 >> gpurun_out/r03_dropin_breakdown.json 2>&1
