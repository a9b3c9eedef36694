#!/bin/bash
# tools/ab_lib.sh over several workloads (WLS), stopping at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for wl in ${WLS:-ppo_defaults runsh_recipe cfg3}; do
  echo "== $wl"
  bash tools/ab_lib.sh "$1" "$wl" "${STEPS:-100}" || exit 1
done
