#!/bin/bash
# Bench the workloads $WLS with every library in $LIBS (names under build/variants/libbcmpc_<name>.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for lib in $LIBS; do
  echo "== $lib"
  BCMPC_LIB=$PWD/build/variants/libbcmpc_$lib.so STEPS=${STEPS:-20} bash tools/wl_round.sh || exit $?
done
