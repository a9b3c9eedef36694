#!/bin/bash
# A/B the drop-in (NumPy-stream) p50 between library builds (BCMPC_LIB; "tree" = in-tree), alternating.
# usage: tools/ab_dropin.sh "wl1 wl2" calls lib1 lib2 ...   (env ROUNDS, default 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
WLS=$1; N=$2; shift 2
for r in $(seq 1 ${ROUNDS:-2}); do
  for wl in $WLS; do
    for lib in "$@"; do
      if [ "$lib" = tree ]; then unset BCMPC_LIB; else export BCMPC_LIB=$PWD/$lib; fi
      timeout -k 10 200 python tools/dropin_probe.py "$wl" "$N" | sed "s|^|$lib |" || exit 1
    done
  done
done
