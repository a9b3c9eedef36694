#!/bin/bash
# Phase stamps of the split kernel with and without the fused policy (full X3_STAMP build).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for wl in cfg3 cfg3_policy; do
  BCMPC_LIB=$PWD/build/variants/libbcmpc_stampfull.so BCMPC_X3_STAMPS=1 timeout -k 10 300 \
      python bench.py --workload $wl --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/stamp_$wl.log 2>&1 || exit $?
  echo "== $wl"; grep "x3 stamps" gpurun_out/stamp_$wl.log | tail -2
done
