#!/bin/bash
# GPU parity tests, then cfg2/cfg3/cfg4_shard/cfg5 benched with two libraries, twice each (A/B/A/B):
# build/variants/libbcmpc_head.so (+ zhead2 copy) against the in-tree build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for lib in head new zhead2 znew2; do
  echo "== $lib"
  if [ -f build/variants/libbcmpc_$lib.so ]; then L=$PWD/build/variants/libbcmpc_$lib.so; else L=$PWD/bc_mpc_amd/libbcmpc.so; fi
  BCMPC_LIB=$L WLS="cfg2 cfg3 cfg4_shard cfg5" STEPS=20 bash tools/wl_round.sh || exit $?
done
