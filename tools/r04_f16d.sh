#!/bin/bash
# round 4: (4,4) two workgroups per CU -- does a start stagger (odd workgroups X3_STAGGER x 8k cycles late) de-phase them?
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
for r in 0 1; do
for v in base stag1 stag2 stag3; do
  lib=$R/build/variants/libbcmpc_$v.so; [ $v = base ] && lib=$R/bc_mpc_amd/libbcmpc.so
  echo "== $v"
  BCMPC_LIB=$lib timeout -k 10 120 python -u $R/tools/f16_ab.py --rounds 1 --steps 20 --warmup 3 4,4 4,8 2>&1 | grep round || exit 1
done
done > $R/gpurun_out/r04_f16d_stagger.log
