#!/bin/bash
# round 4: timing-only ablations of the f16 / split kernels (results wrong by construction)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
for v in base notanh noowner nobar noloads; do
  lib=$R/build/variants/libbcmpc_$v.so; [ $v = base ] && lib=$R/bc_mpc_amd/libbcmpc.so
  echo "== $v" 
  BCMPC_LIB=$lib timeout -k 10 120 python -u $R/tools/f16_ab.py --rounds 1 --steps 20 --warmup 3 0,0 4,8 8,8 4,4 2>&1 | grep round || exit 1
done > $R/gpurun_out/r04_f16c_ablate.log
