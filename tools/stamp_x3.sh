#!/bin/bash
# Per-phase s_memtime stamps of the split kernel (X3_STAMP variant build in build/variants).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
BCMPC_LIB=$PWD/${STAMP_LIB:-build/variants/libbcmpc_stamp.so} BCMPC_X3_STAMPS=1 timeout -k 10 300 \
    python bench.py --precision split --steps 3 --warmup 1 --no-cpu-baseline --no-small-k --dropin-calls 0 ${BENCH_ARGS:-} > gpurun_out/stamp.log 2>&1
echo "rc=$?"
grep "x3 stamps" gpurun_out/stamp.log | tail -2
tail -1 gpurun_out/stamp.log | cut -c1-300
