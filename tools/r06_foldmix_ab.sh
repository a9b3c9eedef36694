#!/bin/bash
# Round 6: the f16 pipelined kernel's folded epilogue writing f16 through v_fma_mix{lo,hi}_f16 (tree) against the
# f32 fma + v_cvt_pk form (build/variants/libbcmpc_mix0.so): the f16 tests on the tree, then an alternating A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06r}
mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests/test_gpu_f16.py \
    > "$OUT/pytest_f16.log" 2>&1 || { tail -30 "$OUT/pytest_f16.log"; exit 1; }
tail -1 "$OUT/pytest_f16.log"
ROUNDS=3 AB_ARGS="--precision f16" timeout -k 10 600 bash tools/ab_libs.sh cfg3 100 tree build/variants/libbcmpc_mix0.so \
    > "$OUT/foldmix_ab.txt" 2>&1 || { cat "$OUT/foldmix_ab.txt"; exit 1; }
cat "$OUT/foldmix_ab.txt"
