#!/bin/bash
# round 3: single-pass f16 parity (printed envelopes), then the default bench line + its rocprofv3 summary
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest -m gpu -v -s --timeout 200 --timeout-method thread tests/test_gpu_f16.py \
  > gpurun_out/r03_f16_tests.log 2>&1 &&
timeout -k 10 500 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o run -- \
    python bench.py > gpurun_out/r03_bench_prof.json 2> gpurun_out/r03_bench_prof.err
