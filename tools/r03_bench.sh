#!/bin/bash
# round 3: the default bench line, then rocprofv3 --kernel-trace --stats of the same command
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 500 python bench.py > gpurun_out/r03_bench.json 2> gpurun_out/r03_bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_bench" -o run -- \
    python bench.py > gpurun_out/r03_bench_prof.json 2> gpurun_out/r03_bench_prof.err
