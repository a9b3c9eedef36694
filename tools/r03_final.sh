#!/bin/bash
# round 3 validation at head: the whole GPU suite, smoke(), the default bench line, rocprofv3 of the same command
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests \
  > gpurun_out/r03_final_pytest.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_final_smoke.log 2>&1 &&
timeout -k 10 500 python bench.py > gpurun_out/r03_final_bench.json 2> gpurun_out/r03_final_bench.err &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof_final" -o run -- \
    python bench.py > gpurun_out/r03_final_bench_prof.json 2> gpurun_out/r03_final_bench_prof.err
