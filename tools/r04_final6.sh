#!/bin/bash
# round 4 validation at head (at the end of round 4): the whole GPU suite, smoke(), the default bench
# line, rocprofv3 --kernel-trace --stats of the same command
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 900 python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread tests \
  > gpurun_out/r04_final6_pytest.log 2>&1 || { tail -40 gpurun_out/r04_final6_pytest.log; exit 1; }
tail -1 gpurun_out/r04_final6_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_final6_smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py > gpurun_out/r04_final6_bench.json 2> gpurun_out/r04_final6_bench.err || exit 1
echo bench done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/r04_prof_final6" -o run -- \
    python3 bench.py > gpurun_out/r04_final6_bench_prof.json 2> gpurun_out/r04_final6_bench_prof.err
echo "prof rc=$?"
