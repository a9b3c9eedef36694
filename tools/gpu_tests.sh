#!/bin/bash
# Selected GPU tests (args: pytest selectors), one process, each run under its own time limit.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v -rs --timeout 120 --timeout-method thread -p no:cacheprovider -m gpu "$@" \
    > gpurun_out/pytest_sel.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_sel.log
exit $rc
