#!/bin/bash
# split-kernel session: parity (-k split) on the in-tree lib, stamps, A/B of build/variants.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
bash tools/x3_round.sh || exit $?
bash tools/stamp_x3.sh
