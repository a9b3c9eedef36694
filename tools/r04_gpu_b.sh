#!/bin/bash
# round 4: PP kernel (tests, stamps, A/B) then the HBM-traffic PMC passes at head
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd $R
bash tools/r04_pp2.sh || exit $?
bash tools/r04_traffic.sh > gpurun_out/r04_traffic.log 2>&1
rc=$?; tail -12 gpurun_out/r04_traffic.log; exit $rc
