#!/bin/bash
# Round 6: the parity files over the new K=4096 fixtures, then the ns_shard workgroup-width A/B (NC 2 auto, 4, 1).
# A test failure (pytest rc 1) still runs the A/B; any other status (a fault, a time limit) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r06e}
mkdir -p "$OUT"
timeout -k 10 500 python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_team.py tests/test_gpu_sweep.py > "$OUT/pytest.log" 2>&1
rc=$?
tail -3 "$OUT/pytest.log"
[ $rc -le 1 ] || { echo "pytest rc=$rc: stopping"; exit $rc; }
ROUNDS=2 timeout -k 10 600 bash tools/ab_env.sh ns_shard 50 - BCMPC_KERNEL=split4 BCMPC_KERNEL=split1 \
    > "$OUT/ns_nc_ab.txt" 2>&1 || { cat "$OUT/ns_nc_ab.txt"; exit 1; }
cat "$OUT/ns_nc_ab.txt"
exit $rc
