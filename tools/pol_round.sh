#!/bin/bash
# GPU check of the split kernel's fused policy: policy parity tests, then cfg3_policy bench
# in split and fp32 precision.  Each GPU step has its own limit; a crash ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider -k "${K_EXPR:-policy}" \
    --timeout 120 --timeout-method thread > gpurun_out/pol_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/pol_pytest.log
grep -E "split policy|max\|d" gpurun_out/pol_pytest.log | head -40
[ $rc -le 1 ] || exit $rc
for prec in split fp32; do
    timeout -k 10 300 python bench.py --workload cfg3_policy --precision $prec --steps 10 --warmup 2 \
        --no-cpu-baseline > gpurun_out/pol_bench_$prec.log 2>&1 || exit $?
    tail -1 gpurun_out/pol_bench_$prec.log | cut -c1-400
done
exit $rc
