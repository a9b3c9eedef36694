#!/bin/bash
# GPU check of the split kernel's reward net: reward + policy parity tests, then the learned-reward
# workloads in split and fp32.  Each GPU step has its own limit; a crash ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_reward.py tests/test_gpu_parity.py -m gpu -q -s \
    -p no:cacheprovider -k "${K_EXPR:-reward or policy}" --timeout 120 --timeout-method thread \
    > gpurun_out/rw_pytest.log 2>&1
rc=$?
tail -6 gpurun_out/rw_pytest.log
grep -E "split" gpurun_out/rw_pytest.log | cut -c1-160 | head -60
[ $rc -le 1 ] || exit $rc
for wl in ${WLS:-cfg3_reward cfg3_polrew runsh_recipe}; do
    for prec in split fp32; do
        timeout -k 10 300 python bench.py --workload $wl --precision $prec --steps 10 --warmup 2 \
            --no-cpu-baseline > gpurun_out/rw_bench_${wl}_$prec.log 2>&1 || exit $?
        echo "$wl $prec $(tail -1 gpurun_out/rw_bench_${wl}_$prec.log | cut -c1-230)"
    done
done
exit $rc
