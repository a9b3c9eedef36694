set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q -s -p no:cacheprovider -x tests/test_gpu_cem.py > gpurun_out/pytest_cem.log 2>&1
rc=$?; echo "pytest cem rc=$rc"; grep -E "passed|failed|error|Error" gpurun_out/pytest_cem.log | tail -5
case $rc in 0|1) ;; *) exit $rc ;; esac
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_cem.log; exit 1; }
timeout -k 10 600 python bench.py --workload cfg5 --steps 5 --warmup 1 > gpurun_out/bench_cfg5.log 2>&1
rc=$?; echo "bench cfg5 rc=$rc"; tail -c 2500 gpurun_out/bench_cfg5.log
