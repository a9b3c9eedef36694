set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "split" > gpurun_out/split_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/split_pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --precision split --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/split_bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/split_bench.log
