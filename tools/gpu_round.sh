#!/bin/bash
# One GPU-box session: parity tests -> smoke -> bench -> rocprofv3 kernel trace.
# Every GPU step has its own time limit; any crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
STEPS=${STEPS:-30}
stop_on() {  # stop on anything but success / ordinary test failures
    local rc=$1 what=$2
    echo "$what rc=$rc"
    case $rc in 0) ;; 1) [ "$what" = pytest ] || exit $rc ;; *) echo "stopping after $what"; exit $rc ;; esac
}
if [ "${SKIP_TESTS:-0}" != 1 ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -q -s -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
    stop_on $? pytest
    tail -5 gpurun_out/pytest_gpu.log
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
    stop_on $? smoke
    cat gpurun_out/smoke.log
fi
timeout -k 10 600 python bench.py --steps "$STEPS" --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
stop_on $? bench
tail -2 gpurun_out/bench.log
if [ "${PROFILE:-1}" = 1 ]; then
    cd /tmp && export TMPDIR=/tmp
    timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run -- \
        python3 "$GRAFT_REPO_ROOT/bench.py" --steps "$STEPS" --warmup 3 --no-cpu-baseline ${BENCH_ARGS:-} \
        > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1
    stop_on $? rocprof
    find "$GRAFT_REPO_ROOT/gpurun_out/prof" -name "*stats*" | head
fi
if [ "${REHEARSE:-1}" = 1 ]; then
    cd "${GRAFT_REPO_ROOT:-/root/repo}"
    BCMPC_DIST_BACKEND=gloo BCMPC_BENCH_DEVICE=0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 \
        --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_2rank_rehearsal.log 2>&1
    stop_on $? rehearsal
    tail -1 gpurun_out/bench_2rank_rehearsal.log
fi
