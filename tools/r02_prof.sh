#!/bin/bash
# Round-2 evidence on the box: the default bench line, then rocprofv3 kernel-trace summaries of the cfg3
# bench command and of the small-K workloads (team kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_r02.log 2>&1 || { tail -5 gpurun_out/bench_r02.log; exit 1; }
tail -c 600 gpurun_out/bench_r02.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_cfg3" -o run -- \
    python3 "$R/bench.py" --no-cpu-baseline --no-small-k > "$R/gpurun_out/prof_cfg3.log" 2>&1 || exit 1
for wl in ppo_defaults runsh_recipe cfg1; do
    timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$wl" -o run -- \
        python3 "$R/bench.py" --workload $wl --steps 200 --warmup 20 --no-cpu-baseline --no-small-k --dropin-calls 0 \
        > "$R/gpurun_out/prof_$wl.log" 2>&1 || exit 1
done
for d in cfg3 ppo_defaults runsh_recipe cfg1; do echo "== $d"; cut -d, -f1-4 "$R/gpurun_out/prof_$d/run_kernel_stats.csv" | head -6; done
