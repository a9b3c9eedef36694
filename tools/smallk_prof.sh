#!/bin/bash
# Small-K workloads (the reference's own configs): bench lines + rocprofv3 kernel stats.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
mkdir -p gpurun_out
for wl in ${WLS:-ppo_defaults runsh_recipe}; do
    timeout -k 10 200 python bench.py --workload $wl --steps 200 --warmup 20 --no-cpu-baseline --dropin-calls 0 \
        > gpurun_out/bench_$wl.log 2>&1 || { echo "bench $wl failed"; tail -5 gpurun_out/bench_$wl.log; exit 1; }
    python - "$wl" <<'PY'
import json, sys
l = [x for x in open(f"gpurun_out/bench_{sys.argv[1]}.log") if x.startswith("{")][-1]
d = json.loads(l)
print(sys.argv[1], "p50_ms", round(d["p50_ms"], 4), "kernel_ms", round(d["kernel_ms_avg"], 4), "value", "%.3g" % d["value"])
PY
    ( cd /tmp && export TMPDIR=/tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/prof_$wl" -o run -- python3 "$R/bench.py" --workload $wl --steps 200 --warmup 20 \
        --no-cpu-baseline --dropin-calls 0 > "$R/gpurun_out/prof_$wl.log" 2>&1 ) || exit 1
    cut -d, -f1-4 "$R/gpurun_out/prof_$wl/run_kernel_stats.csv" | head -8
done
