#!/bin/bash
# rocprofv3 kernel stats of the device MT19937 draw (tools/mt_prof.py) for a few plan settings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
R=$PWD
cd /tmp && export TMPDIR=/tmp
for cfg in "${@:-32768:16}"; do
    w=${cfg%%:*}; s=${cfg#*:}
    BCMPC_MT_CHUNK_WORDS=$w BCMPC_MT_SPLITS=$s timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv \
        -d "$R/gpurun_out/mtprof_$w_$s" -o run -- python3 "$R/tools/mt_prof.py" > "$R/gpurun_out/mtprof_${w}_$s.log" 2>&1 || exit 1
    echo "== chunk words $w, slices $s"
    grep -E "mt_|rollout" "$R/gpurun_out/mtprof_$w_$s/run_kernel_stats.csv" | cut -d, -f1-4
done
