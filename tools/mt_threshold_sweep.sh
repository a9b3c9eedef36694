#!/bin/bash
# GPU box: drop-in latency at small/medium K for several jump-ahead split thresholds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mw in 1048576 262144 131072 65536; do
    BCMPC_MT_MIN_WORDS=$mw timeout -k 10 120 python tools/bench_dropin.py --configs 1000x15,4096x20,16384x20 \
        > gpurun_out/mt_sweep_$mw.log 2>&1 || exit $?
    echo "min_words=$mw"; grep '^{' gpurun_out/mt_sweep_$mw.log | python -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(' ', d['config'], {k: round(v, 3) for k, v in d.items() if k.endswith('_ms') or k.endswith('threads')})"
done
