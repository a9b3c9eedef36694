#!/bin/bash
# HBM traffic of the split kernel (cfg3): FETCH_SIZE with actions in HBM and with device-RNG actions
# (the difference calibrates FETCH_SIZE against the known 61440 KB action tensor), WRITE_SIZE.
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/pmctr
mkdir -p "$OUT"
pass() {
  local name=$1 args=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/bench.py" --steps 3 --warmup 1 --no-cpu-baseline --dropin-calls 0 --precision split $args > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
pass fetch_hbm "--actions hbm" FETCH_SIZE
pass fetch_dev "--actions device" FETCH_SIZE
pass write_hbm "--actions hbm" WRITE_SIZE
pass write_dev "--actions device" WRITE_SIZE
python3 - "$OUT" <<'PY'
import csv, glob, os, sys
out = sys.argv[1]
for name in ("fetch_hbm", "fetch_dev", "write_hbm", "write_dev"):
    vals = []
    for f in glob.glob(os.path.join(out, name, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "rollout_x3" in r.get("Kernel_Name", ""):
                vals.append(float(r["Counter_Value"]))
    print(name, "per-dispatch mean KB", sum(vals) / max(1, len(vals)), "n", len(vals))
PY
