#!/bin/bash
# PMC passes (each its own run, --pmc only) over the resident-column kernel (tools/rr_stamp.py driver).
set -u
R=${GRAFT_REPO_ROOT:-/root/repo}
cd /tmp && export TMPDIR=/tmp
OUT=$R/gpurun_out/pmcrr
mkdir -p "$OUT"
pass() {  # name, counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/$name" -o run -- \
      python3 "$R/tools/rr_stamp.py" ${RR_ARGS:-65536 20 500} > "$OUT/$name.log" 2>&1
  local rc=$?; echo "pass $name rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/$name.log"; exit $rc; }
}
pass sq1 GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU
pass sq2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES
pass sq3 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT
pass fetch FETCH_SIZE
python3 - "$OUT" <<'PY'
import csv, glob, os, sys, collections
out = sys.argv[1]
for d in sorted(glob.glob(os.path.join(out, '*'))):
    if not os.path.isdir(d): continue
    files = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    agg = collections.defaultdict(list)
    for f in files:
        for r in csv.DictReader(open(f)):
            if 'rollout_rr' in r.get('Kernel_Name', ''):
                agg[r['Counter_Name']].append(float(r['Counter_Value']))
    for k, v in sorted(agg.items()):
        print(f"{os.path.basename(d):6s} {k:28s} per-dispatch mean {sum(v)/max(1,len(v)):.4g} (n={len(v)})")
PY
