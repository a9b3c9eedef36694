#!/bin/bash
# round 4: where the single-pass f16 step goes -- phase stamps (X3_STAMP variant) and PMC per layout
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
mkdir -p $R/gpurun_out/r04_pmc_f16
for lay in "4,8" "8,8" "4,4"; do
  BCMPC_LIB=$R/build/variants/libbcmpc_stamp.so BCMPC_X3_STAMPS=1 timeout -k 10 120 \
    python -u $R/tools/f16_ab.py --rounds 1 --steps 3 --warmup 1 $lay > $R/gpurun_out/r04_f16b_stamp_$lay.log 2>&1 || exit $?
done
cd /tmp && export TMPDIR=/tmp
pass() {  # layout tag, counters...
  local lay=$1 name=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d "$R/gpurun_out/r04_pmc_f16/${name}_${lay/,/x}" -o run -- \
      python3 "$R/tools/f16_ab.py" --rounds 1 --steps 4 --warmup 1 $lay > "$R/gpurun_out/r04_pmc_f16/${name}_${lay/,/x}.log" 2>&1
  local rc=$?; echo "pass $name $lay rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for lay in "4,8" "8,8" "4,4"; do
  pass $lay p1 GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU || exit $?
  pass $lay p2 SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES || exit $?
  pass $lay p3 SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT || exit $?
  pass $lay p4 TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum || exit $?
done
