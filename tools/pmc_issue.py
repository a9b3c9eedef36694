"""Issue / wait / memory-path summary of one kernel from the PMC passes of tools/gpu_validate.sh (step "issue").
usage: python tools/pmc_issue.py <gpurun_out/TAG> <kernel substring> [candidate-steps per dispatch]

Units (MI355X_MICROARCH.md, constants table): SQ_WAVE_CYCLES, SQ_ACTIVE_INST_*, SQ_WAIT_* count quad-cycles
(x4 -> cycles), summed over waves; SQ_VALU_MFMA_BUSY_CYCLES counts cycles summed over SIMDs; GRBM_GUI_ACTIVE
sums the 8 XCDs (/8 -> clocks of the dispatch).  A SIMD holds the kernel's waves (two per SIMD for 512-thread
workgroups), so "per SIMD" = summed wave figures / (1024 SIMDs x clocks).  TA / TD / TCP counters are per CU
instance (_sum over 256)."""
import collections
import csv
import glob
import os
import sys


def load(path, ksub):
    per = collections.defaultdict(dict)
    dur = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if ksub not in row["Kernel_Name"]:
                continue
            d = int(row["Dispatch_Id"])
            per[d][row["Counter_Name"]] = per[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    return per, dur


def mean_counters(path, ksub):
    per, dur = load(path, ksub)
    ds = sorted(per)[1:] if len(per) > 1 else sorted(per)      # first dispatch dropped (warm-up)
    acc = collections.defaultdict(list)
    for d in ds:
        for k, v in per[d].items():
            acc[k].append(v)
    return {k: sum(v) / len(v) for k, v in acc.items()}, [dur[d] for d in ds]


def main():
    root, ksub = sys.argv[1], sys.argv[2]
    cs = float(sys.argv[3]) if len(sys.argv) > 3 else None
    m, ms = {}, []
    for p in ("pmc_a", "pmc_b", "pmc_c", "pmc_d"):
        c, d = mean_counters(os.path.join(root, p), ksub)
        for k, v in c.items():
            m.setdefault(k, v)
        ms += d
    kms = sum(ms) / max(len(ms), 1)
    clk = m.get("GRBM_GUI_ACTIVE", float("nan")) / 8
    simd = clk * 1024
    q = lambda k: 4.0 * m.get(k, float("nan"))            # quad-cycles -> cycles
    print(f"# {ksub}: {len(ms)} dispatches, kernel {kms:.3f} ms, {clk:.4g} clocks -> {clk / kms / 1e6:.2f} GHz")
    for k in sorted(m):
        print(f"{k:32s} {m[k]:.4g}")
    print("# per SIMD (fraction of SIMD-cycles)")
    print(f"MFMA pipe busy                    {m.get('SQ_VALU_MFMA_BUSY_CYCLES', float('nan')) / simd:.3f}")
    for k in ("SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_LDS",
              "SQ_ACTIVE_INST_SCA", "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_LDS",
              "SQ_INST_CYCLES_VMEM_RD", "SQ_VALU_MFMA_COEXEC_CYCLES", "SQ_ACTIVE_INST_VALU2"):
        if k in m:
            v = m[k] if k == "SQ_VALU_MFMA_COEXEC_CYCLES" else q(k)
            print(f"{k:32s}  {v / simd:.3f}")
    print(f"wave-cycles per SIMD-cycle         {q('SQ_WAVE_CYCLES') / simd:.3f}  (resident waves per SIMD)")
    print("# instruction mix per dispatch" + (f" and per candidate-step ({cs:.4g} per dispatch)" if cs else ""))
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_VALU_TRANS_F32", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_CVT",
              "SQ_INSTS_VMEM_RD", "SQ_INSTS_LDS", "SQ_INSTS_SALU"):
        if k in m:
            print(f"{k:32s} {m[k]:.4g}" + (f"   {m[k] * 64 / cs:.1f} lane-instr/cand-step" if cs else ""))
    print("# memory path (per CU-clock)")
    n = clk * 256
    for k in ("TA_TA_BUSY_sum", "TD_TD_BUSY_sum", "TD_TC_STALL_sum", "TCP_PENDING_STALL_CYCLES_sum"):
        if k in m:
            print(f"{k:32s} {m[k] / n:.3f}")
    if "TCP_TCC_READ_REQ_sum" in m:
        rq = m["TCP_TCC_READ_REQ_sum"]
        print(f"L1->L2 read requests               {rq:.4g}  ({rq * 128 / 1e9:.2f} GB at 128 B, {rq * 128 / n:.1f} B/clk/CU)")
        if "TCP_TCC_READ_REQ_LATENCY_sum" in m:
            print(f"mean L1->L2 read latency          {m['TCP_TCC_READ_REQ_LATENCY_sum'] / rq:.0f} cycles")
    if "TA_BUFFER_READ_WAVEFRONTS_sum" in m:
        print(f"buffer read wave-instructions      {m['TA_BUFFER_READ_WAVEFRONTS_sum']:.4g}")


if __name__ == "__main__":
    main()
