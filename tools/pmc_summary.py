"""Per-dispatch PMC summary of one kernel family from rocprofv3 --pmc CSV directories.
usage: python tools/pmc_summary.py <dir with <variant>_p<i>/.../run_counter_collection.csv> <kernel substring>
Prints, per variant: dispatches, mean kernel ms, L1->L2 read bytes (TCP_TCC_READ_REQ_sum x 128 B) per
dispatch and per CU-clock (GRBM_GUI_ACTIVE / 8: the counter sums the 8 XCDs), MFMA busy fraction (SQ_VALU_MFMA_BUSY_CYCLES over
SIMD-clocks: 4 SIMDs x 256 CUs), L2 hit rate."""
import collections
import csv
import glob
import os
import sys


def load(path, ksub):
    per = collections.defaultdict(dict)          # dispatch -> counter -> value
    dur = {}
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if ksub not in row["Kernel_Name"]:
                continue
            d = int(row["Dispatch_Id"])
            per[d][row["Counter_Name"]] = per[d].get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            dur[d] = (int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6
    return per, dur


def main():
    root, ksub = sys.argv[1], sys.argv[2]
    variants = sorted({os.path.basename(p).rsplit("_p", 1)[0] for p in glob.glob(os.path.join(root, "*_p[0-9]"))})
    for v in variants:
        acc = collections.defaultdict(list)
        ms = []
        for i in (1, 2, 3):
            per, dur = load(os.path.join(root, f"{v}_p{i}"), ksub)
            for d, cs in per.items():
                for k, x in cs.items():
                    acc[(i, k)].append(x)
                ms.append(dur[d])
        mean = {k: sum(x) / len(x) for k, x in acc.items() if x}
        clk1 = mean.get((1, "GRBM_GUI_ACTIVE"), float("nan")) / 8
        clk2 = mean.get((2, "GRBM_GUI_ACTIVE"), float("nan")) / 8
        mfma = mean.get((1, "SQ_VALU_MFMA_BUSY_CYCLES"), float("nan")) / (clk1 * 4 * 256)
        rd = mean.get((2, "TCP_TCC_READ_REQ_sum"), float("nan")) * 128
        hit = mean.get((3, "TCC_HIT_sum"), float("nan"))
        miss = mean.get((3, "TCC_MISS_sum"), float("nan"))
        print(f"{v:10s} dispatches={len(ms) // 3} kernel_ms={sum(ms) / max(len(ms), 1):.3f} "
              f"L1->L2 read GB/dispatch={rd / 1e9:.1f} B/clk/CU={rd / clk2 / 256:.1f} "
              f"clock GHz={clk2 / (sum(ms) / max(len(ms), 1)) / 1e6:.2f} MFMA busy={mfma:.3f} L2 hit={hit / (hit + miss):.4f}")


if __name__ == "__main__":
    main()
