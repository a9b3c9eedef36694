"""HBM traffic per launch of the head kernels from tools/r04_traffic.sh's PMC passes.

Reads gpurun_out/r04_traffic/<pass>/**/*counter_collection.csv (rocprofv3 --pmc, one counter per pass),
takes the rollout kernel's per-dispatch mean (first dispatch dropped: warm-up), calibrates the gfx950
FETCH_SIZE under-count on the action tensor (FETCH with actions read from HBM minus FETCH with device-RNG
actions, against the f64 tensor's K*H*A*8 bytes; MI355X_MICROARCH.md HBM section) and writes
profiles/r04_traffic_per_launch.json with the keys bench.py looks up (workload[:precision][:device]).
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1] if len(sys.argv) > 1 else os.path.join(REPO, "gpurun_out", "r04_traffic")
DST = os.path.join(REPO, "profiles", "r04_traffic_per_launch.json")

K3, H, A = 65536, 20, 6
ACTION_KB = K3 * H * A * 8 / 1024.0     # f64 actions (np.random.uniform)
W_SPLIT = 1179648            # hi + lo f16 fragments of the 2x500 tanh net padded to 512
W_F16 = W_SPLIT // 2         # hi only (F1 never reads lo)


def per_dispatch(name):
    rows = []
    for f in glob.glob(os.path.join(SRC, name, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            rows += [r for r in csv.DictReader(fh) if "rollout" in r["Kernel_Name"]]
    if not rows:
        return None, None, 0
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"], []).append((int(r["Dispatch_Id"]), float(r["Counter_Value"])))
    kern, vals = max(by.items(), key=lambda kv: len(kv[1]))
    vals = [v for _, v in sorted(vals)]
    vals = vals[1:] if len(vals) > 1 else vals
    return kern, sum(vals) / len(vals), len(vals)


def main():
    res = {}
    fh_kb = per_dispatch("fetch_hbm")[1]
    fd_kern, fd_kb, fd_n = per_dispatch("fetch_dev")
    factor = 2.0
    cal = "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM: gfx950 FETCH_SIZE reports half of streamed read bytes)"
    if fh_kb is not None and fd_kb is not None and fh_kb > fd_kb:
        seen = (fh_kb - fd_kb) / ACTION_KB
        cal += f"; calibration this round: FETCH(actions in HBM) - FETCH(device RNG) = {fh_kb - fd_kb:.1f} KB = " \
               f"{seen:.3f} of the {ACTION_KB:.0f} KB action tensor"
    src = "gpurun_out/r04_traffic/{%s} (tools/r04_traffic.sh: rocprofv3 --pmc, one counter per pass, this round's kernels)"

    def entry(key, fetch, write, wbytes, costs, note):
        kern, f_kb, n = per_dispatch(fetch)
        _, w_kb, _ = per_dispatch(write) if write else (None, None, 0)
        if f_kb is None:
            return
        hbm = f_kb * 1024 * factor + (w_kb or 0.0) * 1024
        res[key] = {"hbm_bytes_per_launch": hbm, "fetch_size_kb": f_kb, "write_size_kb": w_kb,
                    "dispatches": n, "correction": cal, "algorithmic_bytes_per_launch": wbytes + costs,
                    "kernel": kern[:160], "reading": note,
                    "source": src % ",".join(p for p in (fetch, write) if p)}

    entry("cfg3:split", "fetch_hbm", None, W_SPLIT + ACTION_KB * 1024, K3 * 8,
          "actions read from HBM (61440 KB tensor) + weights + costs; WRITE_SIZE pass taken in device mode")
    entry("cfg3:split:device", "fetch_dev", "write_dev", W_SPLIT, K3 * 8,
          "device-RNG actions: packed weights (each XCD misses them into its own L2) + the cost vector")
    entry("cfg3:f16_4x4:device", "f16_fetch_dev", "f16_write_dev", W_F16, K3 * 8,
          "single-pass f16, the 4x4 two-workgroup layout (default until the pipelined kernel): it spills 66 "
          "VGPRs at its 256-register cap, WRITE_SIZE is its scratch")
    # the pipelined kernel (rollout_pp, f16 default at large K), PMC passes of tools/r04_final.sh
    global SRC
    src0 = SRC
    SRC = os.path.join(os.path.dirname(src0), "r04_pmc_f16")
    entry("cfg3:f16:device", "fetch_pp", "write_pp", W_F16, K3 * 8,
          "single-pass f16, rollout_pp (two 64-candidate groups per workgroup, spill-free): hi fragments only")
    if "cfg3:f16:device" in res:
        res["cfg3:f16:device"]["source"] = res["cfg3:f16:device"]["source"].replace("r04_traffic/", "r04_pmc_f16/") \
            .replace("tools/r04_traffic.sh", "tools/r04_final.sh")
    SRC = src0
    entry("cfg2:split:device", "cfg2_fetch_dev", "cfg2_write_dev", W_SPLIT, 4096 * 8,
          "cfg2 K=4096: 256 columns, one per CU")
    if "cfg3:split" in res and "cfg3:split:device" in res:
        res["cfg3:split"]["write_size_kb"] = res["cfg3:split:device"]["write_size_kb"]
        res["cfg3:split"]["hbm_bytes_per_launch"] += res["cfg3:split"]["write_size_kb"] * 1024
    json.dump(res, open(DST, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:20s} {v['hbm_bytes_per_launch'] / 1e6:9.3f} MB/launch (alg {v['algorithmic_bytes_per_launch'] / 1e6:8.3f} MB)"
              f"  n={v['dispatches']}  {v['kernel'][:60]}")


if __name__ == "__main__":
    main()
