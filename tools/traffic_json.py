"""HBM traffic per launch of the head kernels from tools/gpu_validate.sh's "traffic" step.

usage: python tools/traffic_json.py gpurun_out/<TAG> [profiles/<out>.json]

Reads <TAG>/traffic_<workload>_<precision>_{fetch,write}/**/*counter_collection.csv (rocprofv3 --pmc, one
counter per pass), takes the rollout kernel's per-dispatch mean (first dispatch dropped: warm-up), applies
the gfx950 FETCH_SIZE correction (x2: MI355X_MICROARCH.md HBM section; calibrated on the action tensor when
the cfg3 hbm-actions pass is present: FETCH with actions read from HBM minus FETCH with device-RNG actions,
against the f64 tensor's K*H*A*8 bytes) and writes the keys bench.py looks up ("<workload>:<precision>:device").
"""
import csv
import glob
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = sys.argv[1]
DST = sys.argv[2] if len(sys.argv) > 2 else os.path.join(REPO, "profiles", "r06_traffic_per_launch.json")

# (K, H, padded hidden, hidden layers) of the bench workloads
SHAPES = {"cfg3": (65536, 20, 512, 2), "cfg2": (4096, 20, 512, 2), "ns_shard": (8192, 20, 512, 2), "cfg4_shard": (32768, 20, 512, 2),
          "cfg5": (65536, 50, 1024, 3)}


READING = {
    "cfg3": "device-RNG actions: the packed weights (each XCD misses them into its own L2) + the cost vector",
    "cfg5": ("the packed weights (9.2 MB split) exceed an XCD's 4 MiB L2, so every column step re-streams them "
             "from the Infinity Cache (FETCH_SIZE counts its hits: MI355X_MICROARCH.md HBM section); one rollout "
             "pass of the CEM call")}


def weight_bytes(hp, L, precision):
    """Packed fragment bytes (capi.cpp pack_x3_layer): layer 0 one k-step, hidden layers P k-steps, the
    output layer 2 tiles; 2 KiB per (tile, k-step) as hi | lo, 1 KiB hi only for the single pass."""
    T, P = hp // 16, hp // 32
    frags = T + (L - 1) * T * P + 2 * P
    return frags * (1024 if precision == "f16" else 2048)


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
    factor = 2.0
    cal = "FETCH_SIZE x2 (MI355X_MICROARCH.md HBM: gfx950 FETCH_SIZE reports half of streamed read bytes)"
    fh_kb = per_dispatch("traffic_cfg3_split_hbm_fetch")[1]
    fd_kb = per_dispatch("traffic_cfg3_split_fetch")[1]
    if fh_kb is not None and fd_kb is not None and fh_kb > fd_kb:
        K, H, _, _ = SHAPES["cfg3"]
        act_kb = K * H * 6 * 8 / 1024.0
        cal += (f"; calibration: FETCH(actions in HBM) - FETCH(device RNG) = {fh_kb - fd_kb:.1f} KB = "
                f"{(fh_kb - fd_kb) / act_kb:.3f} of the {act_kb:.0f} KB action tensor")
    for d in sorted(glob.glob(os.path.join(SRC, "traffic_*_fetch"))):
        name = os.path.basename(d)[len("traffic_"):-len("_fetch")]
        if name.endswith("_hbm"):
            continue
        wl, prec = name.rsplit("_", 1)
        kern, f_kb, n = per_dispatch(f"traffic_{name}_fetch")
        _, w_kb, _ = per_dispatch(f"traffic_{name}_write")
        if f_kb is None or wl not in SHAPES:
            continue
        K, H, hp, L = SHAPES[wl]
        alg = weight_bytes(hp, L, prec) + K * 8
        hbm = f_kb * 1024 * factor + (w_kb or 0.0) * 1024
        res[f"{wl}:{prec}:device"] = {
            "hbm_bytes_per_launch": hbm, "fetch_size_kb": f_kb, "write_size_kb": w_kb, "dispatches": n,
            "correction": cal, "algorithmic_bytes_per_launch": alg, "kernel": kern[:160],
            "reading": READING.get(wl, READING["cfg3"]),
            "source": f"{os.path.relpath(SRC, REPO)}/traffic_{name}_{{fetch,write}} (tools/gpu_validate.sh traffic)"}
    json.dump(res, open(DST, "w"), indent=1)
    for k, v in res.items():
        print(f"{k:24s} {v['hbm_bytes_per_launch'] / 1e6:9.3f} MB/launch (alg {v['algorithmic_bytes_per_launch'] / 1e6:8.3f} MB)"
              f"  n={v['dispatches']}  {v['kernel'][:60]}")


if __name__ == "__main__":
    main()
