"""Rollout-kernel time (HIP events) of the perf mode (in-kernel Philox actions) against the NumPy-stream
mode (the host-drawn rows read in place over the bus), same engine, ppo_defaults: what the zero-copy rows
cost inside the kernel.  usage: python tools/zc_kernel_time.py [workload] [calls]"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "ppo_defaults"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    import torch  # noqa: F401
    wl = bench.WORKLOADS[name]
    p = bench.synthetic_problem(wl)
    eng = bench.make_engine(wl, p, 0, "auto")
    eng.set_timing(True)
    A = bench.A_DIM
    low, high = -np.ones(A), np.ones(A)
    np.random.seed(0)
    out = {"workload": name, "kernel": eng.info()["kernel"]}
    for mode in ("perf", "stream", "perf", "stream"):
        ks = []
        for i in range(calls):
            if mode == "perf":
                eng.get_action(p["state"], None, seed=i + 1)
            else:
                eng.get_action_numpy_stream(p["state"], low, high, wl["K"])
            ks.append(eng.last_kernel_ms()[0])
        out.setdefault(mode + "_kernel_us", []).append(round(float(np.median(ks[20:])) * 1e3, 2))
    eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
