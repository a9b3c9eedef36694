"""End-to-end latency of the drop-in controller, host buffers included.

``bc_mpc_amd.MPCcontroller.get_action(state)`` with the reference's RNG contract (rng="numpy": one
``np.random.uniform(size=[H, K, A])`` from the global stream per call, controllers.py:53, uploaded over
PCIe) and with in-kernel Philox actions (rng="device").  This is the PCIe-inclusive figure DESIGN.md §8
reports beside bench.py's HBM-resident ``value``.  One JSON line per configuration.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


class _Space:
    def __init__(self, n, lo=None, hi=None):
        self.shape = (n,)
        if lo is not None:
            self.low, self.high = lo, hi


class _Env:
    observation_space = _Space(20)
    action_space = _Space(6, -np.ones(6), np.ones(6))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1000x15,4096x20,65536x20", help="KxH list")
    ap.add_argument("--calls", type=int, default=20)
    args = ap.parse_args()
    import torch  # noqa: F401  (single HIP runtime)
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    from bc_mpc_amd.dynamics import NNDynamicsModel
    S, A = 20, 6
    r7 = np.random.RandomState(7)
    mean_obs = 0.1 * r7.standard_normal(S)
    std_obs = np.abs(r7.standard_normal(S)) * 0.5 + 0.2
    norm = [mean_obs, std_obs, np.zeros(A), np.full(A, 1 / np.sqrt(3)), np.zeros(1), np.ones(1),
            mean_obs, std_obs, 0.005 * r7.standard_normal(S), 0.05 * (np.abs(r7.standard_normal(S)) + 0.2)]
    dyn = NNDynamicsModel(_Env(), 2, 500, "tanh", None, norm, 512, 1, 1e-3, device=0)
    state = mean_obs + 0.5 * std_obs * np.random.RandomState(11).standard_normal(S)
    for cfg in args.configs.split(","):
        K, H = (int(x) for x in cfg.split("x"))
        out = {"metric": "drop-in MPCcontroller.get_action wall time (host state in, host action out)",
               "config": f"K={K} H={H} 2x500 tanh, 1 GPU"}
        np.random.seed(0)
        t0 = time.perf_counter()
        for _ in range(3):
            np.random.uniform(-1, 1, size=[H, K, A])
        out["host_rng_ms"] = (time.perf_counter() - t0) / 3 * 1e3
        # the library's draw alone into a resident host array (serial, then split by jump-ahead)
        import ctypes
        from bc_mpc_amd import _lib
        lib = _lib.load()
        buf = np.zeros((H * K, A))
        lo, hi = -np.ones(A), np.ones(A)
        dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
        for name, thr in (("lib_draw_1thread_ms", 1), ("lib_draw_ms", 0)):
            st = np.random.get_state()
            key = np.array(st[1], dtype=np.uint32)
            used = ctypes.c_int32(0)
            ts = []
            for _ in range(5):
                pos = ctypes.c_int32(int(st[2]))
                t0 = time.perf_counter()
                lib.bcmpc_mt19937_uniform_par(key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos),
                                              dp(lo), dp(hi), A, H * K, K, 0, K, dp(buf), thr, -1,
                                              ctypes.byref(used))
                ts.append(time.perf_counter() - t0)
            out[name] = float(np.median(ts)) * 1e3
            out[name.replace("_ms", "_threads")] = used.value
        # numpy: the library's draw (split over host threads by jump-ahead when large);
        # numpy_1thread: the same draw forced serial (BCMPC_MT_THREADS=1, read per call)
        for mode in ("numpy", "numpy_1thread", "device"):
            rng = "device" if mode == "device" else "numpy"
            if mode == "numpy_1thread":
                os.environ["BCMPC_MT_THREADS"] = "1"
            else:
                os.environ.pop("BCMPC_MT_THREADS", None)
            ctrl = MPCcontroller(_Env(), dyn, horizon=H, cost_fn=cheetah_cost_fn, num_simulated_paths=K, rng=rng,
                                 seed=1 if rng == "device" else None)
            for _ in range(3):
                ctrl.get_action(state)
            ts = []
            for _ in range(args.calls):
                t0 = time.perf_counter()
                ctrl.get_action(state)
                ts.append(time.perf_counter() - t0)
            p50 = float(np.median(ts))
            out[f"{mode}_p50_ms"] = p50 * 1e3
            out[f"{mode}_cand_steps_per_s"] = K * H / p50
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
