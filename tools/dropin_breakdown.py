"""Where the drop-in's small-K time goes: p50 of each layer of the NumPy-stream call at a
bench workload (default ppo_defaults: K=400, H=7, 2x256 relu + LN):
  perf      RolloutEngine.get_action(state, None, seed)           in-kernel Philox, no host draw
  stream    RolloutEngine.get_action_numpy_stream(...)            the library's NumPy-stream entry
  ctrl      MPCcontroller.get_action(state)                       the drop-in class
  np_draw   np.random.uniform(low, high, [H, K, A])               NumPy's own draw (reference)
usage: python tools/dropin_breakdown.py [workload] [calls]"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import bench  # noqa: E402


def p50(fn, calls, warm=20):
    for _ in range(warm):
        fn()
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return float(np.median(ts) * 1e3)


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "ppo_defaults"
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    import torch  # noqa: F401
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    from bc_mpc_amd.dynamics import NNDynamicsModel
    wl = bench.WORKLOADS[name]
    p = bench.synthetic_problem(wl)
    K, H, A = wl["K"], wl["H"], bench.A_DIM
    eng = bench.make_engine(wl, p, 0, "auto")
    low, high = -np.ones(A, np.float32), np.ones(A, np.float32)
    out = {"workload": name, "K": K, "H": H, "kernel": eng.info()["kernel"]}
    seed = [0]

    def perf():
        seed[0] += 1
        eng.get_action(p["state"], None, seed=seed[0])
    out["perf_ms"] = p50(perf, calls)
    np.random.seed(0)
    out["stream_ms"] = p50(lambda: eng.get_action_numpy_stream(p["state"], low, high, K), calls)
    # the C entry points alone (ctypes arguments prepared once): perf mode and the NumPy-stream entry
    import ctypes
    from bc_mpc_amd import _lib
    from bc_mpc_amd.engine import _dp, _legacy_mt_state
    lib, h = eng._lib, eng._h
    st = np.ascontiguousarray(p["state"], dtype=np.float64)
    res = _lib.Result()
    args_perf = (h, _dp(st), None, ctypes.c_uint64(1), ctypes.c_int64(0), ctypes.byref(res), None)
    out["perf_c_ms"] = p50(lambda: lib.bcmpc_get_action(*args_perf), calls)
    bg, key_p, pos_p = _legacy_mt_state()
    lo64, hi64 = np.ascontiguousarray(low, np.float64), np.ascontiguousarray(high, np.float64)
    args_mt = (h, _dp(st), key_p, pos_p, _dp(lo64), _dp(hi64), ctypes.c_int64(K), ctypes.c_int64(0),
               ctypes.c_uint64(0), ctypes.byref(res), None)
    out["stream_c_ms"] = p50(lambda: lib.bcmpc_get_action_mt19937(*args_mt), calls)

    def with_gap():                              # a 50-us host gap between calls (env.step stand-in)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 50e-6:
            pass
    ts = []
    for i in range(calls + 20):
        with_gap()
        t0 = time.perf_counter()
        lib.bcmpc_get_action_mt19937(*args_mt)
        if i >= 20:
            ts.append(time.perf_counter() - t0)
    out["stream_c_gap50us_ms"] = float(np.median(ts) * 1e3)
    out["predraw"] = os.environ.get("BCMPC_MT_PREDRAW", "1")
    eng.close()
    dyn = NNDynamicsModel(bench._Env(), wl["L"], wl["hidden"], wl["act"], None, p["norm"], 512, 1, 1e-3,
                          layer_norm=p["ln"], device=0)
    dyn.load_weights(p["kernels"], p["biases"], p["ln_g"], p["ln_b"])
    ctrl = MPCcontroller(bench._Env(), dyn, horizon=H, cost_fn=cheetah_cost_fn, num_simulated_paths=K, device=0)
    np.random.seed(0)
    out["ctrl_ms"] = p50(lambda: ctrl.get_action(p["state"]), calls)

    def slow():                                  # the repeat-call fast path off (every check redone)
        ctrl._fast = None
        ctrl.get_action(p["state"])
    out["ctrl_slowpath_ms"] = p50(slow, calls)

    def gap_p50(fn):
        ts = []
        for i in range(calls + 20):
            with_gap()
            t0 = time.perf_counter()
            fn()
            if i >= 20:
                ts.append(time.perf_counter() - t0)
        return float(np.median(ts) * 1e3)
    out["ctrl_gap50us_ms"] = gap_p50(lambda: ctrl.get_action(p["state"]))
    out["ctrl_slowpath_gap50us_ms"] = gap_p50(slow)
    out["np_draw_ms"] = p50(lambda: np.random.uniform(low, high, [H, K, A]), calls)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
