"""Plan sweep of the device MT19937 draw (csrc/mt_device.hip): p50 of get_action on NumPy's stream
(draw + rollout) minus p50 of get_action with Philox actions (rollout only), per (chunk words,
coefficient slices).  One JSON line per setting."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch  # noqa: F401
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    K, H = (int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "65536x20").split("x"))
    S, A, h = 20, 6, 500
    rs = np.random.RandomState(0)
    dims = [S + A, h, h, S]
    ks = [rs.uniform(-0.1, 0.1, (a, b)).astype(np.float32) for a, b in zip(dims[:-1], dims[1:])]
    bs = [np.zeros(b, np.float32) for b in dims[1:]]
    norm = [np.zeros(S), np.ones(S), np.zeros(A), np.ones(A), np.zeros(1), np.ones(1), np.zeros(S), np.ones(S),
            np.zeros(S), np.full(S, 0.05)]
    state = rs.randn(S) * 0.1
    low, high = -np.ones(A), np.ones(A)
    settings = [("default", None, None)]
    for w in (32768, 49152, 65536, 98304):
        for sp in (8, 16, 32):
            settings.append((f"w{w}_s{sp}", w, sp))
    base = None
    for name, w, sp in settings:
        for k, v in (("BCMPC_MT_CHUNK_WORDS", w), ("BCMPC_MT_SPLITS", sp)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = str(v)
        eng = RolloutEngine(S, A, h, 2, "tanh", False, H, K, device=0)
        eng.set_weights(MLPSpec(ks, bs, "tanh"), norm, 1)
        if base is None:
            ts = []
            for i in range(25):
                t0 = time.perf_counter()
                eng.get_action(state, None, seed=i)
                ts.append(time.perf_counter() - t0)
            base = float(np.median(ts[5:]))
        np.random.seed(0)
        t0 = time.perf_counter()
        eng.get_action_numpy_stream(state, low, high, K)       # plan + polynomials
        plan_s = time.perf_counter() - t0
        ts = []
        for i in range(25):
            t0 = time.perf_counter()
            eng.get_action_numpy_stream(state, low, high, K)
            ts.append(time.perf_counter() - t0)
        p50 = float(np.median(ts[5:]))
        print(json.dumps({"setting": name, "K": K, "H": H, "p50_ms": p50 * 1e3, "philox_p50_ms": base * 1e3,
                          "draw_ms": (p50 - base) * 1e3, "first_call_ms": plan_s * 1e3}), flush=True)
        eng.close()


if __name__ == "__main__":
    main()
