"""Quick GPU check of the resident-column kernel (splitr) against split4 and the oracle.

python tools/rr_check.py [K] [H] [hidden]   -- prints max |dcost| vs split4, an oracle sample
check, and the kernel / get_action times of both kernels (device-RNG actions).
"""
import sys
import time

import numpy as np

import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bc_mpc_amd.engine import MLPSpec, RolloutEngine  # noqa: E402
from oracle import mpc_oracle as orc  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
H = int(sys.argv[2]) if len(sys.argv) > 2 else 20
HID = int(sys.argv[3]) if len(sys.argv) > 3 else 500
w = orc.synthetic_weights(20, 6, HID, 2, "tanh", False)
norm = orc.synthetic_normalization()
state = orc.synthetic_state(norm)
spec = MLPSpec(w.kernels, w.biases, w.activation)
res = {}
for kern in ("splitr", "split4"):
    e = RolloutEngine(20, 6, HID, 2, "tanh", False, H, K, kernel=kern)
    e.set_weights(spec, norm, 1)
    e.set_timing(True)
    r = e.get_action(state, None, seed=7, return_costs=True)
    ts, ks = [], []
    for _ in range(20):
        t0 = time.perf_counter()
        e.get_action(state, None, seed=7)
        ts.append(time.perf_counter() - t0)
        ks.append(e.last_kernel_ms()[0])
    res[kern] = r
    print(f"{kern}: info={e.info()} p50 {1e3 * np.median(ts):.3f} ms kernel {np.median(ks):.3f} ms "
          f"-> {K * H / (np.median(ks) * 1e-3):.3e} cand-steps/s (kernel)", flush=True)
    e.close()
a, b = res["splitr"].costs, res["split4"].costs
d = np.abs(a - b)
print(f"max|splitr - split4| = {np.nanmax(d):.3e}  argmin {res['splitr'].best_index} vs {res['split4'].best_index}")
rs = np.random.RandomState(1)
idx = np.unique(np.concatenate([rs.choice(K, min(K, 255), replace=False), [res['splitr'].best_index]]))
acts = orc.device_rng_actions(7, 0, K, H, -np.ones(6), np.ones(6))[:, idx, :]
want, states = orc.rollout(orc.NumpyDynamics(w, norm), state, acts)
err = np.abs(a[idx] - want)
print(f"oracle sample: max|dcost| = {err.max():.3e} (n={idx.size})")
