"""cProfile of the drop-in MPCcontroller.get_action (NumPy stream) at a small-K workload, plus the
rocprofv3-free GPU view: the same calls timed with the engine's own HIP events.
usage: python tools/dropin_prof.py [workload] [calls]"""
import cProfile
import os
import pstats
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    import torch  # noqa: F401
    import bench
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    from bc_mpc_amd.dynamics import NNDynamicsModel
    from oracle import mpc_oracle as orc
    wl = bench.WORKLOADS[sys.argv[1] if len(sys.argv) > 1 else "ppo_defaults"]
    calls = int(sys.argv[2]) if len(sys.argv) > 2 else 300
    S, A = 20, 6
    w = orc.synthetic_weights(S, A, wl["hidden"], wl["L"], wl["act"], wl.get("ln", False), seed_base=1000)
    norm = orc.synthetic_normalization(S, A)
    state = orc.synthetic_state(norm)
    dyn = NNDynamicsModel(bench._Env(), wl["L"], wl["hidden"], wl["act"], None, norm, 512, 1, 1e-3,
                          layer_norm=wl.get("ln", False), device=0)
    dyn.load_weights(w.kernels, w.biases, w.ln_gamma, w.ln_beta)
    ctrl = MPCcontroller(bench._Env(), dyn, horizon=wl["H"], cost_fn=cheetah_cost_fn,
                         num_simulated_paths=wl["K"], device=0)
    np.random.seed(0)
    for _ in range(10):
        ctrl.get_action(state)
    ts = []
    for _ in range(calls):
        t0 = time.perf_counter()
        ctrl.get_action(state)
        ts.append(time.perf_counter() - t0)
    print(f"drop-in p50 {np.median(ts) * 1e3:.4f} ms over {calls} calls")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(calls):
        ctrl.get_action(state)
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__":
    main()
