"""A short drop-in run for rocprofv3: MPCcontroller.get_action (rng="numpy", device MT19937 draw)
at K x H (default cfg3), 2x500 tanh, 30 calls."""
import os
import sys

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
    eng = RolloutEngine(S, A, h, 2, "tanh", False, H, K, device=0)
    eng.set_weights(MLPSpec(ks, bs, "tanh"), norm, 1)
    np.random.seed(0)
    for _ in range(30):
        eng.get_action_numpy_stream(rs.randn(S) * 0.1, -np.ones(A), np.ones(A), K)
    eng.close()


if __name__ == "__main__":
    main()
