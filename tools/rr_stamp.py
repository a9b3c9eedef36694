"""Per-phase stamps of the splitr kernel (RR_STAMP variant): python tools/rr_stamp.py K H hidden"""
import sys
import numpy as np
import os; sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from bc_mpc_amd.engine import MLPSpec, RolloutEngine  # noqa: E402
from oracle import mpc_oracle as orc  # noqa: E402
K, H, HID = (int(x) for x in sys.argv[1:4])
w = orc.synthetic_weights(20, 6, HID, 2, "tanh", False)
norm = orc.synthetic_normalization()
e = RolloutEngine(20, 6, HID, 2, "tanh", False, H, K, kernel="splitr")
e.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, 1)
e.set_timing(True)
st = orc.synthetic_state(norm)
for i in range(3):
    e.get_action(st, None, seed=7)
    print(f"K={K} kernel {e.last_kernel_ms()[0]:.4f} ms", flush=True)
