"""Dump one engine's cost vector on a fixture (round 6 diagnostics): python tools/r06_dump_costs.py NAME KERNEL OUT.npy"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from conftest import Golden                     # noqa: E402
from bc_mpc_amd.engine import MLPSpec, RolloutEngine   # noqa: E402

name, kernel, out = sys.argv[1:4]
g = Golden(name)
w = g.weights
eng = RolloutEngine(g.S, g.A, w.hidden, w.n_layers, w.activation, w.layer_norm, g.H, g.K, device=0, kernel=kernel)
eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), g.norm, version=1)
res = eng.get_action(g.state, g.actions(), return_costs=True)
np.save(out, res.costs)
print(kernel, "max|d|", float(np.max(np.abs(res.costs - g.costs))))
eng.close()
