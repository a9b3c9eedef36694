"""A/B timing of splitr variants (tools/rr_variants.sh): python tools/rr_ab.py K H hidden lib1 lib2 ...
('base' = the in-tree libbcmpc.so).  Each variant runs in its own process; kernel ms = HIP events."""
import os
import subprocess
import sys

K, H, HID = sys.argv[1:4]
CODE = r'''
import sys, numpy as np
sys.path.insert(0, __import__("os").environ.get("GRAFT_REPO_ROOT", "."))
from bc_mpc_amd.engine import MLPSpec, RolloutEngine
from oracle import mpc_oracle as orc
K, H, HID = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
w = orc.synthetic_weights(20, 6, HID, 2, "tanh", False); norm = orc.synthetic_normalization()
e = RolloutEngine(20, 6, HID, 2, "tanh", False, H, K, kernel="splitr"); e.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, 1); e.set_timing(True)
st = orc.synthetic_state(norm); ks = []
for i in range(25):
    e.get_action(st, None, seed=7); ks.append(e.last_kernel_ms()[0])
print(f"kernel {np.median(ks[5:]):.4f} ms  -> {K * H / (np.median(ks[5:]) * 1e-3):.3e} cand-steps/s")
'''
for rnd in range(2):
    for lib in sys.argv[4:]:
        env = dict(os.environ)
        if lib != "base":
            env["BCMPC_LIB"] = f"build/variants/libbcmpc_{lib}.so"
        out = subprocess.run([sys.executable, "-c", CODE, K, H, HID], env=env, capture_output=True, text=True, timeout=120)
        line = [l for l in out.stdout.splitlines() if l.startswith("kernel")]
        print(f"{lib:12s} {line[0] if line else out.stderr[-300:]}", flush=True)
