"""Cost vectors of one engine configuration under two library builds, compared bitwise (a layout change that
claims the same arithmetic and summation orders, e.g. rollout_pp's PP_QI sweep).

usage: python tools/lib_bitwise.py LIB_A LIB_B [--precision f16] [--K 65536] [--H 20]
Each build runs in its own child process (BCMPC_LIB), Philox actions, two seeds; exit status 1 on a mismatch."""
import argparse
import os
import subprocess
import sys
import tempfile

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import sys, numpy as np
sys.path.insert(0, {repo!r})
from bench import synthetic_problem, make_engine, WORKLOADS
wl = dict(WORKLOADS["cfg3"], K={K}, H={H})
prob = synthetic_problem(wl)
eng = make_engine(wl, prob, 0, {prec!r})
out = []
for seed in (11, 12):
    r = eng.get_action(prob["state"], None, seed=seed, return_costs=True)
    out.append(r.costs)
np.save({path!r}, np.stack(out))
print(eng.info()["layout"])
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("lib_a")
    ap.add_argument("lib_b")
    ap.add_argument("--precision", default="f16")
    ap.add_argument("--K", type=int, default=65536)
    ap.add_argument("--H", type=int, default=20)
    a = ap.parse_args()
    res = []
    with tempfile.TemporaryDirectory() as td:
        for i, lib in enumerate((a.lib_a, a.lib_b)):
            path = os.path.join(td, f"c{i}.npy")
            env = dict(os.environ, BCMPC_LIB=os.path.abspath(lib))
            code = CHILD.format(repo=REPO, K=a.K, H=a.H, prec=a.precision, path=path)
            p = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                print(p.stdout, p.stderr)
                sys.exit(2)
            print(f"{lib}: {p.stdout.strip().splitlines()[-1]}")
            res.append(np.load(path))
    ca, cb = res
    same = np.array_equal(ca, cb, equal_nan=True)
    diff = np.nanmax(np.abs(ca - cb))
    print(f"bitwise equal: {same}  max |diff| {diff:.3g}  ({ca.size} costs)")
    sys.exit(0 if same else 1)


if __name__ == "__main__":
    main()
