"""A/B of single-pass f16 layouts (BCMPC_F16_NC / BCMPC_F16_NW) at cfg3 (K=65536, H=20, 2x500 tanh):
complete get_action (device Philox actions), HIP-event kernel time, rounds alternating the layouts.
usage: python tools/f16_ab.py [--rounds 2] [--steps 30] nc,nw [nc,nw ...]   (nc,nw = 0,0: split engine;
"pp": the two-group pipelined single-pass kernel)"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bc_mpc_amd.engine import MLPSpec, RolloutEngine   # noqa: E402

FLOP = 2 * ((20 + 6) * 500 + 500 * 500 + 500 * 20)


def weights(hidden=500, S=20, A=6, L=2):
    rs = np.random.RandomState(0)
    dims = [S + A] + [hidden] * L + [S]
    k = [(rs.randn(dims[i], dims[i + 1]) / np.sqrt(dims[i])).astype(np.float32) for i in range(L + 1)]
    b = [(0.1 * rs.randn(dims[i + 1])).astype(np.float32) for i in range(L + 1)]
    mo, so = rs.randn(S) * 0.1, np.abs(rs.randn(S)) * 0.5 + 0.2
    # utils.compute_normalization's 10-tuple (utils.py:132-158)
    norm = [mo, so, np.zeros(A), np.full(A, 1 / np.sqrt(3.0)), np.zeros(1), np.zeros(1), mo.copy(), so.copy(),
            0.005 * rs.randn(S), 0.05 * (np.abs(rs.randn(S)) + 0.2)]
    return k, b, norm


def run(layout, k, b, norm, steps, warmup, K=65536, H=20):
    nc, nw = layout
    prec = "split" if nc == 0 else "f16"
    if nc == -1:                                  # the two-group pipelined kernel
        os.environ["BCMPC_F16_PP"] = "1"
    elif nc:
        os.environ["BCMPC_F16_NC"], os.environ["BCMPC_F16_NW"] = str(nc), str(nw)
    eng = RolloutEngine(20, 6, 500, 2, "tanh", False, H, K, precision=prec)
    for v in ("BCMPC_F16_NC", "BCMPC_F16_NW", "BCMPC_F16_PP"):
        os.environ.pop(v, None)
    eng.set_weights(MLPSpec(k, b, "tanh"), norm, version=1)
    eng.set_timing(True)
    state = np.linspace(-0.5, 0.5, 20)
    for i in range(warmup):
        eng.get_action(state, None, seed=11 + i)
    ts, ks = [], []
    for i in range(steps):
        t0 = time.perf_counter()
        eng.get_action(state, None, seed=100 + i)
        ts.append(time.perf_counter() - t0)
        ks.append(eng.last_kernel_ms()[0])
    info = eng.info()
    eng.close()
    km = float(np.mean(ks))
    peak = 2516.6 if nc else 2516.6 / 3
    tf = K * H * FLOP / (km / 1e3) / 1e12
    return {"layout": "f16 pp (two-group pipeline)" if nc == -1 else
            f"{prec} nc={info.get('nc', nc)} nw={info.get('waves_per_block', nw)}",
            "kernel": info["kernel"], "value": K * H / float(np.mean(ts)), "p50_ms": float(np.median(ts) * 1e3),
            "kernel_ms": km, "tflops": tf, "frac": tf / peak}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("layouts", nargs="+")
    a = ap.parse_args()
    k, b, norm = weights()
    lays = [(-1, 0) if s == "pp" else tuple(int(x) for x in s.split(",")) for s in a.layouts]
    for r in range(a.rounds):
        for lay in lays:
            print(json.dumps(dict(round=r, **run(lay, k, b, norm, a.steps, a.warmup))), flush=True)


if __name__ == "__main__":
    main()
