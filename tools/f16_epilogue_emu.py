#!/usr/bin/env python3
"""NumPy emulation of the single-pass f16 engine's arithmetic (rollout_pp<512,fold>) with
alternative tanh epilogues, scored against the f32-grade oracle on cfg3's net (build a cheaper
epilogue only if its +-10 penalty-flip count over 2,000 cfg3 candidates holds against today's).

The emulated kernel, per step and candidate (capi.cpp pack_x3_layer, rollout_x3.hip rollout_pp FOLD):
* layer-0 input [normalised state, normalised action] rounded to f16 (no operand scale, clamped to +-65504);
* hidden-producing layers (dense, dense_1) packed f16(W * 2 log2 e), accumulated in f32 from the bias
  * 2 log2 e (f16 x f16 products are exact in f32), so the accumulator is z = 2 log2(e) y;
* the epilogue turns z into tanh(y) and rounds it to f16 (the next layer's operand);
* the output layer f16(W2 * s) with s the power of two of x3_scale, accumulated in f32, / s, + bias;
* de-normalisation, the residual, the cheetah cost and the trajectory sum in f64 (as the kernel's owner phase).

Epilogues (issue cycles per activation at 8 per quarter-rate transcendental, 4 per full-rate op, packed f16
ops 4 per PAIR; DESIGN.md 6.7's accounting):
* ``today``   : f32 1 - 2 / (1 + 2^z)  (v_exp_f32, v_add_f32, v_rcp_f32, v_fma_f32, 1/2 v_cvt_pk)      ~26
* ``pk16_exp``: v_exp_f32, then packed f16: cvt, +1, v_rcp_f16, fma(-2, r, 1)                          ~22
* ``pk16_all``: f16 z (cvt), v_exp_f16, packed +1, v_rcp_f16, packed fma                               ~22
* ``ratl16``  : f16 odd rational x (27 + x^2) / (27 + 9 x^2) on x = clamp(y, +-3) (one v_rcp_f16)       ~20

usage: python tools/f16_epilogue_emu.py [n_candidates] [out.json]
"""
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from oracle import mpc_oracle as orc   # noqa: E402  (the checker: the f32-grade reference costs)

L2E2 = np.float32(2.0 / np.log(2.0))   # 2 log2(e)
f16, f32 = np.float16, np.float32


def h(x):
    """round to f16 (clamped below its overflow, NaN kept: the kernel's input conversion)"""
    return np.clip(np.asarray(x, np.float32), -65504, 65504).astype(f16)


def epi_today(z):
    r = (f32(1) / (np.exp2(z, dtype=f32) + f32(1))).astype(f32)
    return (f32(1) - f32(2) * r).astype(f32).astype(f16)


def epi_pk16_exp(z):
    e = np.exp2(z, dtype=f32).astype(f16)                      # v_exp_f32 -> v_cvt_pk_f16_f32
    d = (e.astype(np.float64) + 1.0).astype(f16)               # v_pk_add_f16
    r = (1.0 / d.astype(np.float64)).astype(f16)               # v_rcp_f16
    return (1.0 - 2.0 * r.astype(np.float64)).astype(f16)      # v_pk_fma_f16 (one rounding)


def epi_pk16_all(z):
    zh = z.astype(f16)
    e = np.exp2(zh.astype(np.float64)).astype(f16)             # v_exp_f16
    d = (e.astype(np.float64) + 1.0).astype(f16)
    r = (1.0 / d.astype(np.float64)).astype(f16)
    return (1.0 - 2.0 * r.astype(np.float64)).astype(f16)


def epi_ratl16(z):
    y = (z / L2E2).astype(f32)
    x = np.clip(y.astype(f16).astype(np.float64), -3.0, 3.0).astype(f16).astype(np.float64)
    x2 = (x * x).astype(f16).astype(np.float64)
    num = (x * (27.0 + x2).astype(f16).astype(np.float64)).astype(f16).astype(np.float64)
    den = (27.0 + 9.0 * x2).astype(f16).astype(np.float64)
    r = (1.0 / den).astype(f16).astype(np.float64)
    return (num * r).astype(f16)


EPILOGUES = {"today": (epi_today, 26), "pk16_exp": (epi_pk16_exp, 22), "pk16_all": (epi_pk16_all, 22),
             "ratl16": (epi_ratl16, 20)}


class F16Dynamics(orc.NumpyDynamics):
    """NumpyDynamics with the f16 engine's MLP (module docstring)."""

    def __init__(self, weights, normalization, epilogue):
        super().__init__(weights, normalization)
        w = weights
        self.epi = epilogue
        self.Wf = [h(k * L2E2) for k in w.kernels[:-1]]
        self.bf = [(b * L2E2).astype(f32) for b in w.biases[:-1]]
        mx = float(np.max(np.abs(w.kernels[-1])))
        e = np.frexp(mx)[1]
        self.so = f32(np.ldexp(1.0, max(-100, min(100, 12 - e))))
        self.Wo = h(w.kernels[-1] * self.so)
        self.bo = w.biases[-1].astype(f32)

    def mlp(self, x32):
        a = h(x32)
        for W, b in zip(self.Wf, self.bf):
            z = (a.astype(f32) @ W.astype(f32) + b).astype(f32)
            a = self.epi(z)
        out = (a.astype(f32) @ self.Wo.astype(f32)) / self.so + self.bo
        return out.astype(f32)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
    out_path = sys.argv[2] if len(sys.argv) > 2 else None
    H = 20
    import bench
    prob = bench.synthetic_problem(bench.WORKLOADS["cfg3"])
    w = orc.MLPWeights(prob["kernels"], prob["biases"], "tanh")
    norm, state = prob["norm"], prob["state"]
    acts = np.random.RandomState(2024).uniform(-1, 1, (H, n, 6))
    ref, paths = orc.rollout(orc.NumpyDynamics(w, norm), state, acts)
    near = orc.near_threshold_mask(paths)
    res = {"workload": f"cfg3 net (2x500 tanh, synthetic), H={H}, {n} candidates (actions RandomState(2024))",
           "reference": "oracle.NumpyDynamics (f32 MLP, f64 glue): the f32-grade costs",
           "flip_rule": "a candidate whose |cost - oracle| exceeds 5 (one +-10 penalty of cost_functions.py:18-26 "
                        "flipped somewhere on its trajectory)", "epilogues": {}}
    for name, (fn, cyc) in EPILOGUES.items():
        t0 = time.time()
        c, _ = orc.rollout(F16Dynamics(w, norm, fn), state, acts)
        d = np.abs(c - ref)
        flips = int(np.sum(d > 5.0))
        smooth = d[d <= 5.0]
        res["epilogues"][name] = {"issue_cycles_per_activation": cyc, "flips": flips,
                                  "flips_on_oracle_near_threshold": int(np.sum((d > 5.0) & near)),
                                  "median_abs_dcost": float(np.median(smooth)), "p99_abs_dcost": float(np.percentile(smooth, 99)),
                                  "max_abs_dcost_without_flips": float(np.max(smooth)),
                                  "argmin_equal": bool(int(np.argmin(c)) == int(np.argmin(ref))), "seconds": time.time() - t0}
        print(name, json.dumps(res["epilogues"][name]), flush=True)
    base = res["epilogues"]["today"]["flips"]
    res["decision"] = {k: ("holds" if v["flips"] <= max(base, 1) * 1.25 + 2 else "rejected: flips rise")
                       for k, v in res["epilogues"].items() if k != "today"}
    print(json.dumps(res["decision"]))
    if out_path:
        with open(out_path, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
