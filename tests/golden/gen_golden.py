#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ from the REFERENCE code.

Run in the build container only (``/root/reference`` is absent on the GPU box):

    python tests/golden/gen_golden.py

What is pinned, and how:

* The reference's own ``controllers.MPCcontroller.get_action``
  (controllers.py:43-88) and ``cost_functions.cheetah_cost_fn`` /
  ``trajectory_cost_fn`` (cost_functions.py:9-63) are imported from
  ``/root/reference`` and executed unmodified.  They consume the global legacy
  MT19937 stream (controllers.py:53), tile the state (:63), run H x predict
  (:69-71), score (:80), argmin (:82) and copy the first action (:84-85).
* ``dynamics.NNDynamicsModel`` cannot be imported (TensorFlow 1.x is absent
  and unpinned), so ``oracle.NumpyDynamics`` -- the build's restatement of
  ``dynamics.py:54-71,106-119`` -- is injected as ``dyn_model``.
* The per-candidate costs the reference computes are captured by wrapping
  ``controllers.trajectory_cost_fn`` (the name ``get_action`` resolves at call
  time), so fixtures hold the reference's own cost vector, not a replay.
* ``saved_data/ppo-mpc/vars.pkl`` (trained weights) is NOT used: the only
  allowed loader for a pickle shipped in the reference is
  ``torch.load(weights_only=True)``, which refuses this plain (non-torch)
  pickle; the script records that refusal and uses synthetic weights of the
  same shape (2x256 relu) instead.

Fixtures are data only: inputs (seeds, config, small weights) and expected
outputs.  Large action tensors are regenerated from the seed through legacy
``np.random.RandomState`` (stream stable across NumPy versions).
"""
from __future__ import annotations

import json
import os
import re
import sys

import numpy as np

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, REF)

import controllers as ref_controllers      # noqa: E402  (reference, read-only)
import cost_functions as ref_costs         # noqa: E402  (reference, read-only)
from oracle import mpc_oracle as orc       # noqa: E402


class _Box:
    def __init__(self, low, high):
        self.low = np.asarray(low, dtype=np.float32)
        self.high = np.asarray(high, dtype=np.float32)
        self.shape = self.low.shape


class FakeEnv:
    """HalfCheetah contract used by the controller: 6-d Box in [-1, 1]
    (gym HalfCheetah ctrlrange, float32 like gym.spaces.Box), 20-d obs."""

    def __init__(self, state_dim=20, action_dim=6):
        self.action_space = _Box(-np.ones(action_dim), np.ones(action_dim))
        self.observation_space = _Box(-np.inf * np.ones(state_dim), np.inf * np.ones(state_dim))


CASES = [
    # name, K, H, hidden, L, act, ln, seed, extra
    dict(name="tiny_tanh", K=16, H=3, hidden=64, L=2, act="tanh", ln=False, seed=1),
    dict(name="small_relu", K=64, H=5, hidden=128, L=2, act="relu", ln=False, seed=2),
    dict(name="small_ln_relu", K=48, H=4, hidden=96, L=2, act="relu", ln=True, seed=3),
    dict(name="deep3_tanh", K=32, H=4, hidden=64, L=3, act="tanh", ln=False, seed=4),
    dict(name="one_layer_tanh", K=32, H=6, hidden=128, L=1, act="tanh", ln=False, seed=5),
    dict(name="cfg1_2x500_tanh", K=1000, H=15, hidden=500, L=2, act="tanh", ln=False, seed=6),
    dict(name="cfg2_2x500_tanh", K=4096, H=20, hidden=500, L=2, act="tanh", ln=False, seed=7),
    dict(name="ppo_defaults_2x256_relu_ln", K=400, H=7, hidden=256, L=2, act="relu", ln=True, seed=8),
    dict(name="tie_lower_index", K=256, H=6, hidden=128, L=2, act="tanh", ln=False, seed=9, inject="tie"),
    dict(name="nan_candidates", K=128, H=5, hidden=64, L=2, act="tanh", ln=False, seed=10, inject="nan"),
    dict(name="device_rng_2x500", K=512, H=10, hidden=500, L=2, act="tanh", ln=False, seed=11,
         inject="philox", rng_seed=0x5EED_1234_ABCD, cand_offset=1000),
    dict(name="ragged_k1", K=1, H=4, hidden=64, L=2, act="tanh", ln=False, seed=12),
    dict(name="ragged_k17_h1", K=17, H=1, hidden=64, L=2, act="relu", ln=False, seed=13),
]

STORE_WEIGHTS_MAX_HIDDEN = 128
STORE_STATES_MAX = 64 * 8 * 20 * 8  # bytes budget ~80 KB


def try_trained_weights():
    """Only torch.load(weights_only=True) is an allowed loader for the pickle."""
    path = os.path.join(REF, "saved_data/ppo-mpc/vars.pkl")
    try:
        import torch
        torch.load(path, weights_only=True)
        return "loaded (unexpected)"
    except Exception as e:  # refused: plain pickle, not a torch archive
        msg = re.sub(r"\x1b\[[0-9;]*m", "", str(e)).splitlines()[0][:100]
        return f"refused by torch.load(weights_only=True): {type(e).__name__}: {msg}"


def run_case(c):
    S, A = 20, 6
    w = orc.synthetic_weights(S, A, c["hidden"], c["L"], c["act"], c["ln"], seed_base=1000 + 17 * c["seed"])
    norm = orc.synthetic_normalization(S, A, seed=7 + c["seed"])
    state = orc.synthetic_state(norm, seed=11 + c["seed"])
    dyn = orc.NumpyDynamics(w, norm)
    env = FakeEnv(S, A)
    ctrl = ref_controllers.MPCcontroller(env=env, dyn_model=dyn, horizon=c["H"],
                                         cost_fn=ref_costs.cheetah_cost_fn,
                                         num_simulated_paths=c["K"])
    captured = {}
    inject = c.get("inject")
    orig_sample = ctrl.sample_random_actions

    def sample_wrapper():
        ap = orig_sample()                     # consumes the global stream as the reference does
        if inject == "tie":
            # make a LOWER index an exact duplicate of the true best path -> it must win
            costs0, _ = orc.rollout(dyn, state, ap)
            best = int(np.argmin(costs0))
            lo = max(0, best // 2)
            ap[:, lo, :] = ap[:, best, :]
            ap[:, min(c["K"] - 1, best + 7), :] = ap[:, best, :]   # and a higher duplicate
            captured["tie_pair"] = (lo, best)
        elif inject == "nan":
            ap[2, 37, 0] = np.nan
            ap[1, 90, 3] = np.nan
        elif inject == "philox":
            ap = orc.device_rng_actions(c["rng_seed"], c["cand_offset"], c["K"], c["H"],
                                        env.action_space.low, env.action_space.high)
        captured["actions"] = ap
        return ap

    ctrl.sample_random_actions = sample_wrapper
    orig_traj = ref_controllers.trajectory_cost_fn

    def traj_wrapper(cost_fn, states, actions, next_states):
        out = orig_traj(cost_fn, states, actions, next_states)
        captured["costs"] = np.array(out, dtype=np.float64, copy=True)
        captured["states"] = np.concatenate([states, next_states[-1:]], axis=0)
        return out

    ref_controllers.trajectory_cost_fn = traj_wrapper
    try:
        np.random.seed(c["seed"])
        opt_action = ctrl.get_action(state)
        next_draw = np.random.random()          # identifies the RNG stream position afterwards
    finally:
        ref_controllers.trajectory_cost_fn = orig_traj

    costs = captured["costs"]
    order = np.sort(costs[~np.isnan(costs)])
    top2_gap = float(order[1] - order[0]) if order.size > 1 else float("inf")
    near = orc.near_threshold_mask(captured["states"])
    out = dict(
        meta=json.dumps(dict(c, S=S, A=A, weight_digest=w.digest(),
                             weight_seed_base=1000 + 17 * c["seed"], norm_seed=7 + c["seed"],
                             state_seed=11 + c["seed"])),
        state=state,
        mean_obs=norm[0], std_obs=norm[1], mean_action=norm[2], std_action=norm[3],
        mean_deltas=norm[8], std_deltas=norm[9],
        costs=costs,
        argmin=np.int64(np.argmin(costs)),
        opt_action=np.asarray(opt_action, dtype=np.float64),
        top2_gap=np.float64(top2_gap),
        near_threshold=near,
        next_draw=np.float64(next_draw),
        action_digest=np.frombuffer(
            __import__("hashlib").sha256(np.ascontiguousarray(captured["actions"]).tobytes()).digest(),
            dtype=np.uint8),
    )
    if "tie_pair" in captured:
        out["tie_pair"] = np.asarray(captured["tie_pair"], dtype=np.int64)
    if c["hidden"] <= STORE_WEIGHTS_MAX_HIDDEN:
        for i, k in enumerate(w.kernels):
            out[f"W{i}"] = k
            out[f"b{i}"] = w.biases[i]
        if w.layer_norm:
            for i in range(w.n_layers):
                out[f"ln_g{i}"] = w.ln_gamma[i]
                out[f"ln_b{i}"] = w.ln_beta[i]
    if captured["states"].nbytes <= STORE_STATES_MAX:
        out["states"] = captured["states"]
    # sanity: the build's oracle restatement reproduces the reference bit-exactly
    rc, _ = orc.rollout(dyn, state, captured["actions"])
    assert np.array_equal(rc, costs, equal_nan=True), c["name"]
    return out


POLICY_CASES = [
    dict(name="policy_explore05_relu_ln", K=256, H=6, hidden=256, L=2, act="relu", ln=True, seed=21, explore=0.5,
         ph=128, pl=2),
    dict(name="policy_explore03_tanh", K=128, H=5, hidden=500, L=2, act="tanh", ln=False, seed=22, explore=0.3,
         ph=128, pl=2),
    dict(name="policy_explore0_pure", K=64, H=4, hidden=128, L=2, act="relu", ln=False, seed=23, explore=0.0,
         ph=64, pl=1),
    dict(name="policy_explore1_pure_expl", K=96, H=4, hidden=256, L=2, act="tanh", ln=False, seed=24, explore=1.0,
         ph=128, pl=2),
]


def run_policy_case(c):
    """controllers.MPCcontrollerPolicyNet (controllers.py:160-237), self_exp=False."""
    S, A = 20, 6
    w = orc.synthetic_weights(S, A, c["hidden"], c["L"], c["act"], c["ln"], seed_base=1000 + 17 * c["seed"])
    norm = orc.synthetic_normalization(S, A, seed=7 + c["seed"])
    state = orc.synthetic_state(norm, seed=11 + c["seed"])
    pw = orc.synthetic_policy(S, A, c["ph"], c["pl"], seed=500 + c["seed"])
    dyn, pol = orc.NumpyDynamics(w, norm), orc.NumpyPolicy(pw)
    env = FakeEnv(S, A)
    ctrl = ref_controllers.MPCcontrollerPolicyNet(env=env, dyn_model=dyn, policy_net=pol, explore=c["explore"],
                                                  self_exp=False, horizon=c["H"], cost_fn=ref_costs.cheetah_cost_fn,
                                                  num_simulated_paths=c["K"])
    captured = {}
    orig_traj = ref_controllers.trajectory_cost_fn

    def traj_wrapper(cost_fn, states, actions, next_states):
        out = orig_traj(cost_fn, states, actions, next_states)
        captured["costs"] = np.array(out, dtype=np.float64, copy=True)
        captured["states"] = np.concatenate([states, next_states[-1:]], axis=0)
        captured["actions"] = np.array(actions, copy=True)
        return out

    ref_controllers.trajectory_cost_fn = traj_wrapper
    try:
        np.random.seed(c["seed"])
        opt_action = ctrl.get_action(state)
        next_draw = np.random.random()
    finally:
        ref_controllers.trajectory_cost_fn = orig_traj
    costs = captured["costs"]
    order = np.sort(costs[~np.isnan(costs)])
    np.random.seed(c["seed"])
    a2, i2, c2 = orc.policy_get_action(dyn, pol, state, c["H"], c["K"], env.action_space.low,
                                       env.action_space.high, c["explore"])
    assert np.array_equal(c2, costs) and np.array_equal(a2, opt_action), c["name"]   # restatement is exact
    out = dict(
        meta=json.dumps(dict(c, S=S, A=A, weight_digest=w.digest(), weight_seed_base=1000 + 17 * c["seed"],
                             norm_seed=7 + c["seed"], state_seed=11 + c["seed"], policy_seed=500 + c["seed"],
                             policy=True)),
        state=state, mean_obs=norm[0], std_obs=norm[1], mean_action=norm[2], std_action=norm[3],
        mean_deltas=norm[8], std_deltas=norm[9],
        costs=costs, argmin=np.int64(np.argmin(costs)), opt_action=np.asarray(opt_action, dtype=np.float64),
        top2_gap=np.float64(order[1] - order[0]), near_threshold=orc.near_threshold_mask(captured["states"]),
        next_draw=np.float64(next_draw),
        first_actions=captured["actions"][0],
        action_digest=np.frombuffer(
            __import__("hashlib").sha256(np.ascontiguousarray(captured["actions"]).tobytes()).digest(), dtype=np.uint8),
    )
    for i, k in enumerate(pw.kernels):
        out[f"PW{i}"] = k
        out[f"PB{i}"] = pw.biases[i]
    out["P_ob_mean"], out["P_ob_std"], out["P_logstd"] = pw.ob_mean, pw.ob_std, pw.logstd
    return out


def main():
    note = try_trained_weights()
    print("vars.pkl:", note)
    with open(os.path.join(HERE, "PROVENANCE.json"), "w") as f:
        json.dump(dict(generator="tests/golden/gen_golden.py",
                       reference_files=["controllers.py", "cost_functions.py"],
                       dynamics="oracle.NumpyDynamics (TF1 absent; restatement of dynamics.py:54-71,106-119)",
                       numpy=np.__version__, trained_weights=note,
                       cases=[c["name"] for c in CASES] + [c["name"] for c in POLICY_CASES],
                       policy_cases="controllers.MPCcontrollerPolicyNet with oracle.NumpyPolicy (MlpPolicy.act "
                                    "deterministic branch, ppo_bc_policy.py:54-88,174-185; TF/baselines absent)"),
                  f, indent=1)
    for c in POLICY_CASES:
        out = run_policy_case(c)
        np.savez_compressed(os.path.join(HERE, f"{c['name']}.npz"), **out)
        print(f"{c['name']:32s} K={c['K']:5d} H={c['H']:3d} argmin={int(out['argmin']):5d} "
              f"gap={float(out['top2_gap']):.4g} near={int(out['near_threshold'].sum())}")
    for c in CASES:
        out = run_case(c)
        np.savez_compressed(os.path.join(HERE, f"{c['name']}.npz"), **out)
        print(f"{c['name']:32s} K={c['K']:5d} H={c['H']:3d} argmin={int(out['argmin']):5d} "
              f"gap={float(out['top2_gap']):.4g} near={int(out['near_threshold'].sum())}")


if __name__ == "__main__":
    main()
