"""Cost-function objects with the reference's API (cost_functions.py:9-63).

``MPCcontroller`` receives ``cost_fn`` as an argument (controllers.py:32) and
the driver passes ``cost_functions.cheetah_cost_fn`` (train_mpc_ppo.py:515).
The rollout engine fuses that cost into the HIP kernel; these NumPy callables
exist so user code can keep importing and passing them, and so a caller can
score a trajectory the engine returns in trajectory mode.  ``is_cheetah_cost``
decides whether a given callable may be fused.
"""
from __future__ import annotations

import numpy as np


def cheetah_cost_fn(state, action, next_state):
    """cost_functions.py:9-52: heading penalties (+10 each) minus torso progress / 0.01."""
    if len(state.shape) > 1:
        heading_penalty_factor = 10
        scores = np.zeros((state.shape[0],))
        scores[state[:, 5] >= 0.2] += heading_penalty_factor
        scores[state[:, 6] >= 0] += heading_penalty_factor
        scores[state[:, 7] >= 0] += heading_penalty_factor
        scores -= (next_state[:, 17] - state[:, 17]) / 0.01
        return scores
    heading_penalty_factor = 10
    score = 0
    if state[5] >= 0.2:
        score += heading_penalty_factor
    if state[6] >= 0:
        score += heading_penalty_factor
    if state[7] >= 0:
        score += heading_penalty_factor
    score -= (next_state[17] - state[17]) / 0.01
    return score


cheetah_cost_fn.__bcmpc_fused__ = "cheetah"


def trajectory_cost_fn(cost_fn, states, actions, next_states):
    """cost_functions.py:59-63: sum of per-step costs over the horizon."""
    trajectory_cost = 0
    for i in range(len(actions)):
        trajectory_cost += cost_fn(states[i], actions[i], next_states[i])
    return trajectory_cost


_PROBED: dict = {}     # (cost_fn, state_dim, action_dim) -> verdict of the probe below


def is_cheetah_cost(cost_fn, state_dim: int = 20, action_dim: int = 6) -> bool:
    """True when ``cost_fn`` computes exactly cost_functions.cheetah_cost_fn.

    Our own function is recognised by its marker.  Any other callable named
    ``cheetah_cost_fn`` (e.g. the reference module's) must also reproduce the
    fused formula bit-for-bit on a probe batch that straddles every threshold.
    """
    if getattr(cost_fn, "__bcmpc_fused__", None) == "cheetah":
        return True
    if getattr(cost_fn, "__name__", "") != "cheetah_cost_fn" or state_dim < 18:
        return False
    try:
        return _PROBED[(cost_fn, state_dim, action_dim)]    # probed once per function (every env step asks)
    except (KeyError, TypeError):
        pass
    verdict = _probe(cost_fn, state_dim, action_dim)
    try:
        _PROBED[(cost_fn, state_dim, action_dim)] = verdict
    except TypeError:                                       # unhashable callable
        pass
    return verdict


def _probe(cost_fn, state_dim: int, action_dim: int) -> bool:
    rs = np.random.RandomState(20240601)
    s = rs.standard_normal((64, state_dim)) * 0.3
    s[:8, 5] = 0.2
    s[8:16, 6] = 0.0
    s[16:24, 7] = 0.0
    ns = s + rs.standard_normal((64, state_dim)) * 0.01
    a = rs.uniform(-1, 1, (64, action_dim))
    try:
        got = np.asarray(cost_fn(s, a, ns), dtype=np.float64)
    except Exception:
        return False
    want = cheetah_cost_fn(s, a, ns)
    return got.shape == want.shape and bool(np.array_equal(got, want))
