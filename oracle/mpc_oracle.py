"""CPU oracle for the random-shooting MPC hot path -- TEST INFRASTRUCTURE ONLY.

This module is the *checker*, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py`` may
import it.  The shipped path (``bc_mpc_amd``) never imports anything under
``oracle/`` and fails loudly when its HIP library is missing.

It is a NumPy restatement of the reference path, function by function:

* ``NumpyDynamics.predict``   <- ``dynamics.py:106-119`` (NNDynamicsModel.predict):
  f64 normalisation, cast to f32 at the TF placeholder feed
  (``dynamics.py:23-24``), f32 MLP, f64 de-normalisation + residual add.
* ``NumpyDynamics.mlp``       <- ``dynamics.py:54-71`` (build_network):
  ``tf.layers.dense`` == ``x @ W + b`` with W stored ``[in, out]``; optional
  ``tf.contrib.layers.layer_norm`` after each hidden activation
  (``dynamics.py:68-69``; TF1 defaults: last-axis moments, eps 1e-12,
  ``x*inv + (beta - mean*inv)`` with ``inv = rsqrt(var+eps)*gamma``).
* ``cheetah_cost_fn``         <- ``cost_functions.py:9-52``.
* ``trajectory_cost_fn``      <- ``cost_functions.py:59-63``.
* ``get_action``              <- ``controllers.py:43-88`` (MPCcontroller).
* ``policy_get_action``       <- ``controllers.py:160-237`` (MPCcontrollerPolicyNet, self_exp=False).
* ``NumpyRewardDynamics``     <- ``dynamics.py:121-238`` (NNDynamicsRewardModel two-head net).
* ``reward_get_action``       <- ``controllers.py:90-158`` (MPCcontrollerReward, argmax).
* ``policy_reward_get_action``<- ``controllers.py:289-363`` (MPCcontrollerPolicyNetReward).
* ``mcts_get_action``         <- ``controllers.py:365-457`` (MCTScontrollerPolicyNetReward), given the
  first-stage actions (the stochastic policy's TF draws are not restatable; the engine's Philox
  normals are, ``device_rng_normals``).
* ``cem_*``                   <- no reference (BASELINE cfg5 CEM): the engine's own CEM semantics
  (DESIGN.md "CEM"), restated exactly; parity there is self-consistency, not reference-pinned.

Parity status: the controller / cost / RNG half is PINNED bit-exactly against
fixtures produced by running the reference's own ``controllers.py`` +
``cost_functions.py`` (``tests/golden/gen_golden.py``).  The MLP half lives in
TensorFlow 1.x inside the reference, which is absent (version unpinned, no
reference test pins it); it is restated here from ``dynamics.py:54-71`` and is
therefore pinned only through this restatement (fp32 tolerance).
"""
from __future__ import annotations

import hashlib
from dataclasses import dataclass, field
from typing import List, Optional, Sequence

import numpy as np

NORM_EPS = 1e-10          # dynamics.py:109-110 (std + 1e-10)
LN_EPS = 1e-12            # tf.contrib.layers.layer_norm default variance_epsilon (TF1)
HEADING_PENALTY = 10      # cost_functions.py:12
COST_DT = 0.01            # cost_functions.py:28


# ----------------------------------------------------------------------------
# cost_functions.py restatement
# ----------------------------------------------------------------------------
def cheetah_cost_fn(state, action, next_state):
    """Restates ``cost_functions.cheetah_cost_fn`` (cost_functions.py:9-52)."""
    if len(state.shape) > 1:                          # batched branch :10-30
        scores = np.zeros((state.shape[0],))
        scores[state[:, 5] >= 0.2] += HEADING_PENALTY  # :16-18 front leg
        scores[state[:, 6] >= 0] += HEADING_PENALTY    # :20-22 front shin
        scores[state[:, 7] >= 0] += HEADING_PENALTY    # :24-26 front foot
        scores -= (next_state[:, 17] - state[:, 17]) / COST_DT   # :28
        return scores
    score = 0                                          # scalar branch :32-52
    if state[5] >= 0.2:
        score += HEADING_PENALTY
    if state[6] >= 0:
        score += HEADING_PENALTY
    if state[7] >= 0:
        score += HEADING_PENALTY
    score -= (next_state[17] - state[17]) / COST_DT
    return score


def trajectory_cost_fn(cost_fn, states, actions, next_states):
    """Restates ``cost_functions.trajectory_cost_fn`` (cost_functions.py:59-63)."""
    trajectory_cost = 0
    for i in range(len(actions)):
        trajectory_cost += cost_fn(states[i], actions[i], next_states[i])
    return trajectory_cost


# ----------------------------------------------------------------------------
# dynamics.py restatement
# ----------------------------------------------------------------------------
@dataclass
class MLPWeights:
    """Dense stack ``26 -> h (x L) -> 20`` in TF layout (kernel ``[in, out]``)."""
    kernels: List[np.ndarray]
    biases: List[np.ndarray]
    activation: str = "tanh"                     # "tanh" | "relu"
    ln_gamma: Optional[List[np.ndarray]] = None  # one per hidden layer when LN is on
    ln_beta: Optional[List[np.ndarray]] = None

    @property
    def n_layers(self) -> int:
        return len(self.kernels) - 1

    @property
    def hidden(self) -> int:
        return int(self.kernels[0].shape[1])

    @property
    def layer_norm(self) -> bool:
        return self.ln_gamma is not None

    def digest(self) -> str:
        h = hashlib.sha256()
        for a in list(self.kernels) + list(self.biases) + list(self.ln_gamma or []) + list(self.ln_beta or []):
            h.update(np.ascontiguousarray(a, dtype=np.float32).tobytes())
        h.update(self.activation.encode())
        return h.hexdigest()


def _act(x: np.ndarray, kind: str) -> np.ndarray:
    if kind == "tanh":
        return np.tanh(x)
    if kind == "relu":
        return np.maximum(x, np.float32(0))
    raise ValueError(kind)


def layer_norm_tf1(x: np.ndarray, gamma: np.ndarray, beta: np.ndarray) -> np.ndarray:
    """tf.contrib.layers.layer_norm (TF1) over the last axis, f32.

    nn.moments -> mean, mean(squared_difference(x, mean)); then
    nn.batch_normalization: inv = rsqrt(var + eps) * gamma;
    y = x * inv + (beta - mean * inv).
    """
    x = x.astype(np.float32, copy=False)
    mean = np.mean(x, axis=-1, keepdims=True, dtype=np.float32)
    var = np.mean(np.square(x - mean), axis=-1, keepdims=True, dtype=np.float32)
    inv = (np.float32(1) / np.sqrt(var + np.float32(LN_EPS))) * gamma.astype(np.float32)
    return x * inv + (beta.astype(np.float32) - mean * inv)


class NumpyDynamics:
    """Duck-typed stand-in for ``dynamics.NNDynamicsModel`` (dynamics.py:7-119).

    Exposes the same attributes ``MPCcontroller`` and the build's weight
    adapter read: ``mean_obs, std_obs, mean_action, std_action, mean_deltas,
    std_deltas`` (dynamics.py:41) and ``predict`` (dynamics.py:106).
    """

    def __init__(self, weights: MLPWeights, normalization: Sequence[np.ndarray]):
        (self.mean_obs, self.std_obs, self.mean_action, self.std_action,
         self.mean_reward, self.std_reward, self.mean_nxt_state, self.std_nxt_state,
         self.mean_deltas, self.std_deltas) = normalization
        self.weights = weights

    # dynamics.py:54-71
    def mlp(self, x32: np.ndarray) -> np.ndarray:
        w = self.weights
        out = x32
        for li in range(w.n_layers):
            out = out @ w.kernels[li] + w.biases[li]          # tf.layers.dense
            out = _act(out, w.activation)
            if w.layer_norm:                                   # FLAGS.LAYER_NORM
                out = layer_norm_tf1(out, w.ln_gamma[li], w.ln_beta[li])
        out = out @ w.kernels[-1] + w.biases[-1]               # output_activation=None
        return out.astype(np.float32, copy=False)

    # dynamics.py:106-119
    def predict(self, unnormalized_state, unnormalized_action):
        normalized_state = (unnormalized_state - self.mean_obs) / (self.std_obs + NORM_EPS)
        normalized_action = (unnormalized_action - self.mean_action) / (self.std_action + NORM_EPS)
        # feed_dict into tf.float32 placeholders (dynamics.py:23-24) then tf.concat (:26)
        x = np.concatenate([np.asarray(normalized_state).astype(np.float32),
                            np.asarray(normalized_action).astype(np.float32)], axis=1)
        normalized_state_delta = self.mlp(x)
        unnormalized_state_delta = normalized_state_delta * self.std_deltas + self.mean_deltas
        return unnormalized_state + unnormalized_state_delta


class NumpyDynamicsF64(NumpyDynamics):
    """The same net evaluated in f64 (matmuls, activation, LayerNorm), the output rounded to f32 as the
    reference's feed / fetch do -- NOT the reference's arithmetic: a yardstick for how strongly a fixture's
    dynamics amplify the MLP's f32 rounding over the horizon (``conditioning`` in tests/golden/, round 6).
    Any implementation that rounds differently from TF's f32 order inherits at least that spread."""

    def mlp(self, x32: np.ndarray) -> np.ndarray:
        w = self.weights
        out = np.asarray(x32, dtype=np.float64)
        for li in range(w.n_layers):
            out = out @ w.kernels[li].astype(np.float64) + w.biases[li].astype(np.float64)
            out = np.tanh(out) if w.activation == "tanh" else np.maximum(out, 0.0)
            if w.layer_norm:
                m = out.mean(axis=-1, keepdims=True)
                v = np.square(out - m).mean(axis=-1, keepdims=True)
                out = (out - m) / np.sqrt(v + LN_EPS) * w.ln_gamma[li].astype(np.float64) + \
                    w.ln_beta[li].astype(np.float64)
        out = out @ w.kernels[-1].astype(np.float64) + w.biases[-1].astype(np.float64)
        return out.astype(np.float32)


class NumpyDynamicsChunked(NumpyDynamics):
    """The reference's f32 MLP with every dense layer's k-sum split into ``chunks`` partial f32 GEMMs added in
    f32 (in reverse chunk order with ``reverse``): the same arithmetic type as TF's, another summation order --
    a second yardstick beside NumpyDynamicsF64 for a fixture's rounding spread (``conditioning``)."""

    def __init__(self, weights, normalization, chunks=4, reverse=False):
        super().__init__(weights, normalization)
        self.chunks, self.reverse = int(chunks), bool(reverse)

    def _mm(self, a, W):
        if self.chunks <= 0:                       # one product at a time in k order (a sequential f32 chain)
            acc = np.zeros((a.shape[0], W.shape[1]), np.float32)
            for k in range(a.shape[1]):
                acc = (acc + (a[:, k:k + 1] * W[k]).astype(np.float32)).astype(np.float32)
            return acc
        q = np.linspace(0, a.shape[1], self.chunks + 1).astype(int)
        acc = np.zeros((a.shape[0], W.shape[1]), np.float32)
        order = range(self.chunks)[::-1] if self.reverse else range(self.chunks)
        for i in order:
            acc = (acc + (a[:, q[i]:q[i + 1]] @ W[q[i]:q[i + 1]]).astype(np.float32)).astype(np.float32)
        return acc

    def mlp(self, x32: np.ndarray) -> np.ndarray:
        w = self.weights
        out = x32
        for li in range(w.n_layers):
            out = _act(self._mm(out, w.kernels[li]) + w.biases[li], w.activation)
            if w.layer_norm:
                out = layer_norm_tf1(out, w.ln_gamma[li], w.ln_beta[li])
        return (self._mm(out, w.kernels[-1]) + w.biases[-1]).astype(np.float32)


def conditioning(weights, normalization, state, action_paths, costs) -> np.ndarray:
    """Per candidate, the largest |cost - costs| over five other roundings of the same net (f64 arithmetic;
    f32 with the k-sums in 4 chunks, 4 chunks reversed, 2 chunks, and one product at a time in k order): how
    far these dynamics carry a change of rounding order over the horizon -- any implementation that does not
    replay TF's own f32 order inherits that spread (tests/golden, round 6)."""
    dyns = [NumpyDynamicsF64(weights, normalization), NumpyDynamicsChunked(weights, normalization, 4),
            NumpyDynamicsChunked(weights, normalization, 4, reverse=True), NumpyDynamicsChunked(weights, normalization, 2),
            NumpyDynamicsChunked(weights, normalization, 0)]
    return np.max([np.abs(rollout(d, state, action_paths)[0] - costs) for d in dyns], axis=0)


# ----------------------------------------------------------------------------
# controllers.py restatement (MPCcontroller, controllers.py:26-88)
# ----------------------------------------------------------------------------
def rollout(dyn: NumpyDynamics, state, action_paths, cost_fn=cheetah_cost_fn):
    """Body of ``MPCcontroller.get_action`` after sampling (controllers.py:62-82).

    ``state`` is ``(S,)`` (tiled K times, controllers.py:63) or ``(K, S)``.
    Returns ``(costs[K] f64, states_paths_all[H+1, K, S] f64)``.
    """
    H, K, _ = action_paths.shape
    state = np.asarray(state)
    states = np.tile(state, [K, 1]) if state.ndim == 1 else state
    states_paths_all = [states]
    for i in range(H):
        states = dyn.predict(states, action_paths[i, :, :])
        states_paths_all.append(states)
    states_paths_all = np.asarray(states_paths_all)
    costs = trajectory_cost_fn(cost_fn, states_paths_all[:-1], action_paths, states_paths_all[1:])
    return costs, states_paths_all


def get_action(dyn: NumpyDynamics, state, horizon: int, num_simulated_paths: int,
               low, high, cost_fn=cheetah_cost_fn, rng=None):
    """``MPCcontroller.get_action`` (controllers.py:57-88), returning extras.

    ``rng`` defaults to the global legacy ``np.random`` stream, exactly like
    ``controllers.py:53``.  Returns ``(opt_action f64 (A,), argmin, costs)``.
    """
    rng = np.random if rng is None else rng
    action_paths = rng.uniform(low=low, high=high, size=[horizon, num_simulated_paths, len(high)])
    costs, _ = rollout(dyn, state, action_paths, cost_fn)
    i = int(np.argmin(costs))
    return action_paths[:, i, :][0].copy(), i, costs


# ----------------------------------------------------------------------------
# Policy-guided MPC (controllers.py:160-237) + the policy net (ppo_bc_policy.py)
# ----------------------------------------------------------------------------
@dataclass
class PolicyWeights:
    """MlpPolicy 'pi/pol' stack (ppo_bc_policy.py:66-80) + its obfilter.

    kernels/biases: fc1..fcL (tanh) then 'final' (no activation), TF layout
    [in, out]; ob_mean / ob_std: baselines RunningMeanStd.mean / .std as f32
    (mean = f32(sum/count); std = sqrt(max(f32(sumsq/count) - mean^2, 1e-2)));
    logstd: the DiagGaussian log-std variable (ppo_bc_policy.py:79)."""
    kernels: List[np.ndarray]
    biases: List[np.ndarray]
    ob_mean: np.ndarray
    ob_std: np.ndarray
    logstd: np.ndarray

    @property
    def n_layers(self) -> int:
        return len(self.kernels) - 1

    @property
    def hidden(self) -> int:
        return int(self.kernels[0].shape[1])


class NumpyPolicy:
    """Duck-typed stand-in for ppo_bc_policy.MlpPolicy.act (ppo_bc_policy.py:174-185),
    deterministic branch (``stochastic=False`` -> ``pd.mode()`` = the mean)."""

    def __init__(self, w: PolicyWeights):
        self.w = w

    def mean(self, ob) -> np.ndarray:
        ob = np.asarray(ob)
        if ob.ndim == 1:
            ob = ob[None]
        x = ob.astype(np.float32)                                   # tf.float32 placeholder 'ob' (:28)
        obz = np.clip((x - self.w.ob_mean) / self.w.ob_std, np.float32(-5.0), np.float32(5.0))   # :60
        last = obz
        for k, b in zip(self.w.kernels[:-1], self.w.biases[:-1]):  # :70-71
            last = np.tanh(last @ k + b)
        return (last @ self.w.kernels[-1] + self.w.biases[-1]).astype(np.float32)   # :72

    def act(self, ob, stochastic=True):
        if stochastic:
            raise NotImplementedError("TF's random_normal stream is not reproducible outside TF")
        return self.mean(ob), None


def policy_get_action(dyn: NumpyDynamics, policy, state, horizon: int, num_simulated_paths: int,
                      low, high, explore: float, cost_fn=cheetah_cost_fn, rng=None):
    """MPCcontrollerPolicyNet.get_action with self_exp=False (controllers.py:189-237).
    Returns ``(opt_action, argmin, costs)``."""
    rng = np.random if rng is None else rng
    exploration = rng.uniform(low=low, high=high, size=[horizon, num_simulated_paths, len(high)])   # :185
    states = np.tile(state, [num_simulated_paths, 1])
    states_paths_all, action_paths = [states], []
    for i in range(horizon):
        actions, _ = policy.act(states, stochastic=False)
        actions = (1 - explore) * actions + explore * exploration[i, :, :]                             # :208
        states = dyn.predict(states, actions)
        states_paths_all.append(states)
        action_paths.append(actions)
    states_paths_all = np.asarray(states_paths_all)
    action_paths = np.asarray(action_paths)
    costs = trajectory_cost_fn(cost_fn, states_paths_all[:-1], action_paths, states_paths_all[1:])
    i = int(np.argmin(costs))
    return action_paths[:, i, :][0].copy(), i, costs


def synthetic_policy(state_dim=20, action_dim=6, hidden=128, n_layers=2, seed=2024) -> PolicyWeights:
    """MlpPolicy-shaped weights (normc-like init, ppo_bc_policy.py:63-72) and an obfilter."""
    rs = np.random.RandomState(seed)
    dims = [state_dim] + [hidden] * n_layers + [action_dim]
    ks, bs = [], []
    for i in range(len(dims) - 1):
        k = rs.standard_normal((dims[i], dims[i + 1]))
        k *= (1.0 if i < n_layers else 0.5) / np.sqrt(np.square(k).sum(axis=0, keepdims=True))
        ks.append(k.astype(np.float32))
        bs.append((0.05 * rs.standard_normal(dims[i + 1])).astype(np.float32))
    count = 1000.0
    mean64 = 0.1 * rs.standard_normal(state_dim)
    sumsq = (np.square(mean64) + np.square(np.abs(rs.standard_normal(state_dim)) * 0.5 + 0.2)) * count
    mean = (mean64 * count / count).astype(np.float32)
    std = np.sqrt(np.maximum((sumsq / count).astype(np.float32) - np.square(mean), np.float32(1e-2)))
    logstd = (-0.5 + 0.1 * rs.standard_normal(action_dim)).astype(np.float32)
    return PolicyWeights(ks, bs, mean, std.astype(np.float32), logstd)


# ----------------------------------------------------------------------------
# Learned-reward MPC: NNDynamicsRewardModel (dynamics.py:121-238) +
# MPCcontrollerReward (controllers.py:90-158) / MPCcontrollerPolicyNetReward
# (controllers.py:289-363)
# ----------------------------------------------------------------------------
@dataclass
class RewardMLPWeights:
    """Two-head net of ``NNDynamicsRewardModel.build_network`` (dynamics.py:150-177),
    in TF variable-creation order:

    kernels/biases: ``dense`` (shared trunk, [S+A, h]), ``dense_1`` (delta hidden,
    [h, h]), ``dense_2`` (delta out, [h, S]), ``dense_3`` (reward hidden, [h, h]),
    ``dense_4`` (reward out, [h, 1]); tanh on every hidden layer (the default
    ``activation=tf.tanh``, dynamics.py:150).  ln_gamma/ln_beta (FLAGS.LAYER_NORM):
    ``LayerNorm`` (trunk), ``LayerNorm_1`` (delta head), ``LayerNorm_2`` (reward head).
    """
    kernels: List[np.ndarray]
    biases: List[np.ndarray]
    ln_gamma: Optional[List[np.ndarray]] = None
    ln_beta: Optional[List[np.ndarray]] = None
    activation: str = "tanh"

    @property
    def hidden(self) -> int:
        return int(self.kernels[0].shape[1])

    @property
    def layer_norm(self) -> bool:
        return self.ln_gamma is not None

    def digest(self) -> str:
        h = hashlib.sha256()
        for a in list(self.kernels) + list(self.biases) + list(self.ln_gamma or []) + list(self.ln_beta or []):
            h.update(np.ascontiguousarray(a, dtype=np.float32).tobytes())
        h.update(b"reward")
        return h.hexdigest()


class NumpyRewardDynamics(NumpyDynamics):
    """Duck-typed stand-in for ``dynamics.NNDynamicsRewardModel`` (dynamics.py:121-238):
    ``predict(s, a) -> (next_state [K,S] f64, reward [K,1] f64)``."""

    def __init__(self, weights: RewardMLPWeights, normalization: Sequence[np.ndarray]):
        super().__init__(weights, normalization)   # same 10-tuple order (dynamics.py:143)

    # dynamics.py:150-177 (LAYER_NORM branch :153-166, plain branch :167-174)
    def mlp(self, x32: np.ndarray):
        w = self.weights
        ln = w.layer_norm

        def dense_act(x, i, ln_i):
            y = np.tanh(x @ w.kernels[i] + w.biases[i])
            return layer_norm_tf1(y, w.ln_gamma[ln_i], w.ln_beta[ln_i]) if ln else y

        share = dense_act(x32, 0, 0)
        d = dense_act(share, 1, 1)
        d = (d @ w.kernels[2] + w.biases[2]).astype(np.float32, copy=False)
        r = dense_act(share, 3, 2)
        r = (r @ w.kernels[4] + w.biases[4]).astype(np.float32, copy=False)
        return d, r

    # dynamics.py:225-238
    def predict(self, unnormalized_state, unnormalized_action):
        normalized_state = (unnormalized_state - self.mean_obs) / (self.std_obs + NORM_EPS)
        normalized_action = (unnormalized_action - self.mean_action) / (self.std_action + NORM_EPS)
        x = np.concatenate([np.asarray(normalized_state).astype(np.float32),
                            np.asarray(normalized_action).astype(np.float32)], axis=1)
        normalized_state_delta, normalized_reward = self.mlp(x)
        unnormalized_state_delta = (normalized_state_delta * self.std_deltas) + self.mean_deltas   # denomalize :78
        unnormalized_nxt_state = unnormalized_state + unnormalized_state_delta
        unnormalized_reward = (normalized_reward * self.std_reward) + self.mean_reward
        return unnormalized_nxt_state, unnormalized_reward


def reward_rollout(dyn: NumpyRewardDynamics, state, action_paths, gamma: float = 1.0):
    """Body of ``MPCcontrollerReward.get_action`` after sampling (controllers.py:131-152).
    Returns ``(rewards[K] f64, states_paths_all[H+1, K, S])``; the sum over steps is
    NumPy's axis-0 reduction (sequential in h)."""
    H, K, _ = action_paths.shape
    states = np.tile(state, [K, 1])
    paths, rewards_all = [states], []
    for i in range(H):
        states, reward = dyn.predict(states, action_paths[i, :, :])
        paths.append(states)
        rewards_all.append(reward * gamma ** i)
    rewards_all = np.sum(np.asarray(rewards_all), axis=0).reshape([-1])
    return rewards_all, np.asarray(paths)


def env_sample_actions(sample, horizon: int, num_simulated_paths: int) -> np.ndarray:
    """``MPCcontrollerReward.sample_random_actions`` (controllers.py:108-119): K*H calls
    of ``env.action_space.sample()`` (n-major), reshaped to ``[H, K, A]``."""
    actions = [sample() for _ in range(num_simulated_paths) for _ in range(horizon)]
    return np.reshape(np.asarray(actions), [horizon, num_simulated_paths, -1])


def reward_get_action(dyn: NumpyRewardDynamics, sample, state, horizon: int, num_simulated_paths: int,
                      gamma: float = 1.0):
    """``MPCcontrollerReward.get_action`` (controllers.py:121-158): argmax of the
    discounted predicted reward.  Returns ``(opt_action, argmax, rewards, action_paths)``."""
    action_paths = env_sample_actions(sample, horizon, num_simulated_paths)
    rewards, _ = reward_rollout(dyn, state, action_paths, gamma)
    i = int(np.argmax(rewards))
    return action_paths[:, i, :][0].copy(), i, rewards, action_paths


def policy_reward_get_action(dyn: NumpyRewardDynamics, policy, state, horizon: int, num_simulated_paths: int,
                             low, high, explore: float, rng=None):
    """``MPCcontrollerPolicyNetReward.get_action`` with self_exp=False (controllers.py:318-363):
    undiscounted reward sum, argmax.  Returns ``(opt_action, argmax, rewards, action_paths)``."""
    rng = np.random if rng is None else rng
    exploration = rng.uniform(low=low, high=high, size=[horizon, num_simulated_paths, len(high)])   # :314
    states = np.tile(state, [num_simulated_paths, 1])
    rewards_all, action_paths = [], []
    for i in range(horizon):
        actions, _ = policy.act(states, stochastic=False)
        actions = (1 - explore) * actions + explore * exploration[i, :, :]                             # :338
        states, reward = dyn.predict(states, actions)
        action_paths.append(actions)
        rewards_all.append(reward)
    action_paths = np.asarray(action_paths)
    rewards = np.sum(np.asarray(rewards_all), axis=0).reshape([-1])
    i = int(np.argmax(rewards))
    return action_paths[:, i, :][0].copy(), i, rewards, action_paths


def mcts_get_action(dyn: NumpyRewardDynamics, policy, state, horizon: int, action_1s, random_path_per_action: int):
    """``MCTScontrollerPolicyNetReward.get_action`` (controllers.py:397-457) with the first-stage
    actions given (``action_1s``: N arrays of shape [1, A], controllers.py:405-414).  Each first
    action is scored by ``predict`` from the root (:416-418), its next state tiled R times (:421-424),
    the follow-up paths rolled with the DETERMINISTIC policy (:430-440), reward sums averaged over
    the R paths and added to the first reward (:442-449).  Returns ``(best, total_rewards,
    reward_1s, rewards_all [N, R])``."""
    state_init = np.expand_dims(state, axis=0)
    reward_1s, states_all_actions = [], []
    for action_1 in action_1s:
        state_1, reward_1 = dyn.predict(state_init, action_1)
        reward_1s.append(reward_1[0][0])
        states_all_actions.append(np.tile(state_1, [random_path_per_action, 1]))
    states = np.asarray(states_all_actions).reshape((-1, state.shape[0]))
    rewards_all = []
    for i in range(horizon):
        actions, _ = policy.act(states, stochastic=False)
        states, reward = dyn.predict(states, actions)
        rewards_all.append(reward)
    rewards_all = np.sum(np.asarray(rewards_all), axis=0)
    rewards_all = rewards_all.reshape((len(action_1s), -1))
    total_rewards = np.asarray(reward_1s) + np.mean(rewards_all, axis=1)
    return int(np.argmax(total_rewards)), total_rewards, np.asarray(reward_1s), rewards_all


def synthetic_reward_weights(state_dim=20, action_dim=6, hidden=500, layer_norm=False,
                             seed_base=3000) -> RewardMLPWeights:
    """Glorot-uniform kernels of the two-head net (TF default initializer), biases
    ~ 0.1 N(0,1); LN gamma ~ 1 + 0.1 N, beta ~ 0.1 N."""
    S, A, h = state_dim, action_dim, hidden
    dims = [(S + A, h), (h, h), (h, S), (h, h), (h, 1)]
    ks, bs = [], []
    for i, (fi, fo) in enumerate(dims):
        rs = np.random.RandomState(seed_base + i)
        lim = np.sqrt(6.0 / (fi + fo))
        ks.append(rs.uniform(-lim, lim, size=(fi, fo)).astype(np.float32))
        bs.append((0.1 * rs.standard_normal(fo)).astype(np.float32))
    gs = bts = None
    if layer_norm:
        rs = np.random.RandomState(seed_base + 99)
        gs = [(1.0 + 0.1 * rs.standard_normal(h)).astype(np.float32) for _ in range(3)]
        bts = [(0.1 * rs.standard_normal(h)).astype(np.float32) for _ in range(3)]
    return RewardMLPWeights(ks, bs, gs, bts)


# ----------------------------------------------------------------------------
# Philox4x32-10 restatement of the engine's device RNG ("perf" action mode)
# ----------------------------------------------------------------------------
_PH_M0, _PH_M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
_PH_W0, _PH_W1 = np.uint64(0x9E3779B9), np.uint64(0xBB67AE85)
_M32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 (Salmon et al., SC'11).  uint32 arrays in/out."""
    c0, c1, c2, c3 = (np.asarray(c, dtype=np.uint64) & _M32 for c in (c0, c1, c2, c3))
    k0 = np.uint64(k0) & _M32
    k1 = np.uint64(k1) & _M32
    for r in range(10):
        p0 = _PH_M0 * c0
        p1 = _PH_M1 * c2
        hi0, lo0 = p0 >> np.uint64(32), p0 & _M32
        hi1, lo1 = p1 >> np.uint64(32), p1 & _M32
        c0, c1, c2, c3 = (hi1 ^ c1 ^ k0) & _M32, lo1, (hi0 ^ c3 ^ k1) & _M32, lo0
        if r != 9:
            k0 = (k0 + _PH_W0) & _M32
            k1 = (k1 + _PH_W1) & _M32
    return [c.astype(np.uint32) for c in (c0, c1, c2, c3)]


def device_rng_actions(seed: int, cand_offset: int, K: int, H: int, low, high) -> np.ndarray:
    """Actions the engine draws on-device in RNG mode, as ``[H, K, A]`` f64.

    Counter = (lo32(g), hi32(g), h, j) for global candidate g, step h, draw j;
    key = (lo32(seed), hi32(seed)).  Each Philox block gives 4 u32 = two
    53-bit doubles built like NumPy's legacy ``random_sample``
    (``((a >> 5) * 67108864 + (b >> 6)) / 2**53``); action = low + (high-low)*u,
    the form of ``np.random.uniform`` used at controllers.py:53.
    """
    low = np.asarray(low, dtype=np.float64)
    high = np.asarray(high, dtype=np.float64)
    A = low.shape[0]
    ndraw = (A + 1) // 2
    g = (np.arange(K, dtype=np.uint64) + np.uint64(cand_offset))
    out = np.empty((H, K, A), dtype=np.float64)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    for h in range(H):
        u = np.empty((K, 2 * ndraw), dtype=np.float64)
        for j in range(ndraw):
            r = philox4x32_10(g & _M32, g >> np.uint64(32), np.full(K, h, np.uint64),
                              np.full(K, j, np.uint64), k0, k1)
            for p in range(2):
                a = (r[2 * p].astype(np.uint64) >> np.uint64(5)).astype(np.float64)
                b = (r[2 * p + 1].astype(np.uint64) >> np.uint64(6)).astype(np.float64)
                u[:, 2 * j + p] = (a * 67108864.0 + b) / 9007199254740992.0
        out[h] = low + (high - low) * u[:, :A]
    return out


POLICY_NORMAL_KEY_XOR = 0x9E3779B97F4A7C15


def device_rng_normals(seed: int, cand_offset: int, K: int, h: int, A: int) -> np.ndarray:
    """The N(0, 1) draws the engine's stochastic policy uses at step ``h`` (self_exp=True,
    controllers.py:202-203 -> ppo_bc_policy.py:174-185 ``act(stochastic=True)`` = DiagGaussianPd.sample
    = mean + exp(logstd) * N(0, 1); TF's own sampler is not restatable, so the engine draws with
    Philox), as ``[K, A]`` f64.

    Restates the kernel's ``rng_normal`` (csrc/device_common.h): key = seed ^ 0x9E3779B97F4A7C15,
    counter (lo32(g), hi32(g), h, 0x80000000 | j) for global candidate g; u1 = ((c0 >> 8) + 0.5) / 2^24,
    u2 = (c1 >> 8) / 2^24 (both exact); z = sqrt(-2 ln u1) cos(2 pi u2) (Box-Muller).  The kernel
    evaluates the transcendentals in f32 (a few ulp); this restatement does so in f64, so the two agree
    to ~1e-6 relative, not bitwise."""
    key = (seed ^ POLICY_NORMAL_KEY_XOR) & 0xFFFFFFFFFFFFFFFF
    k0, k1 = key & 0xFFFFFFFF, (key >> 32) & 0xFFFFFFFF
    g = np.arange(K, dtype=np.uint64) + np.uint64(cand_offset)
    out = np.empty((K, A), dtype=np.float64)
    for j in range(A):
        r = philox4x32_10(g & _M32, g >> np.uint64(32), np.full(K, h, np.uint64),
                          np.full(K, 0x80000000 | j, np.uint64), k0, k1)
        u1 = ((r[0] >> np.uint32(8)).astype(np.float64) + 0.5) / 16777216.0
        u2 = (r[1] >> np.uint32(8)).astype(np.float64) / 16777216.0
        out[:, j] = np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)
    return out


# ----------------------------------------------------------------------------
# CEM outer loop (BASELINE cfg5; NOT in the reference -- semantics defined in
# DESIGN.md "CEM" and restated here exactly as the engine computes them)
# ----------------------------------------------------------------------------
def cem_normals(seed: int, iteration: int, cand_offset: int, K: int, H: int, A: int, index=None) -> np.ndarray:
    """z = Irwin-Hall(12) - 6 per (h, k, j) as ``[H, K, A]`` f64: twelve 24-bit uniforms from
    three Philox blocks, counter (lo32(g), hi32(g), h, 0x40000000 | it<<8 | j<<2 | c); the
    integer sum is exact, so z is exact (engine: cem_normal, device_common.h).  Candidates
    are cand_offset + [0, K), or the global indices ``index`` when given."""
    if index is not None:
        g = np.asarray(index, dtype=np.uint64)
        K = g.shape[0]
    else:
        g = np.arange(K, dtype=np.uint64) + np.uint64(cand_offset)
    k0, k1 = seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF
    out = np.empty((H, K, A), dtype=np.float64)
    for h in range(H):
        for j in range(A):
            tot = np.zeros(K, dtype=np.uint64)
            for c in range(3):
                w3 = 0x40000000 | (iteration << 8) | (j << 2) | c
                r = philox4x32_10(g & _M32, g >> np.uint64(32), np.full(K, h, np.uint64),
                                  np.full(K, w3, np.uint64), k0, k1)
                for x in r:
                    tot += x.astype(np.uint64) >> np.uint64(8)
            out[h, :, j] = tot.astype(np.float64) * (1.0 / 16777216.0) - 6.0
    return out


def cem_actions(seed, iteration, cand_offset, K, H, mu, sigma, low, high, index=None) -> np.ndarray:
    """``np.clip(mu + sigma * z, low, high)`` as ``[H, K, A]`` (mu, sigma: ``[H, A]``)."""
    mu = np.asarray(mu, dtype=np.float64)
    sigma = np.asarray(sigma, dtype=np.float64)
    z = cem_normals(seed, iteration, cand_offset, K, H, mu.shape[1], index)
    return np.clip(mu[:, None, :] + sigma[:, None, :] * z, np.asarray(low, np.float64), np.asarray(high, np.float64))


def cem_select(costs, index, n_elite: int, maximize: bool = False) -> np.ndarray:
    """The n_elite best records (stable sort: NaN last, ties to the lower index; +-0
    equal), returned as global indices in ascending order (engine: select_kernel)."""
    costs = np.asarray(costs, dtype=np.float64)
    index = np.asarray(index, dtype=np.int64)
    keep = index >= 0
    costs, index = costs[keep], index[keep]
    pos = np.argsort(index, kind="stable")
    costs, index = costs[pos], index[pos]
    obj = -costs if maximize else costs
    order = np.argsort(obj, kind="stable")[:n_elite]
    return np.sort(index[order])


def _wave_sum(x: np.ndarray) -> float:
    """Lane l adds elements l, l+64, ... in order (from 0.0); the 64 partials are then
    combined by the xor butterfly (offsets 32, 16, ..., 1): p[:off] + p[off:2*off]."""
    p = np.zeros(64, dtype=np.float64)
    for start in range(0, x.shape[0], 64):
        chunk = x[start:start + 64]
        p[:chunk.shape[0]] = p[:chunk.shape[0]] + chunk
    off = 32
    while off >= 1:
        p = p[:off] + p[off:2 * off]
        off //= 2
    return float(p[0])


def cem_refit(elite_index, seed, iteration, mu, sigma, low, high, alpha: float):
    """Elite mean / std (np.std ddof 0, two passes) per (h, j) in the engine's reduction
    order, smoothed: new = alpha*old + (1-alpha)*stat (engine: refit_kernel)."""
    mu = np.asarray(mu, dtype=np.float64)
    sigma = np.asarray(sigma, dtype=np.float64)
    n = len(elite_index)
    if n == 0:
        return mu.copy(), sigma.copy()
    H, A = mu.shape
    acts = cem_actions(seed, iteration, 0, 0, H, mu, sigma, low, high, index=elite_index)   # [H, n, A]
    new_mu, new_sd = np.empty_like(mu), np.empty_like(sigma)
    beta = 1.0 - alpha
    for h in range(H):
        for j in range(A):
            a = acts[h, :, j]
            mean = _wave_sum(a) / float(n)
            d = a - mean
            sd = np.sqrt(_wave_sum(d * d) / float(n))
            new_mu[h, j] = alpha * mu[h, j] + beta * mean
            new_sd[h, j] = alpha * sigma[h, j] + beta * sd
    return new_mu, new_sd


def cem_get_action(score, state, H: int, K: int, low, high, iterations: int, n_elite: int, alpha: float,
                   seed: int, mu0, sigma0, maximize: bool = False):
    """The CEM loop the engine runs (bcmpc_cem_get_action).  ``score(state, actions [H,K,A])
    -> objective [K]`` (e.g. ``lambda s, a: rollout(dyn, s, a)[0]``).  Returns
    ``(first_action, position, objective_concat, mu, sigma, history)`` where position
    = iteration*K + candidate is np.argmin (np.argmax when maximize) over the
    iteration-major concatenation, and history holds each iteration's (mu, sigma)."""
    mu, sd = np.array(mu0, dtype=np.float64), np.array(sigma0, dtype=np.float64)
    objs, hist = [], []
    for it in range(iterations):
        hist.append((mu.copy(), sd.copy()))
        acts = cem_actions(seed, it, 0, K, H, mu, sd, low, high)
        obj = np.asarray(score(state, acts), dtype=np.float64)
        objs.append(obj)
        el = cem_select(obj, np.arange(K), n_elite, maximize)
        mu, sd = cem_refit(el, seed, it, mu, sd, low, high, alpha)
    flat = np.concatenate(objs)
    pos = int(np.argmax(flat) if maximize else np.argmin(flat))
    it, i = divmod(pos, K)
    first = cem_actions(seed, it, i, 1, 1, hist[it][0], hist[it][1], low, high)[0, 0]
    return first, pos, flat, mu, sd, hist


# ----------------------------------------------------------------------------
# Synthetic inputs
# ----------------------------------------------------------------------------
def synthetic_weights(state_dim=20, action_dim=6, hidden=500, n_layers=2,
                      activation="tanh", layer_norm=False, seed_base=1000) -> MLPWeights:
    """Glorot-uniform kernels (TF default initializer) from RandomState(1000+layer),
    biases ~ 0.1 N(0,1); LN gamma ~ 1 + 0.1 N, beta ~ 0.1 N (when enabled)."""
    dims = [state_dim + action_dim] + [hidden] * n_layers + [state_dim]
    ks, bs, gs, bts = [], [], [], []
    for li in range(len(dims) - 1):
        rs = np.random.RandomState(seed_base + li)
        lim = np.sqrt(6.0 / (dims[li] + dims[li + 1]))
        ks.append(rs.uniform(-lim, lim, size=(dims[li], dims[li + 1])).astype(np.float32))
        bs.append((0.1 * rs.standard_normal(dims[li + 1])).astype(np.float32))
        if layer_norm and li < n_layers:
            gs.append((1.0 + 0.1 * rs.standard_normal(dims[li + 1])).astype(np.float32))
            bts.append((0.1 * rs.standard_normal(dims[li + 1])).astype(np.float32))
    return MLPWeights(ks, bs, activation, gs if layer_norm else None, bts if layer_norm else None)


def synthetic_normalization(state_dim=20, action_dim=6, seed=7, reward=False):
    """The 10-tuple of utils.compute_normalization (utils.py:132-158), synthetic.
    ``reward=True`` also fills mean_reward / std_reward (shape (1,), utils.py:145,153)."""
    rs = np.random.RandomState(seed)
    mean_obs = 0.1 * rs.standard_normal(state_dim)
    std_obs = np.abs(rs.standard_normal(state_dim)) * 0.5 + 0.2
    mean_action = np.zeros(action_dim)
    std_action = np.full(action_dim, 1.0 / np.sqrt(3.0))
    mean_deltas = 0.005 * rs.standard_normal(state_dim)
    std_deltas = 0.05 * (np.abs(rs.standard_normal(state_dim)) + 0.2)
    mean_reward, std_reward = np.zeros(1), np.zeros(1)
    if reward:
        mean_reward = 0.3 * rs.standard_normal(1)
        std_reward = np.abs(rs.standard_normal(1)) + 0.5
    return [mean_obs, std_obs, mean_action, std_action, mean_reward, std_reward,
            mean_obs.copy(), std_obs.copy(), mean_deltas, std_deltas]


def synthetic_state(normalization, seed=11):
    rs = np.random.RandomState(seed)
    mean_obs, std_obs = normalization[0], normalization[1]
    return mean_obs + 0.5 * std_obs * rs.standard_normal(mean_obs.shape[0])


def near_threshold_mask(states_paths_all: np.ndarray, delta: float = 1e-4) -> np.ndarray:
    """Candidates whose cost has a +-10 penalty within ``delta`` of flipping
    (|s5-0.2|, |s6|, |s7| < delta at any of the H scored states)."""
    s = states_paths_all[:-1]
    m = (np.abs(s[..., 5] - 0.2) < delta) | (np.abs(s[..., 6]) < delta) | (np.abs(s[..., 7]) < delta)
    return m.any(axis=0)


def argmin_ref(costs: np.ndarray) -> int:
    """np.argmin semantics the engine must reproduce (first NaN, else first min)."""
    return int(np.argmin(costs))


# ----------------------------------------------------------------------------
# NNDynamicsModel.fit restatement (dynamics.py:44-52, 81-104) -- SURVEY 8f rank 4
# ----------------------------------------------------------------------------
# TF1 graph: loss = reduce_mean(squared_difference(delta, pred)); AdamOptimizer(lr)
# .minimize(loss).  The gradients below are the autodiff of exactly those ops,
# written out (TF is absent here: "parity unpinned" at the TF boundary, like the
# MLP itself); the Adam step is TF1's ApplyAdam kernel.

@dataclass
class AdamState:
    """tf.train.AdamOptimizer slots + the f32 beta-power variables (persist across fit calls)."""
    m: List[np.ndarray]
    v: List[np.ndarray]
    beta1_power: np.float32
    beta2_power: np.float32

    @classmethod
    def zeros_like(cls, params: Sequence[np.ndarray], beta1=0.9, beta2=0.999) -> "AdamState":
        return cls([np.zeros_like(p, dtype=np.float32) for p in params],
                   [np.zeros_like(p, dtype=np.float32) for p in params], np.float32(beta1), np.float32(beta2))


def fit_params(w: MLPWeights) -> List[np.ndarray]:
    """Trainable variables in TF creation order: per dense layer kernel, bias; per LN gamma... the
    order only matters for bookkeeping -- [W0, b0, ..., WL, bL] + [g0, be0, ...] (LN)."""
    ps = []
    for k, b in zip(w.kernels, w.biases):
        ps += [np.asarray(k, np.float32), np.asarray(b, np.float32)]
    if w.layer_norm:
        for g, be in zip(w.ln_gamma, w.ln_beta):
            ps += [np.asarray(g, np.float32), np.asarray(be, np.float32)]
    return ps


def _split_params(ps: Sequence[np.ndarray], L: int, ln: bool):
    ks = [ps[2 * i] for i in range(L + 1)]
    bs = [ps[2 * i + 1] for i in range(L + 1)]
    gs = [ps[2 * (L + 1) + 2 * i] for i in range(L)] if ln else None
    bes = [ps[2 * (L + 1) + 2 * i + 1] for i in range(L)] if ln else None
    return ks, bs, gs, bes


def fit_batch(normalization, states, actions, deltas):
    """dynamics.py:92-95: normalize(x, std, mean) = (x - mean)/(std + 1e-10) in f64, fed as f32."""
    (mean_obs, std_obs, mean_action, std_action, _mr, _sr, _mn, _sn, mean_deltas, std_deltas) = normalization
    ns = (np.asarray(states, np.float64) - mean_obs) / (std_obs + NORM_EPS)
    na = (np.asarray(actions, np.float64) - mean_action) / (std_action + NORM_EPS)
    nd = (np.asarray(deltas, np.float64) - mean_deltas) / (std_deltas + NORM_EPS)
    x0 = np.concatenate([ns.astype(np.float32), na.astype(np.float32)], axis=1)
    return x0, nd.astype(np.float32)


def fit_grads(ps: Sequence[np.ndarray], L: int, act: str, ln: bool, x0: np.ndarray, t: np.ndarray,
              dtype=np.float32):
    """Loss and d(loss)/d(params) for one batch (f32 throughout, TF op semantics; ``dtype``
    float64 only for the finite-difference check of the restated derivatives)."""
    f32 = dtype
    ks, bs, gs, bes = _split_params(ps, L, ln)
    hs, As, means, rss = [x0], [], [], []
    h = x0
    for l in range(L):
        z = h @ ks[l] + bs[l]
        a = (np.tanh(z) if act == "tanh" else np.maximum(z, f32(0))).astype(f32)
        As.append(a)
        if ln:
            mean = np.mean(a, axis=1, keepdims=True, dtype=f32)
            var = np.mean(np.square(a - mean), axis=1, keepdims=True, dtype=f32)
            rs = f32(1) / np.sqrt(var + f32(LN_EPS))
            inv = rs * gs[l]
            h = a * inv + (bes[l] - mean * inv)
            means.append(mean)
            rss.append(rs)
        else:
            h = a
        hs.append(h)
    p = h @ ks[L] + bs[L]
    n = p.size
    d = t - p
    loss = f32(np.mean(np.square(d), dtype=f32))
    dp = -((f32(2.0) * (f32(1.0) / f32(n))) * d)             # SquaredDifference / Mean grads
    gk = [None] * (L + 1)
    gb = [None] * (L + 1)
    gg = [None] * L if ln else None
    gbe = [None] * L if ln else None
    gk[L] = hs[L].T @ dp
    gb[L] = np.sum(dp, axis=0, dtype=f32)
    dh = dp @ ks[L].T
    for l in range(L - 1, -1, -1):
        a = As[l]
        if ln:
            mean, rs = means[l], rss[l]
            xhat = (a - mean) * rs
            gbe[l] = np.sum(dh, axis=0, dtype=f32)
            gg[l] = np.sum(dh * xhat, axis=0, dtype=f32)
            F = f32(a.shape[1])
            inv = rs * gs[l]
            dmean = -np.sum(dh * inv, axis=1, keepdims=True, dtype=f32)
            drs = np.sum(dh * (a - mean) * gs[l], axis=1, keepdims=True, dtype=f32)
            dvar = f32(-0.5) * drs * rs * rs * rs
            da = dh * inv + dmean / F + dvar * f32(2.0) * (a - mean) / F
        else:
            da = dh
        dz = da * (a > 0) if act == "relu" else da * (f32(1) - a * a)
        dz = dz.astype(f32)
        gk[l] = hs[l].T @ dz
        gb[l] = np.sum(dz, axis=0, dtype=f32)
        if l > 0:
            dh = dz @ ks[l].T
    grads = []
    for l in range(L + 1):
        grads += [gk[l].astype(f32), gb[l].astype(f32)]
    if ln:
        for l in range(L):
            grads += [gg[l], gbe[l]]
    return loss, grads


def adam_apply(ps: List[np.ndarray], grads: Sequence[np.ndarray], st: AdamState, lr: float,
               beta1=0.9, beta2=0.999, eps=1e-8) -> None:
    """TF1 ApplyAdam (training_ops.cc): lr_t = lr*sqrt(1-b2^t)/(1-b1^t) from the f32 beta
    powers; m += (g-m)(1-b1); v += (g^2-v)(1-b2); w -= (m lr_t)/(sqrt(v)+eps); then the
    powers are multiplied by beta (AdamOptimizer._finish)."""
    f32 = np.float32
    b1, b2 = f32(beta1), f32(beta2)
    lr_t = f32(lr) * np.sqrt(f32(1) - st.beta2_power) / (f32(1) - st.beta1_power)
    for i, g in enumerate(grads):
        st.m[i] = (st.m[i] + (g - st.m[i]) * (f32(1) - b1)).astype(f32)
        st.v[i] = (st.v[i] + (g * g - st.v[i]) * (f32(1) - b2)).astype(f32)
        ps[i] = (ps[i] - (st.m[i] * lr_t) / (np.sqrt(st.v[i]) + f32(eps))).astype(f32)
    st.beta1_power = f32(st.beta1_power * b1)
    st.beta2_power = f32(st.beta2_power * b2)


def fit(ps: List[np.ndarray], st: AdamState, L: int, act: str, ln: bool, normalization, data_states,
        data_actions, data_deltas, batches: Sequence[np.ndarray], lr: float):
    """dynamics.py:81-104 over explicit batch index lists; returns the per-step losses."""
    losses = []
    for idx in batches:
        x0, t = fit_batch(normalization, data_states[idx], data_actions[idx], data_deltas[idx])
        loss, grads = fit_grads(ps, L, act, ln, x0, t)
        adam_apply(ps, grads, st, lr)
        losses.append(loss)
    return losses


# ----------------------------------------------------------------------------
# NNDynamicsRewardModel.fit restatement (dynamics.py:153-160, 195-219) -- VERDICT r2 #4
# ----------------------------------------------------------------------------
# TF1 graph: loss = reduce_mean(sqdiff(delta, delta_pred)) + reduce_mean(sqdiff(reward, reward_pred))
# over the two-head net of build_network (dynamics.py:165-177: tanh trunk [+LN], delta head dense(h)
# tanh [+LN] -> dense(S), reward head dense(h) tanh [+LN] -> dense(1)); AdamOptimizer(lr).minimize.
# The gradients are the autodiff of those ops, as fit_grads; the trunk's output feeds both heads, so
# its gradient is the sum (AddN) of the heads' data gradients.  Parameters in TF creation order:
# [W0, b0, W1, b1, W2, b2, W3, b3, W4, b4] (+ [g0, be0, g1, be1, g2, be2] with LayerNorm).

def fit_reward_params(w: "RewardMLPWeights") -> List[np.ndarray]:
    ps = []
    for k, b in zip(w.kernels, w.biases):
        ps += [np.asarray(k, np.float32), np.asarray(b, np.float32)]
    if w.ln_gamma is not None:
        for g, be in zip(w.ln_gamma, w.ln_beta):
            ps += [np.asarray(g, np.float32), np.asarray(be, np.float32)]
    return ps


def fit_reward_batch(normalization, states, actions, rewards, deltas):
    """dynamics.py:201-205: every input normalised in f64 ((x - mean)/(std + 1e-10)), fed as f32; the
    reward reshaped to [-1, 1] (:210)."""
    x0, t = fit_batch(normalization, states, actions, deltas)
    mean_r, std_r = normalization[4], normalization[5]
    nr = (np.asarray(rewards, np.float64).reshape(-1) - np.asarray(mean_r, np.float64).reshape(-1)) / \
        (np.asarray(std_r, np.float64).reshape(-1) + NORM_EPS)
    return x0, t, nr.astype(np.float32).reshape(-1, 1)


def _ln_fwd(a, g, be, f32):
    mean = np.mean(a, axis=1, keepdims=True, dtype=f32)
    var = np.mean(np.square(a - mean), axis=1, keepdims=True, dtype=f32)
    rs = f32(1) / np.sqrt(var + f32(LN_EPS))
    inv = rs * g
    return a * inv + (be - mean * inv), mean, rs


def _ln_bwd(dh, a, mean, rs, g, f32):
    """TF1 layer_norm autodiff (as fit_grads): returns (d a, d gamma, d beta)."""
    xhat = (a - mean) * rs
    gbe = np.sum(dh, axis=0, dtype=f32)
    gg = np.sum(dh * xhat, axis=0, dtype=f32)
    F = f32(a.shape[1])
    inv = rs * g
    dmean = -np.sum(dh * inv, axis=1, keepdims=True, dtype=f32)
    drs = np.sum(dh * (a - mean) * g, axis=1, keepdims=True, dtype=f32)
    dvar = f32(-0.5) * drs * rs * rs * rs
    da = dh * inv + dmean / F + dvar * f32(2.0) * (a - mean) / F
    return da, gg, gbe


def fit_reward_grads(ps: Sequence[np.ndarray], ln: bool, x0: np.ndarray, t: np.ndarray, r: np.ndarray,
                     dtype=np.float32):
    """(loss_dynamic, loss_reward, grads) for one batch; f32 TF op semantics (``dtype`` float64 only for
    the finite-difference check)."""
    f32 = dtype
    W = [ps[2 * i] for i in range(5)]
    b = [ps[2 * i + 1] for i in range(5)]
    G = [ps[10 + 2 * i] for i in range(3)] if ln else None
    BE = [ps[10 + 2 * i + 1] for i in range(3)] if ln else None

    def layer(h, i, j):              # dense i (tanh) [+ LayerNorm j]
        a = np.tanh(h @ W[i] + b[i]).astype(f32)
        if not ln:
            return a, a, None, None
        hh, mean, rs = _ln_fwd(a, G[j], BE[j], f32)
        return a, hh, mean, rs

    a0, h0, m0, r0 = layer(x0, 0, 0)
    ad, hd, md, rd = layer(h0, 1, 1)
    ar, hr, mr, rr = layer(h0, 3, 2)
    pd = hd @ W[2] + b[2]
    pr = hr @ W[4] + b[4]
    dd, dr_ = t - pd, r - pr
    loss_d = f32(np.mean(np.square(dd), dtype=f32))
    loss_r = f32(np.mean(np.square(dr_), dtype=f32))
    dpd = -((f32(2.0) * (f32(1.0) / f32(dd.size))) * dd)
    dpr = -((f32(2.0) * (f32(1.0) / f32(dr_.size))) * dr_)
    g = [None] * 10
    gl = [None] * 6

    def head(hin, a, hh, mean, rs, dp, iw, iwo, j):
        g[2 * iwo] = hh.T @ dp
        g[2 * iwo + 1] = np.sum(dp, axis=0, dtype=f32)
        dh = dp @ W[iwo].T
        if ln:
            da, gl[2 * j], gl[2 * j + 1] = _ln_bwd(dh, a, mean, rs, G[j], f32)
        else:
            da = dh
        dz = (da * (f32(1) - a * a)).astype(f32)
        g[2 * iw] = hin.T @ dz
        g[2 * iw + 1] = np.sum(dz, axis=0, dtype=f32)
        return dz @ W[iw].T

    dh0 = head(h0, ad, hd, md, rd, dpd, 1, 2, 1) + head(h0, ar, hr, mr, rr, dpr, 3, 4, 2)
    if ln:
        da0, gl[0], gl[1] = _ln_bwd(dh0, a0, m0, r0, G[0], f32)
    else:
        da0 = dh0
    dz0 = (da0 * (f32(1) - a0 * a0)).astype(f32)
    g[0] = x0.T @ dz0
    g[1] = np.sum(dz0, axis=0, dtype=f32)
    grads = [x.astype(f32) for x in g] + ([x.astype(f32) for x in gl] if ln else [])
    return loss_d, loss_r, grads


def fit_reward(ps: List[np.ndarray], st: AdamState, ln: bool, normalization, data_states, data_actions,
               data_rewards, data_deltas, batches: Sequence[np.ndarray], lr: float):
    """dynamics.py:195-219 over explicit batch index lists; returns the per-step (model_loss, reward_loss)."""
    out = []
    for idx in batches:
        x0, t, r = fit_reward_batch(normalization, data_states[idx], data_actions[idx], data_rewards[idx],
                                    data_deltas[idx])
        ld, lr_, grads = fit_reward_grads(ps, ln, x0, t, r)
        adam_apply(ps, grads, st, lr)
        out.append((ld, lr_))
    return out
