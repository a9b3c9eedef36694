"""Drop-in controllers with the reference's API (controllers.py:6-88).

``MPCcontroller(env, dyn_model, horizon, cost_fn, num_simulated_paths, gamma)``
and ``get_action(state) -> np.ndarray (A,) float64`` keep the reference's
signatures so ``train_mpc_ppo.py:218-222`` / ``utils.py:202`` run unchanged.
The rollout itself -- state fan-out, H x dynamics MLP, cheetah cost, argmin --
runs in libbcmpc's HIP kernels (``bc_mpc_amd/csrc/rollout.hip``).

Action source (``rng=``):

* ``"numpy"`` (default, parity mode): exactly one
  ``np.random.uniform(low, high, size=[H, K, A])`` draw from the global legacy
  stream per call, as controllers.py:53 does, so a seeded driver
  (train_mpc_ppo.py:499) sees the same RNG side effects and the same actions.
  The returned action is ``action_paths[0, argmin, :].copy()`` of that array
  (controllers.py:84-85), bit-identical to the reference.
* ``"device"`` (perf mode): actions are drawn inside the kernel with
  Philox4x32-10 keyed by (seed, global candidate, step, draw); one 64-bit seed
  per call is taken from ``np.random`` (or from ``seed=`` if given).

Multi-GPU: when torch.distributed is initialised each rank owns a contiguous
slice of the K candidates (``distributed.shard_range``) and the ranks agree on
the argmin through one all-gather of (3 + A) doubles per step.

The siblings run on the same engine:

* ``MPCcontrollerPolicyNet`` (controllers.py:160-239): policy MLP fused into
  the rollout kernel;
* ``MPCcontrollerReward`` (controllers.py:90-158) and
  ``MPCcontrollerPolicyNetReward`` (controllers.py:289-363): the two-head
  ``NNDynamicsRewardModel`` net (dynamics.py:121-238) in the kernel, objective =
  argmax of the (discounted) predicted reward sum;
* ``MCTScontrollerPolicyNetReward`` (controllers.py:365-457): two engine
  launches per step (first-stage actions, then the policy-guided follow-up paths).
"""
from __future__ import annotations

import copy
import math
import os
from typing import Optional

import numpy as np

from . import distributed as _dist
from . import policy as _policy
from . import weights as _weights
from .cost_functions import is_cheetah_cost, trajectory_cost_fn
from .engine import RolloutEngine


class Controller():
    """controllers.py:6-12."""

    def __init__(self):
        pass

    def get_action(self, state):
        pass


class RandomController(Controller):
    """controllers.py:15-24 (uniform env.action_space.sample())."""

    def __init__(self, env):
        self.env = env

    def get_action(self, state):
        return self.env.action_space.sample()


def _stock(fn):
    """Mark a sample_random_actions body that is the reference's np.random.uniform draw verbatim:
    get_action may then make that same draw in the library (same values, same stream advance)."""
    fn._bcmpc_stock_sampler = True
    return fn


def _stock_sampler(obj) -> bool:
    return ("sample_random_actions" not in obj.__dict__
            and getattr(type(obj).sample_random_actions, "_bcmpc_stock_sampler", False))


def _default_device() -> int:
    if "LOCAL_RANK" in os.environ:
        return int(os.environ["LOCAL_RANK"])
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.current_device()
    except Exception:  # pragma: no cover
        pass
    return 0


def _comm_device(ctrl) -> int:
    """The GPU of a controller's engine: the min-loc record goes through it under RCCL."""
    if ctrl._engine is not None:
        return ctrl._engine.device
    return _default_device() if ctrl._device is None else ctrl._device


def _attach_comm(ctrl, eng: RolloutEngine, fused: bool = True) -> RolloutEngine:
    """Under RCCL, give the engine the library's communicator (created once per controller, a
    collective on the first call every rank makes together): its get_action then returns the global
    best itself.  Only when every rank holds candidates (K >= world) and the cost is fused."""
    rank, ws = _dist.world(ctrl._group)
    want = fused and ws > 1 and int(ctrl.num_simulated_paths) >= ws and _dist.use_library_comm(ctrl._group)
    if want and getattr(eng, "comm", None) is None:
        if getattr(ctrl, "_comm", None) is None:
            ctrl._comm = _dist.LibraryComm(eng.device, ctrl._group)
        eng.set_comm(ctrl._comm)
    elif not want and getattr(eng, "comm", None) is not None:
        # (K fell below the world size: a rank may hold no candidates and must join the torch
        #  all-gather, so every rank's engine drops the communicator -- every rank decides alike)
        eng.set_comm(None)
    return eng


def _minloc(ctrl, eng, valid, cost, index, first, A):
    """The ranks' agreement on (cost, index, first action): already made inside the library when the
    engine that ran THIS step (``eng``: None when this rank launched nothing) has a communicator, else
    one torch all-gather of the records."""
    if valid and _dist.world(ctrl._group)[1] == 1:      # one rank: nothing to agree on
        return float(cost), int(index), np.array(first, dtype=np.float64)
    if eng is not None and getattr(eng, "comm", None) is not None:
        return float(cost), int(index), np.asarray(first, dtype=np.float64).copy()
    return _dist.allgather_minloc(valid, cost, index, first, A, ctrl._group, device=_comm_device(ctrl))


class MPCcontroller(Controller):
    """Random-shooting MPC (controllers.py:26-88) on the MI355X rollout engine."""

    def __init__(self,
                 env,
                 dyn_model,
                 horizon=5,
                 cost_fn=None,
                 num_simulated_paths=10,
                 gamma=1.,
                 *,
                 rng: str = "numpy",
                 seed: Optional[int] = None,
                 device: Optional[int] = None,
                 process_group=None):
        self.env = env
        self.dyn_model = dyn_model
        self.horizon = horizon
        self.cost_fn = cost_fn
        self.num_simulated_paths = num_simulated_paths
        self.gamma = gamma                      # stored, unused (as in the reference)
        if rng not in ("numpy", "device"):
            raise ValueError("rng must be 'numpy' or 'device'")
        self.rng = rng
        self._seed_rng = np.random.RandomState(seed) if seed is not None else None
        self._device = device
        self._group = process_group
        self._engine: Optional[RolloutEngine] = None
        self._engine_key = None
        self._fast = None                       # get_action's repeat-call fast path (see there)
        self._traj_buf = None
        # diagnostics of the last call (not part of the reference API)
        self.last_cost = None
        self.last_index = None
        self.last_costs = None
        self.keep_costs = False

    # controllers.py:43-55
    @_stock
    def sample_random_actions(self):
        np_action_paths = np.random.uniform(low=self.env.action_space.low, high=self.env.action_space.high,
                                            size=[self.horizon, self.num_simulated_paths,
                                                  len(self.env.action_space.high)])
        return np_action_paths

    # ------------------------------------------------------------------ engine
    def _dims(self):
        S = int(math.prod(self.env.observation_space.shape))
        A = len(self.env.action_space.high)
        return S, A

    def _engine_for(self, spec, S, A, k_local, fused) -> RolloutEngine:
        dev = _default_device() if self._device is None else self._device
        key = (S, A, spec.hidden, spec.n_layers, spec.activation, spec.layer_norm, int(self.horizon),
               int(k_local), dev, fused)
        if self._engine is None or self._engine_key != key:
            if self._engine is not None:
                self._engine.close()
            self._engine = RolloutEngine(S, A, spec.hidden, spec.n_layers, spec.activation, spec.layer_norm,
                                         int(self.horizon), int(k_local), device=dev,
                                         cost="cheetah" if fused else "none")
            self._engine.set_action_bounds(np.asarray(self.env.action_space.low, dtype=np.float64),
                                           np.asarray(self.env.action_space.high, dtype=np.float64))
            self._engine_key = key
            self._traj_buf = None
        return _attach_comm(self, self._engine, fused)

    def _next_seed(self) -> int:
        src = self._seed_rng if self._seed_rng is not None else np.random
        return int(src.randint(0, 2**62, dtype=np.int64))

    # controllers.py:57-88
    def get_action(self, state):
        fp = getattr(self, "_fast", None)
        if fp is not None:
            # the per-env-step repeat (utils.py:202): same env / model / cost / shape as the last call, the
            # model's weights version and normalisation objects unchanged, one rank -- the checks below
            # were all made by that call, so only the NumPy-stream launch remains
            if (fp[0] == (self.env, self.dyn_model, self.cost_fn, self.horizon, self.num_simulated_paths, self.rng,
                          self.keep_costs) and _weights.same_token(self.dyn_model, fp[1])
                    and "sample_random_actions" not in self.__dict__ and _dist.world(self._group)[1] == 1):
                space = self.env.action_space
                res = fp[2].get_action_numpy_stream(state, space.low, space.high, fp[3])
                if res is not None:
                    self.last_costs = None
                    self.last_cost, self.last_index = res.best_cost, res.best_index
                    return res.first_action
            self._fast = None
        S, A = self._dims()
        K = int(self.num_simulated_paths)
        if self.horizon < 1:
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")   # controllers.py:85 at H=0
        state = np.asarray(state, dtype=np.float64).reshape(-1)
        rank, ws = _dist.world(self._group)
        lo, hi = _dist.shard_range(K, rank, ws)
        spec, norm, version = _weights.extract(self.dyn_model)
        if spec.model != "delta":
            raise TypeError("MPCcontroller needs an NNDynamicsModel: NNDynamicsRewardModel.predict returns "
                            "(next_state, reward) (dynamics.py:238); use MPCcontrollerReward")
        fused = is_cheetah_cost(self.cost_fn, S, A)
        if not fused and self.rng != "numpy":
            raise ValueError("a non-cheetah cost_fn needs rng='numpy' (actions must exist on the host)")

        if K == 0:                                          # (the reference draws before failing)
            if self.rng == "numpy":
                self.sample_random_actions()
            else:
                self._next_seed()
            raise ValueError("attempt to get argmin of an empty sequence")
        # the reference's draw, made by the library straight into pinned memory and uploaded step
        # by step (same values, same stream advance) unless sample_random_actions is overridden
        if self.rng == "numpy" and fused and hi > lo and _stock_sampler(self):
            eng = self._engine_for(spec, S, A, hi - lo, fused)
            eng.set_weights(spec, norm, version)
            res = eng.get_action_numpy_stream(state, self.env.action_space.low, self.env.action_space.high, K, lo,
                                              return_costs=self.keep_costs)
            if res is not None:
                self.last_costs = res.costs
                cost, index, first_g = _minloc(self, eng, True, res.best_cost, res.best_index, res.first_action, A)
                self.last_cost, self.last_index = cost, index
                tok = _weights.weight_token(self.dyn_model)
                if ws == 1 and not self.keep_costs and tok is not None and eng.comm is None:
                    self._fast = ((self.env, self.dyn_model, self.cost_fn, self.horizon, self.num_simulated_paths,
                                   self.rng, self.keep_costs), tok, eng, K)
                return first_g                               # = action_paths[0, index] (controllers.py:84-85)

        action_paths = None
        seed = 0
        if self.rng == "numpy":
            action_paths = self.sample_random_actions()      # every rank draws the full [H, K, A]
        else:
            seed = self._next_seed()

        valid, cost, index, first = False, float("inf"), -1, None
        if hi > lo:
            eng = self._engine_for(spec, S, A, hi - lo, fused)
            eng.set_weights(spec, norm, version)            # no-op unless the version changed
            local = None if action_paths is None else np.ascontiguousarray(action_paths[:, lo:hi, :])
            if fused:
                res = eng.get_action(state, local, seed=seed, cand_offset=lo, return_costs=self.keep_costs)
                valid, cost, index, first = True, res.best_cost, res.best_index, res.first_action
                self.last_costs = res.costs
            else:
                costs = self._trajectory_costs(eng, state, local)
                i = int(np.argmin(costs))
                valid, cost, index, first = True, float(costs[i]), lo + i, local[0, i, :].copy()
                self.last_costs = costs

        cost, index, first_g = _minloc(self, self._engine if valid else None, valid, cost, index, first, A)
        self.last_cost, self.last_index = cost, index
        if action_paths is not None:
            opt_action_path = action_paths[:, index, :]     # controllers.py:84-85
            return opt_action_path[0].copy()
        return first_g

    def _trajectory_costs(self, eng: RolloutEngine, state, local_actions) -> np.ndarray:
        """Non-fused cost_fn: the engine returns states_paths_all (controllers.py:65-74)
        and the caller's cost_fn scores them through trajectory_cost_fn (:80)."""
        import torch
        dev = torch.device("cuda", eng.device)
        H, Kl, A = local_actions.shape
        S = eng.state_dim
        d_state = torch.from_numpy(state).to(dev)
        d_act = torch.from_numpy(local_actions).to(dev)
        d_traj = torch.empty((H + 1, Kl, S), dtype=torch.float64, device=dev)
        stream = torch.cuda.current_stream(dev)
        eng.rollout_async(d_state.data_ptr(), 0, d_act.data_ptr(), 0, 0, None, d_traj.data_ptr(), None,
                          stream.cuda_stream)
        traj = d_traj.cpu().numpy()                       # synchronises the stream
        eng.check_status()
        return np.asarray(trajectory_cost_fn(self.cost_fn, traj[:-1], local_actions, traj[1:]), dtype=np.float64)


class _SeedStream:
    """A controller's per-call Philox seeds: ``RandomState(seed).randint(0, 2**62)``, one per call, drawn 64 at
    a time (legacy randint fills a batch in call order, so the sequence is the one-at-a-time sequence) -- a call
    pays a list pop instead of a ~3-us scalar randint.  ``get_state`` / ``set_state`` carry the unread seeds."""

    def __init__(self, seed):
        self._rs = np.random.RandomState(seed)
        self._buf = []                          # unread seeds, next last

    def next(self) -> int:
        if not self._buf:
            self._buf = self._rs.randint(0, 2**62, size=64, dtype=np.int64).tolist()[::-1]
        return self._buf.pop()

    def unread(self, seed: int) -> None:
        self._buf.append(seed)

    def get_state(self):
        return self._rs.get_state(), tuple(self._buf)

    def set_state(self, state) -> None:
        self._rs.set_state(state[0])
        self._buf = list(state[1])


class MPCcontrollerPolicyNet(Controller):
    """Policy-guided MPC (controllers.py:160-237) on the MI355X rollout engine.

    Each horizon step the policy net's action for every candidate is computed
    inside the rollout kernel (fused 20->h->h->6 tanh MLP, ppo_bc_policy.py:
    54-88), mixed with the exploration draw and fed to the dynamics MLP:

    * ``self_exp=False`` (train_mpc_ppo.py default, FLAGS.SELFEXP):
      ``(1 - explore) * mean + explore * exploration[i]`` (controllers.py:204-208)
      -- deterministic given the global NumPy stream, bit-for-bit parity;
    * ``self_exp=True``: ``mean + exp(logstd) * N(0, 1)`` (DiagGaussianPd.sample).
      TF's random_normal stream cannot be reproduced outside TF; the engine
      draws N(0,1) with Philox (seed from ``seed=`` or a private generator, so
      the global NumPy stream is consumed exactly as the reference does).

    ``sample_random_actions`` is still called once per step in both modes
    (controllers.py:191), preserving the reference's RNG side effect.
    """

    def __init__(self,
                 env,
                 dyn_model,
                 policy_net,
                 explore=1.,
                 self_exp=True,
                 horizon=5,
                 cost_fn=None,
                 num_simulated_paths=10,
                 *,
                 seed: Optional[int] = None,
                 device: Optional[int] = None,
                 process_group=None):
        self.env = env
        self.dyn_model = dyn_model
        self.policy_net = policy_net
        self.horizon = horizon
        self.cost_fn = cost_fn
        self.num_simulated_paths = num_simulated_paths
        self.self_exp = self_exp
        self.explore = explore
        self._seed_rng = _SeedStream(0x5EEDF00D if seed is None else seed)
        self._device = device
        self._group = process_group
        self._engine = None
        self._engine_key = None
        self._fast = None                       # get_action's repeat-call fast path
        self.last_cost = None
        self.last_index = None
        self.last_costs = None
        self.keep_costs = False

    # controllers.py:181-186
    @_stock
    def sample_random_actions(self):
        np_action_paths = np.random.uniform(low=self.env.action_space.low, high=self.env.action_space.high,
                                            size=[self.horizon, self.num_simulated_paths,
                                                  len(self.env.action_space.high)])
        return np_action_paths

    def _engine_for(self, spec, pspec, S, A, k_local) -> RolloutEngine:
        dev = _default_device() if self._device is None else self._device
        mode = "stochastic" if self.self_exp else "explore"
        key = (S, A, spec.model, spec.hidden, spec.n_layers, spec.activation, spec.layer_norm, int(self.horizon),
               int(k_local), dev, pspec.hidden, pspec.n_layers, mode)
        if self._engine is None or self._engine_key != key:
            if self._engine is not None:
                self._engine.close()
            reward = spec.model == "reward"
            self._engine = RolloutEngine(S, A, spec.hidden, spec.n_layers, spec.activation, spec.layer_norm,
                                         int(self.horizon), int(k_local), device=dev,
                                         cost="reward" if reward else "cheetah", model=spec.model,
                                         policy_hidden=pspec.hidden, policy_layers=pspec.n_layers,
                                         policy_mode=mode)
            self._engine.set_action_bounds(np.asarray(self.env.action_space.low, dtype=np.float64),
                                           np.asarray(self.env.action_space.high, dtype=np.float64))
            self._engine_key = key
        return _attach_comm(self, self._engine)

    _MODEL = "delta"     # NNDynamicsModel + cheetah cost, argmin

    def _fast_key(self):
        return (self.env, self.dyn_model, self.policy_net, self.cost_fn, self.horizon, self.num_simulated_paths,
                self.explore, self.self_exp, self.keep_costs)

    # controllers.py:189-237
    def get_action(self, state):
        fp = getattr(self, "_fast", None)
        if fp is not None:
            # the per-env-step repeat (as MPCcontroller.get_action): same env / models / cost / shape /
            # exploration as the last call, the dynamics weights version and normalisation objects and the
            # policy's integer version unchanged, one rank, NumPy's verified legacy stream
            from .engine import _legacy_mt_state
            if (fp[0] == self._fast_key() and _weights.same_token(self.dyn_model, fp[1])
                    and _policy.int_version(self.policy_net) == fp[2] and "sample_random_actions" not in self.__dict__
                    and _dist.world(self._group)[1] == 1 and _legacy_mt_state() is not None):
                space = self.env.action_space
                seed = self._seed_rng.next()
                res = fp[3].get_action_numpy_stream(state, space.low, space.high, fp[4], 0, seed=seed)
                if res is not None:
                    self.last_costs = None
                    self.last_cost, self.last_index = res.best_cost, res.best_index
                    return res.first_action
                self._seed_rng.unread(seed)                      # (nothing drawn: the slow path draws it)
            self._fast = None
        S = int(math.prod(self.env.observation_space.shape))
        A = len(self.env.action_space.high)
        K = int(self.num_simulated_paths)
        if self.horizon < 1:
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")
        reward = self._MODEL == "reward"
        if not reward and not is_cheetah_cost(self.cost_fn, S, A):
            raise ValueError("MPCcontrollerPolicyNet on the engine needs the fused cheetah cost_fn")
        state = np.asarray(state, dtype=np.float64).reshape(-1)
        rank, ws = _dist.world(self._group)
        lo, hi = _dist.shard_range(K, rank, ws)
        spec, norm, version = _weights.extract(self.dyn_model)
        _check_model(spec, self._MODEL, type(self).__name__)
        pspec, pversion = _policy.extract(self.policy_net)
        sign = -1.0 if reward else 1.0                         # argmax(r) == argmin(-r), ties and NaN alike
        if K > 0 and hi > lo and _stock_sampler(self):
            # the exploration draw (controllers.py:191) made by the library into pinned memory,
            # same values and stream advance as sample_random_actions
            eng = self._engine_for(spec, pspec, S, A, hi - lo)
            eng.set_weights(spec, norm, version)
            eng.set_policy(pspec, float(self.explore), pversion)
            seed = self._seed_rng.next()
            res = eng.get_action_numpy_stream(state, self.env.action_space.low, self.env.action_space.high, K,
                                              lo, return_costs=self.keep_costs, seed=seed)
            if res is None:
                self._seed_rng.unread(seed)                  # (nothing drawn: the host path draws the seed)
            if res is not None:
                self.last_costs = res.costs
                cost, index, first_g = _minloc(self, eng, True, sign * res.best_cost, res.best_index,
                                               res.first_action, A)
                self.last_cost, self.last_index = sign * cost, index
                tok, pv = _weights.weight_token(self.dyn_model), _policy.int_version(self.policy_net)
                if ws == 1 and not self.keep_costs and tok is not None and pv is not None and eng.comm is None:
                    self._fast = (self._fast_key(), tok, pv, eng, K)
                return first_g
        exploration = self.sample_random_actions()           # every rank draws the full [H, K, A]
        seed = self._seed_rng.next()
        if K == 0:
            raise ValueError(f"attempt to get {'argmax' if reward else 'argmin'} of an empty sequence")
        valid, cost, index, first = False, float("inf"), -1, None
        if hi > lo:
            eng = self._engine_for(spec, pspec, S, A, hi - lo)
            eng.set_weights(spec, norm, version)
            eng.set_policy(pspec, float(self.explore), pversion)
            local = np.ascontiguousarray(exploration[:, lo:hi, :])
            res = eng.get_action(state, local, seed=seed, cand_offset=lo, return_costs=self.keep_costs)
            valid, cost, index, first = True, res.best_cost, res.best_index, res.first_action
            self.last_costs = res.costs
        cost, index, first_g = _minloc(self, self._engine if valid else None, valid, sign * cost, index, first, A)
        self.last_cost, self.last_index = sign * cost, index
        return first_g                                         # copy of action_paths[0, argmin] (:233-235)

    get_action_mcs = get_action                                # controllers.py:239 (identical body)


def _check_model(spec, want: str, who: str) -> None:
    if spec.model != want:
        need = "NNDynamicsRewardModel (dynamics.py:121)" if want == "reward" else "NNDynamicsModel (dynamics.py:7)"
        raise TypeError(f"{who} needs an {need}; got a {spec.model!r} dynamics net")


class MPCcontrollerReward(Controller):
    """Learned-reward random-shooting MPC (controllers.py:90-158) on the engine.

    ``dyn_model`` is an ``NNDynamicsRewardModel`` (dynamics.py:121-238): the
    kernel runs its two-head net each step and accumulates
    ``sum_h reward_h * gamma**h`` (controllers.py:139,150); the controller
    returns the first action of the ARGMAX path (controllers.py:152-156).

    Action source (``rng=``):

    * ``"env"`` (default, parity mode): ``sample_random_actions`` makes K*H
      ``env.action_space.sample()`` calls and reshapes them to ``[H, K, A]``
      exactly as controllers.py:108-119 (same env-RNG side effect, same dtype --
      a float32 Box gives float32 actions, widened exactly to f64 for the engine);
    * ``"device"`` (perf mode): Philox draws in the kernel, one 64-bit seed per
      call from a private generator (``seed=``), env RNG untouched.
    """

    def __init__(self,
                 env,
                 dyn_model,
                 horizon=5,
                 cost_fn=None,
                 num_simulated_paths=10,
                 gamma=1.,
                 *,
                 rng: str = "env",
                 seed: Optional[int] = None,
                 device: Optional[int] = None,
                 process_group=None):
        self.env = env
        self.dyn_model = dyn_model
        self.horizon = horizon
        self.cost_fn = cost_fn                  # stored, unused (as in the reference)
        self.num_simulated_paths = num_simulated_paths
        self.gamma = gamma
        if rng not in ("env", "device"):
            raise ValueError("rng must be 'env' or 'device'")
        self.rng = rng
        self._seed_rng = np.random.RandomState(0x5EED0BAD if seed is None else seed)
        self._device = device
        self._group = process_group
        self._engine: Optional[RolloutEngine] = None
        self._engine_key = None
        self._gamma_set = None
        self.last_reward = None
        self.last_index = None
        self.last_rewards = None
        self.keep_costs = False

    # controllers.py:108-119
    def sample_random_actions(self):
        actions = []
        for n in range(self.num_simulated_paths):
            for h in range(self.horizon):
                actions.append(self.env.action_space.sample())
        np_action_paths = np.asarray(actions)
        np_action_paths = np.reshape(np_action_paths, [self.horizon, self.num_simulated_paths, -1])
        return np_action_paths

    def _engine_for(self, spec, S, A, k_local) -> RolloutEngine:
        dev = _default_device() if self._device is None else self._device
        key = (S, A, spec.hidden, spec.layer_norm, int(self.horizon), int(k_local), dev)
        if self._engine is None or self._engine_key != key:
            if self._engine is not None:
                self._engine.close()
            self._engine = RolloutEngine(S, A, spec.hidden, 2, "tanh", spec.layer_norm, int(self.horizon),
                                         int(k_local), device=dev, cost="reward", model="reward")
            self._engine.set_action_bounds(np.asarray(self.env.action_space.low, dtype=np.float64),
                                           np.asarray(self.env.action_space.high, dtype=np.float64))
            self._engine_key = key
            self._gamma_set = None
        if self._gamma_set != float(self.gamma):
            self._engine.set_discount(float(self.gamma))
            self._gamma_set = float(self.gamma)
        return _attach_comm(self, self._engine)

    # controllers.py:121-158
    def get_action(self, state):
        S = int(math.prod(self.env.observation_space.shape))
        A = len(self.env.action_space.high)
        K = int(self.num_simulated_paths)
        if self.horizon < 1:
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")
        state = np.asarray(state, dtype=np.float64).reshape(-1)
        rank, ws = _dist.world(self._group)
        lo, hi = _dist.shard_range(K, rank, ws)
        spec, norm, version = _weights.extract(self.dyn_model)
        _check_model(spec, "reward", type(self).__name__)
        action_paths, seed = None, 0
        if self.rng == "env":
            action_paths = self.sample_random_actions()      # every rank draws the full [H, K, A]
        else:
            seed = int(self._seed_rng.randint(0, 2**62, dtype=np.int64))
        if K == 0:
            raise ValueError("attempt to get argmax of an empty sequence")
        valid, neg, index, first = False, float("inf"), -1, None
        if hi > lo:
            eng = self._engine_for(spec, S, A, hi - lo)
            eng.set_weights(spec, norm, version)
            local = None if action_paths is None else np.ascontiguousarray(action_paths[:, lo:hi, :],
                                                                           dtype=np.float64)
            res = eng.get_action(state, local, seed=seed, cand_offset=lo, return_costs=self.keep_costs)
            valid, neg, index, first = True, -res.best_cost, res.best_index, res.first_action
            self.last_rewards = res.costs
        neg, index, first_g = _minloc(self, self._engine if valid else None, valid, neg, index, first, A)
        self.last_reward, self.last_index = -neg, index
        if action_paths is not None:
            return copy.copy(action_paths[:, index, :][0])    # controllers.py:154-156
        return first_g


class MPCcontrollerPolicyNetReward(MPCcontrollerPolicyNet):
    """Policy-guided learned-reward MPC (controllers.py:289-363) on the engine:
    the fused policy of ``MPCcontrollerPolicyNet`` plus the two-head reward net;
    argmax of the UNdiscounted reward sum (``gamma`` is stored but unused,
    controllers.py:345).  The reference's debug print of the reward-vector
    shape (controllers.py:351) is not reproduced."""

    _MODEL = "reward"

    def __init__(self,
                 env,
                 dyn_model,
                 policy_net,
                 explore=1.,
                 self_exp=True,
                 horizon=5,
                 cost_fn=None,
                 num_simulated_paths=10,
                 gamma=1.,
                 *,
                 seed: Optional[int] = None,
                 device: Optional[int] = None,
                 process_group=None):
        super().__init__(env, dyn_model, policy_net, explore=explore, self_exp=self_exp, horizon=horizon,
                         cost_fn=cost_fn, num_simulated_paths=num_simulated_paths, seed=seed, device=device,
                         process_group=process_group)
        self.gamma = gamma

    # controllers.py:310-316
    @_stock
    def sample_random_actions(self):
        np_action_paths = np.random.uniform(low=self.env.action_space.low, high=self.env.action_space.high,
                                            size=[self.horizon, self.num_simulated_paths,
                                                  len(self.env.action_space.high)])
        return np_action_paths


class MCTScontrollerPolicyNetReward(Controller):
    """Two-stage policy-guided search (controllers.py:365-457) on the engine.

    Stage 1 (controllers.py:403-425): ``num_first_stage_actions`` (N) first actions from the root
    state -- the policy's stochastic sample (``self_exp=True``, Philox normals as in
    ``MPCcontrollerPolicyNet``), its mean (``self_exp=False``), or ``env.action_space.sample()``
    (``random_first_stage_action``) -- each scored by one ``predict`` step of the two-head
    ``NNDynamicsRewardModel``: one engine launch of N candidates, horizon 1, returning the first
    actions, the rewards and the next states.  Stage 2 (controllers.py:427-449): every next state
    tiled ``random_path_per_action`` (R) times and rolled ``horizon`` steps with the DETERMINISTIC
    policy (the reference's ``stochastic=False``): one launch of N*R candidates with per-candidate
    initial states and the fused policy at ``explore = 0``, returning the reward sums.  The mean over
    the R paths, the sum with the first reward and the argmax stay NumPy (:442-451).  Returns the
    chosen first action with the reference's shape ``[1, A]`` (float32 for the policy's actions).
    The reference's follow-up paths of one first action are identical (deterministic policy and
    model), so the engine computes N*R equal rows exactly as the reference does.
    """

    def __init__(self,
                 env,
                 dyn_model,
                 policy_net,
                 explore=1.,
                 self_exp=True,
                 horizon=5,
                 cost_fn=None,
                 num_first_stage_actions=10,
                 random_path_per_action=10,
                 random_first_stage_action=False,
                 *,
                 seed: Optional[int] = None,
                 device: Optional[int] = None):
        self.env = env
        self.dyn_model = dyn_model
        self.policy_net = policy_net
        self.horizon = horizon
        self.cost_fn = cost_fn
        self.num_first_stage_actions = num_first_stage_actions
        self.random_path_per_action = random_path_per_action
        self.self_exp = self_exp
        self.explore = explore
        self.random_first_stage_action = random_first_stage_action
        self._seed_rng = np.random.RandomState(0x5EEDC0DE if seed is None else seed)
        self._device = device
        self._engines = {}
        self.last_index = None
        self.last_total_rewards = None
        self.last_first_actions = None
        self.last_seeds = None

    # controllers.py:390-395, verbatim: __init__ never sets num_simulated_paths, so (as in the
    # reference) calling it raises AttributeError; get_action does not use it
    def sample_random_actions(self):
        np_action_paths = np.random.uniform(low=self.env.action_space.low, high=self.env.action_space.high,
                                            size=[self.horizon, self.num_simulated_paths,
                                                  len(self.env.action_space.high)])
        return np_action_paths

    def _engine_for(self, stage, spec, pspec, S, A, K, H, mode, dev) -> RolloutEngine:
        key = (S, A, spec.hidden, spec.layer_norm, pspec.hidden, pspec.n_layers, int(K), int(H), mode, dev)
        eng, old = self._engines.get(stage, (None, None))
        if eng is None or old != key:
            if eng is not None:
                eng.close()
            eng = RolloutEngine(S, A, spec.hidden, 2, "tanh", spec.layer_norm, int(H), int(K), device=dev,
                                cost="reward", model="reward", policy_hidden=pspec.hidden,
                                policy_layers=pspec.n_layers, policy_mode=mode)
            eng.set_action_bounds(np.asarray(self.env.action_space.low, dtype=np.float64),
                                  np.asarray(self.env.action_space.high, dtype=np.float64))
            self._engines[stage] = (eng, key)
        return eng

    # controllers.py:397-457
    def get_action(self, state):
        import torch
        S = int(math.prod(self.env.observation_space.shape))
        A = len(self.env.action_space.high)
        N, R = int(self.num_first_stage_actions), int(self.random_path_per_action)
        state = np.asarray(state, dtype=np.float64).reshape(-1)
        spec, norm, version = _weights.extract(self.dyn_model)
        _check_model(spec, "reward", type(self).__name__)
        pspec, pversion = _policy.extract(self.policy_net)
        dev = _default_device() if self._device is None else self._device
        tdev = torch.device("cuda", dev)
        stream = torch.cuda.current_stream(tdev).cuda_stream
        if N == 0:
            raise ValueError("attempt to get argmax of an empty sequence")
        # ---- first stage (controllers.py:403-418) ----
        action_1s, d_act = None, None
        if self.random_first_stage_action:
            action_1s = [np.expand_dims(self.env.action_space.sample(), axis=0) for _ in range(N)]
            mode, explore = "explore", 1.0                       # (1 - 1) * mean + 1 * U = U exactly
            d_act = torch.from_numpy(np.concatenate(action_1s).astype(np.float64)[None]).to(tdev)
        elif self.self_exp:
            mode, explore = "stochastic", float(self.explore)    # mean + exp(logstd) * N(0, 1)
        else:
            mode, explore = "explore", 0.0                       # the mean
        seed1 = int(self._seed_rng.randint(0, 2**62, dtype=np.int64))
        e1 = self._engine_for("first", spec, pspec, S, A, N, 1, mode, dev)
        e1.set_weights(spec, norm, version)
        e1.set_policy(pspec, explore, pversion)
        d_state = torch.from_numpy(state).to(tdev)
        d_r1 = torch.empty(N, dtype=torch.float64, device=tdev)
        d_traj = torch.empty((2, N, S), dtype=torch.float64, device=tdev)
        e1.rollout_async(d_state.data_ptr(), 0, d_act.data_ptr() if d_act is not None else None, seed1, 0,
                         d_r1.data_ptr(), d_traj.data_ptr(), None, stream)
        reward_1s = d_r1.cpu().numpy()                           # reward_1[0][0] of each predict (:418)
        e1.check_status()
        first = e1.first_actions()
        if action_1s is None:                                    # policy.act's f32 [1, A] rows
            action_1s = [first[i:i + 1].astype(np.float32) for i in range(N)]
        # ---- following stages (controllers.py:421-440): next states tiled R times, action-major ----
        if self.horizon >= 1 and R >= 1:
            seed2 = int(self._seed_rng.randint(0, 2**62, dtype=np.int64))
            e2 = self._engine_for("follow", spec, pspec, S, A, N * R, self.horizon, "explore", dev)
            e2.set_weights(spec, norm, version)
            e2.set_policy(pspec, 0.0, pversion)                  # stochastic=False: the mean
            d_states = torch.repeat_interleave(d_traj[1], R, dim=0).contiguous()
            d_rsum = torch.empty(N * R, dtype=torch.float64, device=tdev)
            e2.rollout_async(d_states.data_ptr(), S, None, seed2, 0, d_rsum.data_ptr(), None, None, stream)
            rewards_all = d_rsum.cpu().numpy().reshape((-1, 1))  # sum over steps of [N*R, 1] (:442-443)
            e2.check_status()
        else:
            seed2 = None
            rewards_all = np.sum(np.asarray([]), axis=0)         # the reference's empty horizon
        rewards_all = rewards_all.reshape((N, -1))              # (:445)
        rewards_all_mean = np.mean(rewards_all, axis=1)
        total_rewards = np.asarray(reward_1s) + rewards_all_mean
        best_action1_idx = int(np.argmax(total_rewards))
        self.last_index, self.last_total_rewards = best_action1_idx, total_rewards
        self.last_first_actions, self.last_seeds = first, (seed1, seed2)
        return action_1s[best_action1_idx]

    def close(self):
        for eng, _ in self._engines.values():
            eng.close()
        self._engines = {}
