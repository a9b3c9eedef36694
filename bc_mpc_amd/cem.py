"""CEM-MPC: the cross-entropy-method outer loop of BASELINE cfg5 on the rollout engine.

The reference has no CEM ("Listed in BASELINE configs, but not
in the reference"), so this controller defines it -- DESIGN.md "CEM" -- with the
reference's constructor and ``get_action(state)`` contract, keyword extras only:

* iteration i samples every candidate's ``[H, A]`` actions as
  ``clip(mu + sigma * z, low, high)`` with z = Irwin-Hall(12) - 6 drawn in the
  rollout kernel (Philox keyed by seed, global candidate, h, j, i);
* the candidates are scored exactly like ``MPCcontroller.get_action`` (fused
  cheetah cost, argmin) or like ``MPCcontrollerReward`` (learned reward, argmax);
* the ``n_elite`` best (NaN last, ties to the lower index) refit mu / sigma to
  their mean / std, smoothed by ``alpha``;
* the answer is the first action of the best candidate of ALL iterations.

Single GPU: one ``bcmpc_cem_get_action`` call (all iterations stream-ordered on
the device, one host sync).  Multi-GPU (torch.distributed, one rank per GPU):
each rank rolls out its contiguous candidate shard; per iteration the ranks
all-gather their local top-E (cost, index) records (E x 16 bytes each), every
rank selects the same global top-E from the gathered records and refits the
same mu / sigma by regenerating the elites' actions from Philox -- no second
collective.  One final all-gather min-loc picks the answer.
"""
from __future__ import annotations

import ctypes
from typing import Optional

import math

import numpy as np

from . import _lib
from . import distributed as _dist
from . import weights as _weights
from .controllers import Controller, _check_model, _default_device
from .cost_functions import is_cheetah_cost
from .engine import RolloutEngine

_ELITE_BYTES = ctypes.sizeof(_lib.Elite)


class CEMcontroller(Controller):
    """Cross-entropy-method MPC on the MI355X engine (BASELINE cfg5 CEM outer loop)."""

    def __init__(self,
                 env,
                 dyn_model,
                 horizon=5,
                 cost_fn=None,
                 num_simulated_paths=10,
                 gamma=1.,
                 *,
                 iterations: int = 4,
                 elite_frac: float = 0.1,
                 n_elite: Optional[int] = None,
                 alpha: float = 0.1,
                 init_std: Optional[float] = None,
                 warm_start: bool = True,
                 seed: Optional[int] = None,
                 device: Optional[int] = None,
                 process_group=None):
        self.env = env
        self.dyn_model = dyn_model
        self.horizon = horizon
        self.cost_fn = cost_fn
        self.num_simulated_paths = num_simulated_paths
        self.gamma = gamma
        if iterations < 1:
            raise ValueError("iterations must be >= 1")
        self.iterations = int(iterations)
        self.elite_frac = float(elite_frac)
        self._n_elite = n_elite
        self.alpha = float(alpha)
        self.init_std = init_std
        self.warm_start = warm_start
        self._seed_rng = np.random.RandomState(0xCE5EED if seed is None else seed)
        self._device = device
        self._group = process_group
        self._engine: Optional[RolloutEngine] = None
        self._engine_key = None
        self._gamma_set = None
        self._mu = None
        self.last_mu = self.last_sigma = None
        self.last_cost = None
        self.last_position = None

    @property
    def n_elite(self) -> int:
        if self._n_elite is not None:
            return int(self._n_elite)
        return max(1, int(round(self.elite_frac * int(self.num_simulated_paths))))

    def reset(self) -> None:
        """Forget the warm-start mean (call at episode boundaries)."""
        self._mu = None

    def _bounds(self):
        return (np.asarray(self.env.action_space.low, dtype=np.float64),
                np.asarray(self.env.action_space.high, dtype=np.float64))

    def initial_distribution(self):
        """mu0: the previous solution shifted by one step (warm start) or the box centre;
        sigma0: init_std, default (high - low) / 4."""
        low, high = self._bounds()
        H = int(self.horizon)
        mid = (low + high) / 2.0
        sd = np.full_like(low, self.init_std) if self.init_std is not None else (high - low) / 4.0
        if self.warm_start and self._mu is not None and self._mu.shape == (H, low.shape[0]):
            mu = np.vstack([self._mu[1:], mid[None]])
        else:
            mu = np.tile(mid, (H, 1))
        return mu, np.tile(sd, (H, 1))

    def _engine_for(self, spec, S, A, k_local) -> RolloutEngine:
        dev = _default_device() if self._device is None else self._device
        key = (S, A, spec.model, spec.hidden, spec.n_layers, spec.activation, spec.layer_norm, int(self.horizon),
               int(k_local), dev)
        if self._engine is None or self._engine_key != key:
            if self._engine is not None:
                self._engine.close()
            reward = spec.model == "reward"
            self._engine = RolloutEngine(S, A, spec.hidden, spec.n_layers, spec.activation, spec.layer_norm,
                                         int(self.horizon), int(k_local), device=dev,
                                         cost="reward" if reward else "cheetah", model=spec.model)
            self._engine.set_action_bounds(*self._bounds())
            self._engine_key = key
            self._gamma_set = None
        if spec.model == "reward" and self._gamma_set != float(self.gamma):
            self._engine.set_discount(float(self.gamma))
            self._gamma_set = float(self.gamma)
        return self._engine

    def get_action(self, state):
        S = int(math.prod(self.env.observation_space.shape))
        A = len(self.env.action_space.high)
        K = int(self.num_simulated_paths)
        if self.horizon < 1:
            raise IndexError("index 0 is out of bounds for axis 0 with size 0")
        if K == 0:
            raise ValueError("attempt to get argmin of an empty sequence")
        state = np.asarray(state, dtype=np.float64).reshape(-1)
        spec, norm, version = _weights.extract(self.dyn_model)
        reward = spec.model == "reward"
        if not reward:
            _check_model(spec, "delta", type(self).__name__)
            if not is_cheetah_cost(self.cost_fn, S, A):
                raise ValueError("CEMcontroller needs the fused cheetah cost_fn or a learned-reward dyn_model")
        mu0, sd0 = self.initial_distribution()
        seed = int(self._seed_rng.randint(0, 2**62, dtype=np.int64))
        rank, ws = _dist.world(self._group)
        lo, hi = _dist.shard_range(K, rank, ws)
        E = min(self.n_elite, K)
        if ws == 1:
            eng = self._engine_for(spec, S, A, K)
            eng.set_weights(spec, norm, version)
            res, mu, sd = eng.cem_get_action(state, mu0, sd0, self.iterations, E, self.alpha, seed)
            cost, pos, first = res.best_cost, res.best_index, res.first_action
        else:
            if K < ws:
                raise ValueError(f"multi-rank CEM needs num_simulated_paths >= world size ({K} < {ws})")
            shard = _EngineShard(self, spec, norm, version, S, A, hi - lo)
            cost, pos, first, mu, sd = cem_multi_rank(shard, state, mu0, sd0, self.iterations, E, self.alpha, seed,
                                                      lo, hi, K, A, reward, self._group)
        self._mu = mu
        self.last_mu, self.last_sigma = mu, sd
        self.last_cost, self.last_position = cost, pos
        return first


class _EngineShard:
    """This rank's engine behind the tensor-level interface cem_multi_rank drives
    (tests substitute a NumPy double with the same methods)."""

    def __init__(self, ctrl: CEMcontroller, spec, norm, version, S, A, k_local):
        import torch
        self.eng = ctrl._engine_for(spec, S, A, k_local)
        self.eng.set_weights(spec, norm, version)
        self.device = torch.device("cuda", self.eng.device)

    def stream(self) -> int:
        import torch
        return torch.cuda.current_stream(self.device).cuda_stream

    def rollout(self, d_state, d_mu, d_sigma, seed, it, lo, k_global, d_costs, d_res, merge):
        self.eng.cem_rollout_async(d_state.data_ptr(), d_mu.data_ptr(), d_sigma.data_ptr(), seed, it, lo, k_global,
                                   d_costs.data_ptr(), d_res.data_ptr(), merge, self.stream())

    def check_status(self):
        self.eng.check_status()

    def select(self, d_pairs, d_costs, m, index_base, n_elite, d_out, d_count):
        self.eng.select_async(d_pairs.data_ptr() if d_pairs is not None else None,
                              d_costs.data_ptr() if d_costs is not None else None, m, index_base, n_elite,
                              d_out.data_ptr(), d_count.data_ptr(), self.stream())

    def refit(self, d_elite, d_count, seed, it, alpha, d_mu, d_sigma):
        self.eng.cem_refit_async(d_elite.data_ptr(), d_count.data_ptr(), seed, it, alpha, d_mu.data_ptr(),
                                 d_sigma.data_ptr(), self.stream())


def cem_multi_rank(shard, state, mu0, sd0, iterations, n_elite, alpha, seed, lo, hi, k_global, A, maximize,
                   group=None):
    """The multi-rank CEM loop (one RCCL all-gather of E (cost, index) records per
    iteration + one final min-loc); every rank owns >= 1 candidate.  Returns
    (objective, position, first_action, mu, sigma), identical on every rank."""
    import torch
    import torch.distributed as dist
    rank, ws = _dist.world(group)
    backend = dist.get_backend(group)
    dev = shard.device
    comm_dev = dev if backend == "nccl" else torch.device("cpu")
    k_local = hi - lo
    f64 = dict(dtype=torch.float64, device=dev)
    d_state = torch.from_numpy(np.ascontiguousarray(state, dtype=np.float64)).to(dev)
    d_mu = torch.from_numpy(np.ascontiguousarray(mu0, dtype=np.float64)).to(dev)
    d_sigma = torch.from_numpy(np.ascontiguousarray(sd0, dtype=np.float64)).to(dev)
    d_costs = torch.empty(max(1, k_local), **f64)
    d_res = torch.zeros(ctypes.sizeof(_lib.Result), dtype=torch.uint8, device=dev)
    nbytes = n_elite * _ELITE_BYTES
    d_local = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_count = torch.zeros(1, dtype=torch.int32, device=dev)
    d_gath = torch.empty(ws * nbytes, dtype=torch.uint8, device=dev)
    d_elite = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    d_gcount = torch.zeros(1, dtype=torch.int32, device=dev)
    for it in range(iterations):
        shard.rollout(d_state, d_mu, d_sigma, seed, it, lo, k_global, d_costs, d_res, it > 0)
        shard.select(None, d_costs, k_local, lo, n_elite, d_local, d_count)
        send = d_local.to(comm_dev)
        recv = torch.empty(ws * nbytes, dtype=torch.uint8, device=comm_dev)
        dist.all_gather_into_tensor(recv, send, group=group)          # ws x E records, rank order
        d_gath.copy_(recv.to(dev))
        shard.select(d_gath, None, ws * n_elite, 0, n_elite, d_elite, d_gcount)
        shard.refit(d_elite, d_gcount, seed, it, alpha, d_mu, d_sigma)
    raw = d_res.cpu().numpy()
    if hasattr(shard, "check_status"):                 # a team-kernel launch that gave up raises here
        shard.check_status()
    best_i = int(raw[:8].view(np.int64)[0])
    best_c = float(raw[8:16].view(np.float64)[0])
    first = raw[16:16 + 8 * A].view(np.float64).copy()
    sign = -1.0 if maximize else 1.0
    cost, pos, first_g = _dist.allgather_minloc(True, sign * best_c, best_i, first, A, group)
    return sign * cost, pos, first_g, d_mu.cpu().numpy(), d_sigma.cpu().numpy()
