"""RolloutEngine: one device's share of MPCcontroller.get_action on libbcmpc.

Thin host wrapper over the C ABI (include/bcmpc.h).  All arithmetic happens in
the HIP kernels; this file only marshals pointers.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib

_ACT = {"tanh": _lib.ACT_TANH, "relu": _lib.ACT_RELU}


@dataclass
class MLPSpec:
    """Dense stack in TF layout: kernels[l] is ``[in, out]`` (tf.layers.dense,
    dynamics.py:67,70), biases[l] ``[out]``; LN params per hidden layer.

    ``model="reward"``: the two-head NNDynamicsRewardModel net (dynamics.py:150-177),
    kernels in TF creation order dense (trunk), dense_1 (delta hidden), dense_2
    (delta out), dense_3 (reward hidden), dense_4 (reward out [h, 1]); LN params
    LayerNorm (trunk), LayerNorm_1 (delta), LayerNorm_2 (reward); tanh."""
    kernels: List[np.ndarray]
    biases: List[np.ndarray]
    activation: str = "tanh"
    ln_gamma: Optional[List[np.ndarray]] = None
    ln_beta: Optional[List[np.ndarray]] = None
    model: str = "delta"

    @property
    def n_layers(self) -> int:
        return 2 if self.model == "reward" else len(self.kernels) - 1

    @property
    def hidden(self) -> int:
        return int(np.shape(self.kernels[0])[1])

    @property
    def layer_norm(self) -> bool:
        return self.ln_gamma is not None


@dataclass
class PolicySpec:
    """MlpPolicy 'pi/pol' stack (ppo_bc_policy.py:66-80): tanh dense layers then
    'final' (no activation), TF layout [in, out]; the obfilter's f32 mean/std
    (RunningMeanStd, ppo_bc_policy.py:57-60) and the DiagGaussian logstd (:79)."""
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
        return int(np.shape(self.kernels[0])[1])


@dataclass
class StepResult:
    best_index: int            # global candidate index (np.argmin semantics)
    best_cost: float
    first_action: np.ndarray   # (A,) f64
    costs: Optional[np.ndarray] = None


def _f32(a) -> np.ndarray:
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(a, dtype=np.float32)


def _f64(a) -> np.ndarray:
    if hasattr(a, "detach"):
        a = a.detach().cpu().numpy()
    return np.ascontiguousarray(a, dtype=np.float64)


def _dp(a: np.ndarray):
    return a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))


# RolloutEngine.get_action's prepared-argument path for the per-step call (BCMPC_PY_FASTPATH=0: build the
# ctypes arguments every call, for A/B runs)
_GA_FAST = os.environ.get("BCMPC_PY_FASTPATH", "1") != "0"


_MT_STATE = [None]          # (bit generator, key pointer, pos pointer) of the verified global MT19937


def _legacy_mt_state():
    """NumPy's global legacy RandomState, when it runs MT19937: its bit generator and pointers to the C
    state behind ``np.random.get_state()`` -- numpy's ``mt19937_state {uint32 key[624]; int pos}`` at
    ``MT19937.ctypes.state_address`` -- which bcmpc_get_action_mt19937 reads and advances in place
    (only on success, as with the tuple path).  The layout is verified once against get_state() per
    generator object; None (the get_state / set_state path) when anything does not match."""
    bg = getattr(getattr(np.random.mtrand, "_rand", None), "_bit_generator", None)
    if type(bg) is not np.random.MT19937:
        return None
    cached = _MT_STATE[0]
    if cached is not None and cached[0] is bg:
        return cached if cached[1] is not None else None
    try:
        addr = bg.ctypes.state_address
        key_p = ctypes.cast(addr, ctypes.POINTER(ctypes.c_uint32))
        pos_p = ctypes.cast(addr + 624 * 4, ctypes.POINTER(ctypes.c_int32))
        with bg.lock:
            st = np.random.get_state()
            ok = (st[0] == "MT19937" and pos_p[0] == int(st[2])
                  and np.array_equal(np.ctypeslib.as_array(key_p, shape=(624,)), np.asarray(st[1], np.uint32)))
    except Exception:
        ok = False
    _MT_STATE[0] = (bg, key_p, pos_p) if ok else (bg, None, None)
    return _MT_STATE[0] if ok else None


class RolloutEngine:
    """Owns one bcmpc_engine (one device, one candidate shard of size K)."""

    def __init__(self, state_dim: int, action_dim: int, hidden: int, n_layers: int,
                 activation: str, layer_norm: bool, horizon: int, num_paths: int,
                 device: int = 0, cost: str = "cheetah", kernel: Optional[str] = None,
                 policy_hidden: int = 0, policy_layers: int = 0, policy_mode: str = "explore",
                 model: str = "delta", precision: Optional[str] = None):
        """``precision``: "fp32" (v_mfma_f32_16x16x4_f32), "split" (f32-accurate hi/lo f16
        operands on v_mfma_f32_16x16x32_f16, rollout_x3.hip; relu / LayerNorm only for the plain delta net
        with hidden <= 512; a fused policy needs a tanh net of hidden 449..1024, 449..512 with the reward
        net), "f16" (one f16 MFMA pass on the split slab kernels: BASELINE cfg3's "bf16 MFMA GEMM + fp32
        cost accumulate", the tanh delta net only; NOT the fp32 tolerance) or "auto" (split
        where it applies, else fp32).
        Default: "split" for the split* kernels, else $BCMPC_PRECISION or "auto"."""
        self._lib = _lib.load()
        if activation not in _ACT:
            raise ValueError(f"unsupported activation {activation!r} (tanh | relu)")
        cfg = _lib.Config()
        cfg.state_dim, cfg.action_dim, cfg.hidden, cfg.n_layers = state_dim, action_dim, hidden, n_layers
        cfg.activation = _ACT[activation]
        cfg.layer_norm = int(bool(layer_norm))
        cfg.horizon = int(horizon)
        costs = {"cheetah": _lib.COST_CHEETAH, "none": _lib.COST_NONE, "reward": _lib.COST_REWARD}
        models = {"delta": _lib.MODEL_DELTA, "reward": _lib.MODEL_REWARD}
        if cost not in costs or model not in models:
            raise ValueError(f"cost must be one of {sorted(costs)}, model one of {sorted(models)}")
        cfg.cost, cfg.model = costs[cost], models[model]
        cfg.num_paths = int(num_paths)
        cfg.device = int(device)
        kernel = kernel or os.environ.get("BCMPC_KERNEL", "auto")
        if kernel not in _lib.KERNELS:
            raise ValueError(f"unknown kernel {kernel!r}; one of {sorted(_lib.KERNELS)}")
        cfg.kernel = _lib.KERNELS[kernel]
        if precision is None:
            precision = "split" if kernel.startswith("split") or kernel == "team" else os.environ.get("BCMPC_PRECISION", "auto")
        if precision == "auto":
            # a fused policy runs in the split kernel's 8-wave groups (dynamics hidden 449..1024;
            # the reward net: hidden <= 512)
            top = 512 if model == "reward" else 1024
            plain = activation == "tanh" and not layer_norm
            split_ok = ((plain or (model == "delta" and not policy_hidden and hidden <= 512))
                        and (model == "delta" or state_dim >= 16)
                        and (not policy_hidden or 448 < hidden <= top)
                        and kernel in ("auto", "split1", "split2", "split4", "team"))
            # the small-K team kernel also takes relu / LayerNorm dynamics under a fused policy (hidden
            # <= 256: train_mpc_ppo.py's 2x256 relu + LN net) and the LayerNorm reward net (the run.sh
            # recipe) when its grid is resident: tried in split, fp32 when bcmpc_create refuses
            team_try = (not split_ok and kernel == "auto" and n_layers == 2 and state_dim >= 16
                        and bool(policy_hidden or model == "reward"))
            precision = "split" if split_ok or team_try else "fp32"
        else:
            team_try = False
        if precision not in _lib.PRECISIONS:
            raise ValueError(f"unknown precision {precision!r}; one of {sorted(_lib.PRECISIONS)}")
        cfg.precision = _lib.PRECISIONS[precision]
        self.precision = precision
        if policy_mode not in _lib.POLICY_MODES:
            raise ValueError(f"unknown policy_mode {policy_mode!r}")
        cfg.policy_hidden, cfg.policy_layers = int(policy_hidden), int(policy_layers)
        cfg.policy_mode = _lib.POLICY_MODES[policy_mode]
        h = ctypes.c_void_p()
        rc = self._lib.bcmpc_create(ctypes.byref(cfg), ctypes.byref(h))
        if rc == _lib.ERR_UNSUPPORTED and team_try:
            precision = "fp32"
            cfg.precision = _lib.PRECISIONS[precision]
            self.precision = precision
            rc = self._lib.bcmpc_create(ctypes.byref(cfg), ctypes.byref(h))
        _lib.check(rc)
        self._h = h
        self.state_dim, self.action_dim = state_dim, action_dim
        self.hidden, self.n_layers, self.activation = hidden, n_layers, activation
        self.layer_norm, self.horizon, self.num_paths = bool(layer_norm), horizon, num_paths
        self.device, self.cost, self.model = device, cost, model
        self.policy_hidden, self.policy_layers, self.policy_mode = policy_hidden, policy_layers, policy_mode
        self._keep = []
        self._wver = None
        self._pol = None
        self.comm = None
        self._mt_fast = None        # get_action_numpy_stream's prepared ctypes arguments
        self._ga_fast = None        # get_action's (device actions, no cost vector) prepared ctypes arguments

    # ------------------------------------------------------------------ weights
    def set_weights(self, spec: MLPSpec, normalization: Sequence, version: int) -> None:
        """Re-sync hook; idempotent on ``version``."""
        if spec.model != self.model or spec.n_layers != self.n_layers or spec.hidden != self.hidden:
            raise ValueError("weight shapes do not match the engine configuration")
        if version == self._wver:       # bcmpc_set_weights returns at once on a known version: skip the marshalling
            return
        ks = [_f32(k) for k in spec.kernels]
        bs = [_f32(b) for b in spec.biases]
        S, A, h = self.state_dim, self.action_dim, self.hidden
        if self.model == "reward":
            exp = [(S + A, h), (h, h), (h, S), (h, h), (h, 1)]
        else:
            exp = [(S + A, h)] + [(h, h)] * (self.n_layers - 1) + [(h, S)]
        if len(ks) != len(exp) or len(bs) != len(exp):
            raise ValueError(f"expected {len(exp)} dense layers, got {len(ks)} kernels / {len(bs)} biases")
        for k, b, e in zip(ks, bs, exp):
            if k.shape != e or b.shape != (e[1],):
                raise ValueError(f"kernel {k.shape}/bias {b.shape} != expected {e}")
        FP = ctypes.POINTER(ctypes.c_float)
        karr = (FP * len(ks))(*[k.ctypes.data_as(FP) for k in ks])
        barr = (FP * len(bs))(*[b.ctypes.data_as(FP) for b in bs])
        w = _lib.Weights()
        w.kernels, w.biases = karr, barr
        keep = [ks, bs, karr, barr]
        if self.layer_norm:
            if not spec.layer_norm:
                raise ValueError("engine built with layer_norm but weights have no LN params")
            gs = [_f32(g) for g in spec.ln_gamma]
            bts = [_f32(b) for b in spec.ln_beta]
            n_ln = 3 if self.model == "reward" else self.n_layers
            if len(gs) != n_ln or len(bts) != n_ln or any(x.shape != (h,) for x in gs + bts):
                raise ValueError(f"expected {n_ln} LayerNorm gamma/beta pairs of shape ({h},)")
            garr = (FP * len(gs))(*[g.ctypes.data_as(FP) for g in gs])
            btarr = (FP * len(bts))(*[b.ctypes.data_as(FP) for b in bts])
            w.ln_gamma, w.ln_beta = garr, btarr
            keep += [gs, bts, garr, btarr]
        (mean_obs, std_obs, mean_action, std_action, *_rest) = normalization
        mean_deltas, std_deltas = normalization[8], normalization[9]
        stats = [_f64(x) for x in (mean_obs, std_obs, mean_action, std_action, mean_deltas, std_deltas)]
        for x, n in zip(stats, (S, S, A, A, S, S)):
            if x.shape != (n,):
                raise ValueError(f"normalization vector of shape {x.shape}, expected ({n},)")
        (w.mean_obs, w.std_obs, w.mean_action, w.std_action, w.mean_deltas, w.std_deltas) = [_dp(x) for x in stats]
        keep.append(stats)
        if self.model == "reward":      # dynamics.py:236 (mean_reward / std_reward: one value each)
            rstats = [_f64(normalization[4]).reshape(-1), _f64(normalization[5]).reshape(-1)]
            if any(x.shape != (1,) for x in rstats):
                raise ValueError("mean_reward / std_reward must hold exactly one value")
            w.mean_reward, w.std_reward = _dp(rstats[0]), _dp(rstats[1])
            keep.append(rstats)
        _lib.check(self._lib.bcmpc_set_weights(self._h, ctypes.byref(w), ctypes.c_uint64(version)))
        self._wver = version

    def set_policy(self, spec: PolicySpec, explore: float, version: int) -> None:
        """Policy weights of MPCcontrollerPolicyNet (controllers.py:160-178)."""
        if spec.n_layers != self.policy_layers or spec.hidden != self.policy_hidden:
            raise ValueError("policy shapes do not match the engine configuration")
        if self._pol is not None and version == self._pol[0]:   # known version: only ``explore`` can change
            self._pol[1].explore = float(explore)
            _lib.check(self._lib.bcmpc_set_policy(self._h, ctypes.byref(self._pol[1]), ctypes.c_uint64(version)))
            return
        S, A, ph = self.state_dim, self.action_dim, self.policy_hidden
        ks = [_f32(k) for k in spec.kernels]
        bs = [_f32(b) for b in spec.biases]
        exp = [(S, ph)] + [(ph, ph)] * (self.policy_layers - 1) + [(ph, A)]
        for k, b, e in zip(ks, bs, exp):
            if k.shape != e or b.shape != (e[1],):
                raise ValueError(f"policy kernel {k.shape}/bias {b.shape} != expected {e}")
        vecs = [_f32(spec.ob_mean).reshape(-1), _f32(spec.ob_std).reshape(-1), _f32(spec.logstd).reshape(-1)]
        if vecs[0].shape != (S,) or vecs[1].shape != (S,) or vecs[2].shape != (A,):
            raise ValueError("policy ob_mean/ob_std must be (S,), logstd (A,)")
        FP = ctypes.POINTER(ctypes.c_float)
        karr = (FP * len(ks))(*[k.ctypes.data_as(FP) for k in ks])
        barr = (FP * len(bs))(*[b.ctypes.data_as(FP) for b in bs])
        p = _lib.Policy(karr, barr, vecs[0].ctypes.data_as(FP), vecs[1].ctypes.data_as(FP),
                        vecs[2].ctypes.data_as(FP), float(explore))
        _lib.check(self._lib.bcmpc_set_policy(self._h, ctypes.byref(p), ctypes.c_uint64(version)))
        self._pol = (version, p, ks, bs, vecs, karr, barr)     # the struct's pointers stay valid while held here

    def first_actions(self) -> np.ndarray:
        """Step-0 actions of every candidate of the last rollout (policy engines), [K, A] f64."""
        out = np.empty((self.num_paths, self.action_dim), dtype=np.float64)
        _lib.check(self._lib.bcmpc_first_actions(self._h, _dp(out)))
        return out

    def set_discount(self, gamma: float) -> None:
        """MPCcontrollerReward.gamma (controllers.py:139): step h's reward is scaled by gamma**h."""
        _lib.check(self._lib.bcmpc_set_discount(self._h, ctypes.c_double(float(gamma))))

    @property
    def weights_version(self) -> int:
        return int(self._lib.bcmpc_weights_version(self._h))

    def predraw_stats(self) -> dict:
        """The NumPy-stream draw's counters (bcmpc_predraw_stats): the small draws' host pre-draw (hits incl.
        late, late, misses) and the large draws' speculative device draw (spec_hits, spec_misses)."""
        out = (ctypes.c_uint64 * 5)()
        _lib.check(self._lib.bcmpc_predraw_stats(self._h, out))
        return {"hits": int(out[0]), "late": int(out[1]), "misses": int(out[2]), "spec_hits": int(out[3]),
                "spec_misses": int(out[4])}

    def set_action_bounds(self, low, high) -> None:
        lo, hi = _f64(low), _f64(high)
        _lib.check(self._lib.bcmpc_set_action_bounds(self._h, _dp(lo), _dp(hi)))

    # ------------------------------------------------------------------ rollout
    def get_action(self, state, actions: Optional[np.ndarray] = None, seed: int = 0,
                   cand_offset: int = 0, return_costs: bool = False) -> StepResult:
        """Synchronous host-memory control step (bcmpc_get_action)."""
        if actions is None and not return_costs and _GA_FAST:
            # the per-step call with in-kernel actions: ctypes arguments built once per shard offset and
            # reused (state copied into an engine-owned buffer, the first action out of a NumPy view on the
            # result record) -- as get_action_numpy_stream's fast path, several us of Python less per call
            fa = self._ga_fast
            if fa is None or fa[0] != cand_offset:
                sbuf = np.zeros(self.state_dim, dtype=np.float64)
                res = _lib.Result()
                first = np.ctypeslib.as_array(res.first_action)[: self.action_dim]
                cseed = ctypes.c_uint64(0)
                args = (self._h, _dp(sbuf), None, cseed, ctypes.c_int64(cand_offset), ctypes.byref(res), None)
                fa = self._ga_fast = (cand_offset, sbuf, res, first, args, cseed)
            _, sbuf, res, first, args, cseed = fa
            s = state if type(state) is np.ndarray else _f64(state)
            if s.size != self.state_dim:
                raise ValueError(f"state has {s.size} dims, expected {self.state_dim}")
            np.copyto(sbuf, s.reshape(-1), casting="unsafe")
            cseed.value = seed & (2**64 - 1)
            rc = self._lib.bcmpc_get_action(*args)
            if rc:
                _lib.check(rc)
            return StepResult(res.best_index, res.best_cost, first.copy(), None)
        st = _f64(state).reshape(-1)
        if st.shape[0] != self.state_dim:
            raise ValueError(f"state has {st.shape[0]} dims, expected {self.state_dim}")
        act_p = None
        if actions is not None:
            actions = _f64(actions)
            if actions.shape != (self.horizon, self.num_paths, self.action_dim):
                raise ValueError(f"actions shape {actions.shape} != (H, K, A) = "
                                 f"{(self.horizon, self.num_paths, self.action_dim)}")
            act_p = _dp(actions)
        res = _lib.Result()
        costs = np.empty(self.num_paths, dtype=np.float64) if return_costs else None
        _lib.check(self._lib.bcmpc_get_action(
            self._h, _dp(st), act_p, ctypes.c_uint64(seed & (2**64 - 1)), ctypes.c_int64(cand_offset),
            ctypes.byref(res), _dp(costs) if costs is not None else None))
        return StepResult(int(res.best_index), float(res.best_cost),
                          np.array(res.first_action[: self.action_dim], dtype=np.float64), costs)

    def _numpy_bounds(self, low, high):
        """Per-action f64 bounds with a finite range (np.random.uniform would not raise), else None
        (checked once per bounds content: every env step passes the same action_space arrays)."""
        key = None
        if isinstance(low, np.ndarray) and isinstance(high, np.ndarray):
            key = (low.dtype.str, low.tobytes(), high.dtype.str, high.tobytes())
            hit = getattr(self, "_bounds_cache", None)
            if hit is not None and hit[0] == key:
                return hit[1]
        lo = np.asarray(low, dtype=np.float64)
        hi = np.asarray(high, dtype=np.float64)
        if lo.shape != (self.action_dim,) or hi.shape != (self.action_dim,) or not np.all(np.isfinite(hi - lo)):
            return None
        out = (np.ascontiguousarray(lo), np.ascontiguousarray(hi))
        if key is not None:
            self._bounds_cache = (key, out)
        return out

    def numpy_stream_available(self, low, high) -> bool:
        """The global generator is NumPy's legacy MT19937 and the bounds are per-action vectors
        with a finite range (np.random.uniform would not raise)."""
        st = np.random.get_state()
        lo = np.asarray(low, dtype=np.float64)
        hi = np.asarray(high, dtype=np.float64)
        return (isinstance(st, tuple) and st[0] == "MT19937" and lo.shape == (self.action_dim,)
                and hi.shape == (self.action_dim,) and bool(np.all(np.isfinite(hi - lo))))

    def get_action_numpy_stream(self, state, low, high, k_global: int, cand_offset: int = 0,
                                return_costs: bool = False, seed: int = 0) -> Optional[StepResult]:
        """get_action on the actions ``np.random.uniform(low, high, [H, k_global, A])`` would
        return from the global legacy stream (controllers.py:53), drawn by the library's MT19937
        restatement from ``np.random.get_state()`` on the GPU (default) or on the host
        (BCMPC_MT_PATH=host) by bcmpc_get_action_mt19937; the global stream is then advanced
        exactly as that one NumPy call advances it -- only when the call succeeds (a failing call
        raises and leaves the stream untouched).  Returns None (nothing drawn) when the global
        generator is not the legacy MT19937 or the bounds are not per-action vectors."""
        mt = _legacy_mt_state()
        if mt is not None:
            # NumPy's own MT19937 state struct, read and advanced in place by the library (under the
            # generator's lock): no get_state / set_state tuple round trips (~30 us each)
            bounds = self._numpy_bounds(low, high)
            if bounds is None:
                return None
            bg, key_p, pos_p = mt
            if return_costs:
                s = _f64(state).reshape(-1)
                if s.shape[0] != self.state_dim:
                    raise ValueError(f"state has {s.shape[0]} dims, expected {self.state_dim}")
                res = _lib.Result()
                costs = np.empty(self.num_paths, dtype=np.float64)
                with bg.lock:
                    _lib.check(self._lib.bcmpc_get_action_mt19937(
                        self._h, _dp(s), key_p, pos_p, _dp(bounds[0]), _dp(bounds[1]), ctypes.c_int64(k_global),
                        ctypes.c_int64(cand_offset), ctypes.c_uint64(seed & (2**64 - 1)), ctypes.byref(res),
                        _dp(costs)))
                return StepResult(int(res.best_index), float(res.best_cost),
                                  np.array(res.first_action[: self.action_dim], dtype=np.float64), costs)
            # the per-env-step call (no cost vector): ctypes arguments built once per (generator, bounds,
            # shard, seed) and reused -- the state goes into an engine-owned buffer, the first action is
            # copied out of a NumPy view on the result record (~6 us of Python per call less)
            key = (k_global, cand_offset)
            fa = self._mt_fast
            if fa is None or fa[0] != key or fa[5] is not bg or fa[6] is not bounds:
                sbuf = np.zeros(self.state_dim, dtype=np.float64)
                res = _lib.Result()
                first = np.ctypeslib.as_array(res.first_action)[: self.action_dim]
                cseed = ctypes.c_uint64(0)
                args = (self._h, _dp(sbuf), key_p, pos_p, _dp(bounds[0]), _dp(bounds[1]), ctypes.c_int64(k_global),
                        ctypes.c_int64(cand_offset), cseed, ctypes.byref(res), None)
                fa = self._mt_fast = (key, sbuf, res, first, args, bg, bounds, cseed)
            _, sbuf, res, first, args = fa[:5]
            fa[7].value = seed & (2**64 - 1)           # (the policy controllers' per-call Philox seed)
            s = state if type(state) is np.ndarray else _f64(state)
            if s.size != self.state_dim:
                raise ValueError(f"state has {s.size} dims, expected {self.state_dim}")
            np.copyto(sbuf, s.reshape(-1), casting="unsafe")
            with bg.lock:
                rc = self._lib.bcmpc_get_action_mt19937(*args)
            if rc:
                _lib.check(rc)
            return StepResult(res.best_index, res.best_cost, first.copy(), None)
        if not self.numpy_stream_available(low, high):
            return None
        st = np.random.get_state()
        lo = np.asarray(low, dtype=np.float64)
        hi = np.asarray(high, dtype=np.float64)
        s = _f64(state).reshape(-1)
        if s.shape[0] != self.state_dim:
            raise ValueError(f"state has {s.shape[0]} dims, expected {self.state_dim}")
        key = np.array(st[1], dtype=np.uint32)
        pos = ctypes.c_int32(int(st[2]))
        res = _lib.Result()
        costs = np.empty(self.num_paths, dtype=np.float64) if return_costs else None
        _lib.check(self._lib.bcmpc_get_action_mt19937(
            self._h, _dp(s), key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos), _dp(lo),
            _dp(hi), ctypes.c_int64(k_global), ctypes.c_int64(cand_offset), ctypes.c_uint64(seed & (2**64 - 1)),
            ctypes.byref(res),
            _dp(costs) if costs is not None else None))
        np.random.set_state((st[0], key, pos.value, st[3], st[4]))
        return StepResult(int(res.best_index), float(res.best_cost),
                          np.array(res.first_action[: self.action_dim], dtype=np.float64), costs)

    def numpy_stream_draw(self, low, high, k_global: int, cand_offset: int = 0) -> np.ndarray:
        """This engine's shard ``[:, cand_offset:cand_offset + K]`` of the array
        ``np.random.uniform(low, high, [H, k_global, A])`` would return from the global legacy stream,
        drawn on the GPU (bcmpc_mt19937_uniform_device); the global stream is advanced exactly as that
        one NumPy call advances it."""
        st = np.random.get_state()
        if not (isinstance(st, tuple) and st[0] == "MT19937"):
            raise ValueError("the global generator is not NumPy's legacy MT19937")
        lo, hi = _f64(low).reshape(-1), _f64(high).reshape(-1)
        if lo.shape != (self.action_dim,) or hi.shape != (self.action_dim,):
            raise ValueError("low / high must be per-action vectors")
        key = np.array(st[1], dtype=np.uint32)
        pos = ctypes.c_int32(int(st[2]))
        out = np.empty((self.horizon, self.num_paths, self.action_dim), dtype=np.float64)
        _lib.check(self._lib.bcmpc_mt19937_uniform_device(
            self._h, key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos), _dp(lo), _dp(hi),
            ctypes.c_int64(k_global), ctypes.c_int64(cand_offset), _dp(out)))
        np.random.set_state((st[0], key, pos.value, st[3], st[4]))
        return out

    def rollout_async(self, d_state: int, state_stride: int, d_actions: Optional[int], seed: int,
                      cand_offset: int, d_costs: Optional[int], d_traj: Optional[int],
                      d_result: Optional[int], stream: Optional[int] = None) -> None:
        """Device-pointer form (bcmpc_rollout_async); no host synchronisation.

        ``stream`` is a raw hipStream_t (e.g. ``torch.cuda.current_stream().cuda_stream``;
        0 is the null stream); ``None`` means the engine's own stream."""
        if stream is None:
            stream = self.stream
        _lib.check(self._lib.bcmpc_rollout_async(
            self._h, ctypes.c_void_p(d_state), ctypes.c_int64(state_stride),
            ctypes.c_void_p(d_actions) if d_actions else None, ctypes.c_uint64(seed & (2**64 - 1)),
            ctypes.c_int64(cand_offset), ctypes.c_void_p(d_costs) if d_costs else None,
            ctypes.c_void_p(d_traj) if d_traj else None, ctypes.c_void_p(d_result) if d_result else None,
            ctypes.c_void_p(stream)))

    def rollout_policy_async(self, d_state: int, d_actions: Optional[int], seed: int, cand_offset: int,
                             d_costs: Optional[int], d_traj: Optional[int], d_actions_out: int,
                             d_result: Optional[int], stream: Optional[int] = None) -> None:
        """Policy engines: rollout_async plus every step's rolled-out actions ``d_actions_out``
        ``[H, K, A]`` f64 (the reference's action_paths, controllers.py:208-213)."""
        stream = self.stream if stream is None else stream
        vp = lambda x: ctypes.c_void_p(x) if x else None   # noqa: E731
        _lib.check(self._lib.bcmpc_rollout_policy_async(
            self._h, ctypes.c_void_p(d_state), vp(d_actions), ctypes.c_uint64(seed & (2**64 - 1)),
            ctypes.c_int64(cand_offset), vp(d_costs), vp(d_traj), ctypes.c_void_p(d_actions_out), vp(d_result),
            ctypes.c_void_p(stream)))

    # ------------------------------------------------------------------ CEM
    def cem_get_action(self, state, mu, sigma, iterations: int, n_elite: int, alpha: float,
                       seed: int) -> Tuple[StepResult, np.ndarray, np.ndarray]:
        """All CEM iterations on this device (bcmpc_cem_get_action).  ``mu``/``sigma`` are
        ``[H, A]``; returns (result with best_index = iteration*K + candidate, mu', sigma')."""
        st = _f64(state).reshape(-1)
        if st.shape[0] != self.state_dim:
            raise ValueError(f"state has {st.shape[0]} dims, expected {self.state_dim}")
        shape = (self.horizon, self.action_dim)
        m = np.array(mu, dtype=np.float64, copy=True).reshape(shape)
        s = np.array(sigma, dtype=np.float64, copy=True).reshape(shape)
        p = _lib.Cem(int(iterations), int(n_elite), float(alpha), 0)
        res = _lib.Result()
        _lib.check(self._lib.bcmpc_cem_get_action(self._h, _dp(st), ctypes.byref(p),
                                                  ctypes.c_uint64(seed & (2**64 - 1)), _dp(m), _dp(s),
                                                  ctypes.byref(res)))
        return (StepResult(int(res.best_index), float(res.best_cost),
                           np.array(res.first_action[: self.action_dim], dtype=np.float64)), m, s)

    def cem_rollout_async(self, d_state: int, d_mu: int, d_sigma: int, seed: int, iteration: int,
                          cand_offset: int, k_global: int, d_costs: int, d_result: Optional[int], merge: bool,
                          stream: Optional[int] = None) -> None:
        stream = self.stream if stream is None else stream
        _lib.check(self._lib.bcmpc_cem_rollout_async(
            self._h, ctypes.c_void_p(d_state), ctypes.c_void_p(d_mu), ctypes.c_void_p(d_sigma),
            ctypes.c_uint64(seed & (2**64 - 1)), int(iteration), int(cand_offset), int(k_global),
            ctypes.c_void_p(d_costs), ctypes.c_void_p(d_result) if d_result else None, int(bool(merge)),
            ctypes.c_void_p(stream)))

    def select_async(self, d_pairs: Optional[int], d_costs: Optional[int], m: int, index_base: int, n_elite: int,
                     d_out: int, d_count: int, stream: Optional[int] = None) -> None:
        stream = self.stream if stream is None else stream
        _lib.check(self._lib.bcmpc_select_async(
            self._h, ctypes.c_void_p(d_pairs) if d_pairs else None, ctypes.c_void_p(d_costs) if d_costs else None,
            int(m), int(index_base), int(n_elite), ctypes.c_void_p(d_out), ctypes.c_void_p(d_count),
            ctypes.c_void_p(stream)))

    def cem_refit_async(self, d_elite: int, d_count: int, seed: int, iteration: int, alpha: float, d_mu: int,
                        d_sigma: int, stream: Optional[int] = None) -> None:
        stream = self.stream if stream is None else stream
        _lib.check(self._lib.bcmpc_cem_refit_async(
            self._h, ctypes.c_void_p(d_elite), ctypes.c_void_p(d_count), ctypes.c_uint64(seed & (2**64 - 1)),
            int(iteration), float(alpha), ctypes.c_void_p(d_mu), ctypes.c_void_p(d_sigma), ctypes.c_void_p(stream)))

    def set_comm(self, comm) -> None:
        """Attach a ``distributed.LibraryComm`` (None detaches): every get_action of this engine then
        exchanges the ranks' result records over RCCL inside the library and returns the GLOBAL best
        (bcmpc_engine_set_comm)."""
        _lib.check(self._lib.bcmpc_engine_set_comm(self._h, comm.handle if comm is not None else None))
        self.comm = comm

    @property
    def stream(self) -> int:
        return int(self._lib.bcmpc_stream(self._h) or 0)

    def check_status(self) -> None:
        """After the stream of a stream-ordered launch (rollout_async, rollout_policy_async,
        cem_rollout_async) has completed: raise BcmpcError when a team-kernel launch of this engine
        gave up because its workgroups could not all be resident (its outputs are not valid);
        bcmpc_engine_status.  Synchronous calls rerun on a fallback engine instead."""
        _lib.check(self._lib.bcmpc_engine_status(self._h))

    @property
    def team_reruns(self) -> int:
        """Synchronous calls of this engine rerun on its fallback engine (bcmpc_engine_team_reruns)."""
        n = ctypes.c_uint64()
        _lib.check(self._lib.bcmpc_engine_team_reruns(self._h, ctypes.byref(n)))
        return int(n.value)

    def set_timing(self, on: bool = True) -> None:
        """Bracket this engine's launches with HIP events (off by default: ~6 us per synchronous
        get_action at small K) so that last_kernel_ms() can read them (bcmpc_engine_set_timing)."""
        _lib.check(self._lib.bcmpc_engine_set_timing(self._h, 1 if on else 0))

    def last_kernel_ms(self) -> Tuple[float, float]:
        r, m = ctypes.c_float(), ctypes.c_float()
        _lib.check(self._lib.bcmpc_last_kernel_ms(self._h, ctypes.byref(r), ctypes.byref(m)))
        return float(r.value), float(m.value)

    def info(self) -> dict:
        hp, wb, wpb, kn = ctypes.c_int32(), ctypes.c_int64(), ctypes.c_int32(), ctypes.c_int32()
        _lib.check(self._lib.bcmpc_engine_info(self._h, ctypes.byref(hp), ctypes.byref(wb), ctypes.byref(wpb),
                                               ctypes.byref(kn)))
        names = {v: k for k, v in _lib.KERNELS.items()}
        buf = ctypes.create_string_buffer(160)
        _lib.check(self._lib.bcmpc_engine_layout(self._h, buf, len(buf)))
        return dict(hidden_padded=hp.value, packed_weight_bytes=wb.value, waves_per_block=wpb.value,
                    kernel=names.get(kn.value, str(kn.value)), layout=buf.value.decode())

    def close(self) -> None:
        # (the prepared ctypes arguments of the fast paths hold the handle: dropped with it, so a call after
        #  close() passes NULL and gets the library's clean error instead of a freed engine)
        self._ga_fast = None
        self._mt_fast = None
        if getattr(self, "_h", None):
            self.comm = None
            self._lib.bcmpc_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass
