"""GPU NNDynamicsModel.fit (dynamics.py:81-104) on libbcmpc.

``GPUFitter`` owns one ``bcmpc_fitter`` (include/bcmpc.h): the f32 parameters and
the Adam slots on the device, persisting across ``fit`` calls like the
reference's TF optimizer variables (dynamics.py:50-52).  All arithmetic runs in
the HIP kernels of ``csrc/fit.hip``; this file only marshals arrays.

Batches: the reference draws each step's rows with ``DataBufferGeneral.sample``
(data_buffer.py:45-57), i.e. ``random.sample(buffer, min(size, batch_size))`` on
Python's global ``random`` stream.  ``sample_batches`` draws the same row indices
in the same order (``random.sample`` depends only on the population length), so a
seeded run fits on exactly the reference's batches.
"""
from __future__ import annotations

import ctypes
import random
from typing import List, Sequence, Tuple

import numpy as np

from . import _lib
from .engine import MLPSpec, _ACT, _f32, _f64

_FP = ctypes.POINTER(ctypes.c_float)
_DP = ctypes.POINTER(ctypes.c_double)


def sample_batches(size: int, batch_size: int, iterations: int, rng=random) -> List[np.ndarray]:
    """Row indices of ``iterations`` DataBufferGeneral.sample calls (data_buffer.py:45-52)."""
    k = size if size < batch_size else batch_size
    return [np.asarray(rng.sample(range(size), k), dtype=np.int64) for _ in range(iterations)]


class GPUFitter:
    """``model="reward"``: NNDynamicsRewardModel.fit (dynamics.py:195-219) -- loss_dynamic + loss_reward
    over the two-head net; parameters dense .. dense_4 (+ LayerNorm trunk / delta / reward); n_layers 2,
    tanh.  ``set_rewards`` gives the buffer's reward column, ``reward_losses`` the last run's reward
    losses."""

    def __init__(self, state_dim: int, action_dim: int, hidden: int, n_layers: int, activation: str,
                 layer_norm: bool, batch_size: int, learning_rate: float, device: int = 0,
                 beta1: float = 0.9, beta2: float = 0.999, epsilon: float = 1e-8, model: str = "delta"):
        self._lib = _lib.load()
        if activation not in _ACT:
            raise ValueError(f"unsupported activation {activation!r}")
        if model not in ("delta", "reward"):
            raise ValueError("model must be 'delta' or 'reward'")
        c = _lib.FitConfig(int(state_dim), int(action_dim), int(hidden), int(n_layers), _ACT[activation],
                           int(bool(layer_norm)), int(batch_size), int(device), float(learning_rate),
                           float(beta1), float(beta2), float(epsilon),
                           _lib.MODEL_REWARD if model == "reward" else _lib.MODEL_DELTA)
        self.model = model
        h = ctypes.c_void_p()
        _lib.check(self._lib.bcmpc_fit_create(ctypes.byref(c), ctypes.byref(h)), fit=True)
        self._h = h
        self.S, self.A, self.hidden, self.L = state_dim, action_dim, hidden, n_layers
        self.layer_norm = bool(layer_norm)
        self.batch_size = batch_size

    def set_params(self, spec: MLPSpec, normalization: Sequence) -> None:
        ks = [_f32(k) for k in spec.kernels]
        bs = [_f32(b) for b in spec.biases]
        w = _lib.Weights()
        w.kernels = (_FP * len(ks))(*[k.ctypes.data_as(_FP) for k in ks])
        w.biases = (_FP * len(bs))(*[b.ctypes.data_as(_FP) for b in bs])
        keep = [ks, bs]
        if self.layer_norm:
            gs = [_f32(g) for g in spec.ln_gamma]
            bes = [_f32(b) for b in spec.ln_beta]
            w.ln_gamma = (_FP * len(gs))(*[g.ctypes.data_as(_FP) for g in gs])
            w.ln_beta = (_FP * len(bes))(*[b.ctypes.data_as(_FP) for b in bes])
            keep += [gs, bes]
        stats = [_f64(normalization[i]) for i in (0, 1, 2, 3, 8, 9)]
        (w.mean_obs, w.std_obs, w.mean_action, w.std_action, w.mean_deltas, w.std_deltas) = \
            [x.ctypes.data_as(_DP) for x in stats]
        if self.model == "reward":                    # dynamics.py:203 (mean_reward / std_reward)
            rstats = [_f64(normalization[4]).reshape(-1)[:1], _f64(normalization[5]).reshape(-1)[:1]]
            w.mean_reward, w.std_reward = [x.ctypes.data_as(_DP) for x in rstats]
            keep.append(rstats)
        _lib.check(self._lib.bcmpc_fit_set_params(self._h, ctypes.byref(w)), fit=True)
        del keep

    def get_params(self) -> Tuple[List[np.ndarray], List[np.ndarray], list, list]:
        S, A, h, L = self.S, self.A, self.hidden, self.L
        if self.model == "reward":
            shapes = [(S + A, h), (h, h), (h, S), (h, h), (h, 1)]
            nln = 3
        else:
            dims = [S + A] + [h] * L + [S]
            shapes = [(dims[i], dims[i + 1]) for i in range(L + 1)]
            nln = L
        ks = [np.empty(sh, np.float32) for sh in shapes]
        bs = [np.empty(sh[1], np.float32) for sh in shapes]
        gs = [np.empty(h, np.float32) for _ in range(nln)] if self.layer_norm else []
        bes = [np.empty(h, np.float32) for _ in range(nln)] if self.layer_norm else []
        arr = lambda xs: (_FP * max(1, len(xs)))(*[x.ctypes.data_as(_FP) for x in xs])  # noqa: E731
        _lib.check(self._lib.bcmpc_fit_get_params(self._h, arr(ks), arr(bs), arr(gs) if gs else None,
                                                  arr(bes) if bes else None), fit=True)
        return ks, bs, gs, bes

    def set_data(self, states, actions, deltas) -> None:
        s, a, d = _f64(states), _f64(actions), _f64(deltas)
        n = s.shape[0]
        if s.shape != (n, self.S) or a.shape != (n, self.A) or d.shape != (n, self.S):
            raise ValueError("data: states [n, S], actions [n, A], deltas [n, S]")
        _lib.check(self._lib.bcmpc_fit_set_data(self._h, s.ctypes.data_as(_DP), a.ctypes.data_as(_DP),
                                                d.ctypes.data_as(_DP), n), fit=True)

    def set_rewards(self, rewards) -> None:
        r = np.ascontiguousarray(np.asarray(rewards, dtype=np.float64).reshape(-1))
        _lib.check(self._lib.bcmpc_fit_set_rewards(self._h, r.ctypes.data_as(_DP), r.shape[0]), fit=True)

    def reward_losses(self, iterations: int) -> np.ndarray:
        out = np.empty(iterations, dtype=np.float32)
        _lib.check(self._lib.bcmpc_fit_reward_losses(self._h, out.ctypes.data_as(_FP)), fit=True)
        return out

    def run(self, batches: Sequence[np.ndarray]) -> np.ndarray:
        """One Adam step per index array; returns each step's loss (before its update)."""
        sizes = np.asarray([len(b) for b in batches], dtype=np.int32)
        idx = np.ascontiguousarray(np.concatenate(batches) if len(batches) else np.zeros(0), dtype=np.int64)
        losses = np.empty(len(batches), dtype=np.float32)
        _lib.check(self._lib.bcmpc_fit_run(
            self._h, idx.ctypes.data_as(ctypes.POINTER(ctypes.c_int64)),
            sizes.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), len(batches),
            losses.ctypes.data_as(_FP)), fit=True)
        return losses

    def close(self) -> None:
        if getattr(self, "_h", None):
            self._lib.bcmpc_fit_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def buffer_arrays_reward(data) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray]:
    """(states, actions, rewards, deltas) of a DataBufferGeneral(.., 5) (items [ob, ac, rew, nxt_ob,
    nxt_ob - ob], data.sample's order, dynamics.py:200) or of a 4-tuple in that order."""
    if isinstance(data, tuple):
        return tuple(np.asarray(x, dtype=np.float64) for x in data)
    items = list(data.buffer)
    return (np.asarray([it[0] for it in items], np.float64), np.asarray([it[1] for it in items], np.float64),
            np.asarray([np.asarray(it[2], np.float64).reshape(-1)[0] for it in items], np.float64),
            np.asarray([it[4] for it in items], np.float64))


def buffer_arrays(data) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(states, actions, deltas) of a DataBufferGeneral(.., 5) (items [ob, ac, rew, nxt_ob, nxt_ob - ob],
    train_mpc_ppo.py:156-160, :300) or of a (states, actions, deltas) tuple."""
    if isinstance(data, tuple):
        return tuple(np.asarray(x, dtype=np.float64) for x in data)
    items = list(data.buffer)
    return (np.asarray([it[0] for it in items], np.float64), np.asarray([it[1] for it in items], np.float64),
            np.asarray([it[4] for it in items], np.float64))
