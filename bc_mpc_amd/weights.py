"""Pull the dynamics-MLP weights and normalization out of a ``dyn_model``.

``MPCcontroller`` receives ``dyn_model`` (controllers.py:30) and the reference
only ever calls ``dyn_model.predict`` (controllers.py:70).  The engine instead
runs the MLP on the GPU, so it needs the weights.  Supported containers:

1. ``bc_mpc_amd.dynamics.NNDynamicsModel`` (the torch weight container),
2. any object whose ``.weights`` has ``kernels``/``biases``/``activation``
   (+ ``ln_gamma``/``ln_beta``) -- e.g. NumPy stand-ins of NNDynamicsModel,
3. the reference's TF1 ``dynamics.NNDynamicsModel``: variables
   ``NNDynamicsModel/dense{,_1,..}/{kernel,bias}:0`` and
   ``NNDynamicsModel/LayerNorm{,_1,..}/{gamma,beta}:0`` read through its
   ``sess`` (dynamics.py:31-38, 44); the activation is read from the graph's
   op types.  Its ``fit`` (dynamics.py:81) is wrapped to bump a version stamp
   so weights are re-synced after every refit (train_mpc_ppo.py:279).

The learned-reward net of ``NNDynamicsRewardModel`` (dynamics.py:121-238) is
recognised by its shape -- five dense layers in TF creation order, the last
``[h, 1]`` (dense_4, the reward output) -- and read into an ``MLPSpec`` with
``model="reward"``.

Normalization stats are the attributes set at dynamics.py:41 / :143.
"""
from __future__ import annotations

import hashlib
import re
from typing import List, Tuple

import numpy as np

from .engine import MLPSpec

_NORM_ATTRS = ("mean_obs", "std_obs", "mean_action", "std_action", "mean_reward", "std_reward",
               "mean_nxt_state", "std_nxt_state", "mean_deltas", "std_deltas")


_NORM_CACHE: dict = {}      # id(model) -> (the attribute objects, their f64 arrays, generation): slotted models


def _norm_entry(dyn_model):
    """(attribute objects, f64 arrays, generation) of the model's normalisation: converted once per set
    of attribute objects (get_action asks every env step; the reference fixes them at construction,
    dynamics.py:41); the generation counts the sets seen, kept on the model object itself."""
    objs = [getattr(dyn_model, name, None) for name in _NORM_ATTRS]
    hit = getattr(dyn_model, "_bcmpc_norm_cache", None)
    if hit is None:
        hit = _NORM_CACHE.get(id(dyn_model))
    if hit is not None:
        for a, b in zip(hit[0], objs):
            if a is not b:
                break
        else:
            return hit
    out = [np.zeros(1) if v is None else np.asarray(v, dtype=np.float64) for v in objs]
    entry = (objs, out, 0 if hit is None else hit[2] + 1)
    try:
        dyn_model._bcmpc_norm_cache = entry
    except AttributeError:                                  # (a slotted object)
        if len(_NORM_CACHE) > 64:
            _NORM_CACHE.clear()
        _NORM_CACHE[id(dyn_model)] = entry
    return entry


def normalization_of(dyn_model) -> List[np.ndarray]:
    """The 10-tuple of normalisation vectors (utils.py:143-158 order) as f64 arrays."""
    return _norm_entry(dyn_model)[1]


def _with_norm(version: int, gen: int) -> int:
    """The engine's weights version: the model's own stamp with the normalisation generation folded in,
    so replacing a normalisation attribute re-uploads it (set_weights is idempotent on the version)."""
    return ((int(version) & (2**47 - 1)) << 16) | (gen & 0xFFFF)


def _act_name(act) -> str:
    if isinstance(act, str):
        return act.lower()
    name = getattr(act, "__name__", "") or type(act).__name__
    name = name.lower()
    if "tanh" in name:
        return "tanh"
    if "relu" in name:
        return "relu"
    raise ValueError(f"unsupported activation {act!r}")


def is_reward_net(kernels) -> bool:
    """dense, dense_1, dense_2, dense_3, dense_4 of NNDynamicsRewardModel.build_network
    (dynamics.py:150-177): trunk [S+A,h], two [h,h] head layers, outputs [h,S] and [h,1]."""
    if len(kernels) != 5:
        return False
    sh = [tuple(np.shape(k)) for k in kernels]
    h = sh[0][1]
    return sh[1] == (h, h) and sh[3] == (h, h) and sh[2][0] == h and sh[4] == (h, 1)


def _tf_weights(dyn_model, tf=None) -> MLPSpec:
    """Read NNDynamicsModel's variables (dynamics.py:54-71 under scope "NNDynamicsModel", :31)
    through its session: ``dense{,_1,..}/{kernel,bias}:0`` and ``LayerNorm{,_1,..}/{gamma,beta}:0``
    exactly (the Adam slots ``.../kernel/Adam:0`` are not fetched); the activation from the op
    types under ``scope/dense``.  ``tf``: the tensorflow module (default: the imported one; TF1 is
    absent in this image, tests install a stand-in)."""
    if tf is None:
        import tensorflow as tf
    scope = getattr(dyn_model, "scope", "NNDynamicsModel")
    pat = re.compile(rf"{re.escape(scope)}/(dense|LayerNorm)(?:_(\d+))?/(kernel|bias|gamma|beta):0$")
    found = {}
    for v in tf.global_variables():
        m = pat.match(v.name)
        if m:
            found[(m.group(1), 0 if m.group(2) is None else int(m.group(2)), m.group(3))] = v
    keys = sorted(found)
    vals = dict(zip(keys, dyn_model.sess.run([found[k] for k in keys])))
    dense = sorted({i for (kind, i, _) in keys if kind == "dense"})
    kernels = [vals[("dense", i, "kernel")] for i in dense]
    biases = [vals[("dense", i, "bias")] for i in dense]
    lns = sorted({i for (kind, i, _) in keys if kind == "LayerNorm"})
    g = [vals[("LayerNorm", i, "gamma")] for i in lns] or None
    b = [vals[("LayerNorm", i, "beta")] for i in lns] or None
    ops = {op.type for op in dyn_model.sess.graph.get_operations() if op.name.startswith(scope + "/dense")}
    act = "tanh" if "Tanh" in ops else "relu"
    model = "reward" if hasattr(dyn_model, "reward_predict") and is_reward_net(kernels) else "delta"
    return MLPSpec(kernels, biases, act, g, b, model=model)


def _install_fit_hook(dyn_model) -> None:
    if getattr(dyn_model, "_bcmpc_fit_hooked", False) or not hasattr(dyn_model, "fit"):
        return
    fit = dyn_model.fit

    def fit_and_bump(*args, **kwargs):
        out = fit(*args, **kwargs)
        dyn_model._bcmpc_version = getattr(dyn_model, "_bcmpc_version", 1) + 1
        return out

    dyn_model.fit = fit_and_bump
    dyn_model._bcmpc_version = getattr(dyn_model, "_bcmpc_version", 1)
    dyn_model._bcmpc_fit_hooked = True


def _cached(dyn_model, version: int, make):
    """The spec built for ``version`` (kept on the model object): get_action runs once per env
    step, the weights change once per refit."""
    hit = getattr(dyn_model, "_bcmpc_spec_cache", None)
    if hit is not None and hit[0] == version:
        return hit[1]
    spec = make()
    try:
        dyn_model._bcmpc_spec_cache = (version, spec)
    except AttributeError:                                  # (a slotted object: no cache)
        pass
    return spec


def weight_token(dyn_model):
    """A cheap token that changes whenever extract(dyn_model) could return different weights or
    normalisation: the model's version stamp (ours, or the fit hook's on the reference's TF model) and
    the identities of its normalisation attribute objects.  None when the model has no stamp (the
    weights are digested by content each call)."""
    if hasattr(dyn_model, "mlp_spec"):
        v = int(dyn_model.version)
    elif hasattr(dyn_model, "sess") and getattr(dyn_model, "_bcmpc_fit_hooked", False):
        v = int(dyn_model._bcmpc_version)
    else:
        return None
    return (v,) + tuple(getattr(dyn_model, name, None) for name in _NORM_ATTRS)


def same_token(dyn_model, token) -> bool:
    """weight_token(dyn_model) would equal ``token`` (the version, then the normalisation objects by
    identity -- the token holds them, so their ids cannot be reused)."""
    t = weight_token(dyn_model)
    return t is not None and t[0] == token[0] and all(a is b for a, b in zip(t[1:], token[1:]))


def extract(dyn_model) -> Tuple[MLPSpec, List[np.ndarray], int]:
    """Return ``(spec, normalization10, version)`` for the engine (``version``: the weights' stamp with
    the normalisation generation folded in, _with_norm)."""
    _, norm, gen = _norm_entry(dyn_model)
    if hasattr(dyn_model, "mlp_spec"):                      # bc_mpc_amd.dynamics.NNDynamicsModel
        v = int(dyn_model.version)
        return _cached(dyn_model, v, dyn_model.mlp_spec), norm, _with_norm(v, gen)
    w = getattr(dyn_model, "weights", None)
    if w is not None and hasattr(w, "kernels"):             # NumPy stand-ins
        kernels = [np.asarray(k) for k in w.kernels]
        spec = MLPSpec(kernels, [np.asarray(b) for b in w.biases],
                       _act_name(getattr(w, "activation", "tanh")),
                       getattr(w, "ln_gamma", None), getattr(w, "ln_beta", None),
                       model="reward" if is_reward_net(kernels) else "delta")
        version = getattr(dyn_model, "version", None)
        if version is None:      # no stamp: content digest (~1 MB of weights, <1 ms)
            d = hashlib.blake2b(digest_size=8)
            for a in list(w.kernels) + list(w.biases) + list(getattr(w, "ln_gamma", None) or []) \
                    + list(getattr(w, "ln_beta", None) or []):
                d.update(np.ascontiguousarray(a, dtype=np.float32).tobytes())
            version = int.from_bytes(d.digest(), "little") & (2**63 - 1)
        return spec, norm, _with_norm(int(version), gen)
    if hasattr(dyn_model, "sess"):                          # reference TF1 NNDynamicsModel
        _install_fit_hook(dyn_model)
        v = int(dyn_model._bcmpc_version)                   # (variables read once per refit)
        return _cached(dyn_model, v, lambda: _tf_weights(dyn_model)), norm, _with_norm(v, gen)
    raise TypeError(f"cannot read dynamics weights from {type(dyn_model).__name__}")
