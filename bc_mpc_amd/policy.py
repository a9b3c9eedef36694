"""Read the policy net MPCcontrollerPolicyNet consults (controllers.py:160-178).

Supported containers:

1. objects exposing ``policy_spec()`` (returns an ``engine.PolicySpec``),
2. NumPy stand-ins with ``.w.kernels/.biases/.ob_mean/.ob_std/.logstd``,
3. the reference's TF1 ``ppo_bc_policy.MlpPolicy`` (ppo_bc_policy.py:15-88):
   ``pi/pi/pol/fc{1..L}/{kernel,bias}:0``, ``pi/pi/pol/final/{kernel,bias}:0``,
   ``pi/pi/pol/logstd:0`` and the baselines RunningMeanStd under
   ``pi/pi/obfilter`` (``runningsum``, ``runningsumsq``, ``count``) -- the
   scope is doubled because ``build_network(sess, 'pi', ob)`` opens
   ``'pi/pol'`` inside ``variable_scope('pi')`` (ppo_bc_policy.py:31-32, 56,
   64) -- read through ``.sess``; mean = f32(sum/count), std =
   sqrt(max(f32(sumsq/count) - mean^2, 1e-2)) exactly as RunningMeanStd
   builds them.  TF1 is absent here: (3) is tested against a stand-in graph
   with the reference's variable names (tests/test_tf_readers.py).

The policy changes every PPO update, and there is no hook for it, so the
version stamp is a content digest (the 20->128->128->6 stack is ~80 KB), taken
every control step: xxh3-64 over the arrays in place (~10 GB/s; blake2b, ~1 GB/s,
when xxhash is not importable).  A container with an integer ``version``
attribute is trusted instead (no digest).
"""
from __future__ import annotations

import hashlib
from typing import Tuple

import numpy as np

from .engine import PolicySpec


try:
    import xxhash as _xxhash
except Exception:  # pragma: no cover - installed in this image
    _xxhash = None


def _digest(spec: PolicySpec) -> int:
    d = _xxhash.xxh3_64() if _xxhash is not None else hashlib.blake2b(digest_size=8)
    shapes = []
    for a in list(spec.kernels) + list(spec.biases) + [spec.ob_mean, spec.ob_std, spec.logstd]:
        if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous):
            a = np.ascontiguousarray(a, dtype=np.float32)
        d.update(a)                                                # (the buffer in place, no copy)
        shapes.append(a.shape)
    d.update(repr(shapes).encode())
    return int.from_bytes(d.digest(), "little") & (2**63 - 1)


def _policy_prefix(names, scope: str) -> str:
    """MlpPolicy builds its net as ``build_network(sess, 'pi', ob)`` INSIDE ``tf.variable_scope('pi')``
    (ppo_bc_policy.py:31-32, 56, 64), so the variables are ``pi/pi/pol/fc1/kernel:0``,
    ``pi/pi/obfilter/runningsum:0`` ...; ``pi_scope`` is the outer scope ``'pi'``.  A net built
    directly under ``scope`` (``scope/pol/...``) is accepted too."""
    for p in (f"{scope}/{scope}", scope):
        if f"{p}/pol/fc1/kernel:0" in names and f"{p}/obfilter/runningsum:0" in names:
            return p
    raise KeyError(f"no MlpPolicy variables under {scope!r}: expected '{scope}/{scope}/pol/fc1/kernel:0' "
                   f"(ppo_bc_policy.py:31-32,64)")


def _tf_policy(policy_net, tf=None) -> PolicySpec:
    """Read the 'pi' policy of ppo_bc_policy.MlpPolicy through its session.  Only the pol/
    and obfilter/ variables are fetched (not vf/, old_pi/ or the Adam slots): this runs on
    every env step to compute the version digest.  ``tf``: the tensorflow module (default: the
    imported one; TF1 itself is absent in this image, tests install a stand-in)."""
    if tf is None:
        import tensorflow as tf
    scope = getattr(policy_net, "pi_scope", "pi")
    by_name = {v.name: v for v in tf.global_variables()}
    p = _policy_prefix(by_name, scope)
    L = int(getattr(policy_net, "num_hid_layers"))
    want = ([f"{p}/pol/fc{i + 1}/{w}:0" for w in ("kernel", "bias") for i in range(L)]
            + [f"{p}/pol/final/kernel:0", f"{p}/pol/final/bias:0", f"{p}/pol/logstd:0",
               f"{p}/obfilter/runningsum:0", f"{p}/obfilter/runningsumsq:0", f"{p}/obfilter/count:0"])
    vals = dict(zip(want, policy_net.sess.run([by_name[n] for n in want])))
    ks = [vals[f"{p}/pol/fc{i + 1}/kernel:0"] for i in range(L)] + [vals[f"{p}/pol/final/kernel:0"]]
    bs = [vals[f"{p}/pol/fc{i + 1}/bias:0"] for i in range(L)] + [vals[f"{p}/pol/final/bias:0"]]
    ssum = vals[f"{p}/obfilter/runningsum:0"]
    ssq = vals[f"{p}/obfilter/runningsumsq:0"]
    cnt = vals[f"{p}/obfilter/count:0"]
    mean = (ssum / cnt).astype(np.float32)
    std = np.sqrt(np.maximum((ssq / cnt).astype(np.float32) - np.square(mean), np.float32(1e-2)))
    logstd = np.asarray(vals[f"{p}/pol/logstd:0"]).reshape(-1)
    return PolicySpec(ks, bs, mean, std.astype(np.float32), logstd.astype(np.float32))


def int_version(policy_net):
    """The policy container's own integer ``version`` (trusted, as by extract), else None."""
    v = getattr(policy_net, "version", None)
    return v if isinstance(v, int) and not isinstance(v, bool) else None


def extract(policy_net) -> Tuple[PolicySpec, int]:
    if hasattr(policy_net, "policy_spec"):
        spec = policy_net.policy_spec()
    elif hasattr(policy_net, "w") and hasattr(policy_net.w, "ob_mean"):
        w = policy_net.w
        spec = PolicySpec([np.asarray(k) for k in w.kernels], [np.asarray(b) for b in w.biases],
                          np.asarray(w.ob_mean), np.asarray(w.ob_std), np.asarray(w.logstd))
    elif hasattr(policy_net, "sess"):
        spec = _tf_policy(policy_net)
    else:
        raise TypeError(f"cannot read policy weights from {type(policy_net).__name__}")
    v = getattr(policy_net, "version", None)
    if isinstance(v, int) and not isinstance(v, bool):
        return spec, v
    return spec, _digest(spec)
