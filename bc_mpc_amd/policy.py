"""Read the policy net MPCcontrollerPolicyNet consults (controllers.py:160-178).

Supported containers:

1. objects exposing ``policy_spec()`` (returns an ``engine.PolicySpec``),
2. NumPy stand-ins with ``.w.kernels/.biases/.ob_mean/.ob_std/.logstd``,
3. the reference's TF1 ``ppo_bc_policy.MlpPolicy`` (ppo_bc_policy.py:15-88):
   ``pi/pol/fc{1..L}/{kernel,bias}:0``, ``pi/pol/final/{kernel,bias}:0``,
   ``pi/pol/logstd:0`` and the baselines RunningMeanStd under ``pi/obfilter``
   (``runningsum``, ``runningsumsq``, ``count``), read through ``.sess``;
   mean = f32(sum/count), std = sqrt(max(f32(sumsq/count) - mean^2, 1e-2))
   exactly as RunningMeanStd builds them.  TF1 is absent here, so (3) is
   implemented against that naming but untested in this image.

The policy changes every PPO update, and there is no hook for it, so the
version stamp is a content digest (the 20->128->128->6 stack is ~80 KB).
"""
from __future__ import annotations

import hashlib
from typing import Tuple

import numpy as np

from .engine import PolicySpec


def _digest(spec: PolicySpec) -> int:
    d = hashlib.blake2b(digest_size=8)
    for a in list(spec.kernels) + list(spec.biases) + [spec.ob_mean, spec.ob_std, spec.logstd]:
        d.update(np.ascontiguousarray(a, dtype=np.float32).tobytes())
    return int.from_bytes(d.digest(), "little") & (2**63 - 1)


def _tf_policy(policy_net) -> PolicySpec:  # pragma: no cover - TF1 is absent in this image
    import tensorflow as tf
    scope = getattr(policy_net, "pi_scope", "pi")
    var_list = [v for v in tf.global_variables() if v.name.startswith(scope + "/")]
    vals = dict(zip([v.name for v in var_list], policy_net.sess.run(var_list)))
    L = int(getattr(policy_net, "num_hid_layers"))
    ks = [vals[f"{scope}/pol/fc{i + 1}/kernel:0"] for i in range(L)] + [vals[f"{scope}/pol/final/kernel:0"]]
    bs = [vals[f"{scope}/pol/fc{i + 1}/bias:0"] for i in range(L)] + [vals[f"{scope}/pol/final/bias:0"]]
    ssum = vals[f"{scope}/obfilter/runningsum:0"]
    ssq = vals[f"{scope}/obfilter/runningsumsq:0"]
    cnt = vals[f"{scope}/obfilter/count:0"]
    mean = (ssum / cnt).astype(np.float32)
    std = np.sqrt(np.maximum((ssq / cnt).astype(np.float32) - np.square(mean), np.float32(1e-2)))
    logstd = vals[f"{scope}/pol/logstd:0"].reshape(-1)
    return PolicySpec(ks, bs, mean, std.astype(np.float32), logstd.astype(np.float32))


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
    return spec, _digest(spec)
