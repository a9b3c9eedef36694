"""The TF1 variable readers (bc_mpc_amd/weights.py, bc_mpc_amd/policy.py) against a stand-in
graph that names its variables exactly as the reference's TF1 code does.  TensorFlow itself is
absent in this image, so the stand-in installs a minimal ``tensorflow`` module with
``global_variables()`` and a session whose ``run`` returns the stored arrays.

Names follow the reference:
* NNDynamicsModel (dynamics.py:31-38, 54-71): ``NNDynamicsModel/dense{,_1,_2}/{kernel,bias}:0``,
  ``NNDynamicsModel/LayerNorm{,_1}/{gamma,beta}:0``, plus the AdamOptimizer slots
  ``.../kernel/Adam:0`` that ``minimize`` adds (dynamics.py:50-52);
* MlpPolicy (ppo_bc_policy.py:31-32, 54-80): ``build_network(sess, 'pi', ob)`` inside
  ``variable_scope('pi')`` -> ``pi/pi/obfilter/{runningsum,runningsumsq,count}:0``,
  ``pi/pi/vf/...``, ``pi/pi/pol/fc{1,2}/{kernel,bias}:0``, ``pi/pi/pol/final/...``,
  ``pi/pi/pol/logstd:0``; the same under ``old_pi/old_pi`` (:35-37); Adam slots.
"""
import sys
import types

import numpy as np
import pytest

from bc_mpc_amd import policy as bpol
from bc_mpc_amd import weights as bw


class _Var:
    def __init__(self, name):
        self.name = name


class _Op:
    def __init__(self, name, type_):
        self.name, self.type = name, type_


class _Sess:
    def __init__(self, values, ops=()):
        self.values = values
        self.fetched = []
        self.graph = types.SimpleNamespace(get_operations=lambda: list(ops))

    def run(self, fetches):
        self.fetched.append([v.name for v in fetches])
        return [self.values[v.name] for v in fetches]


@pytest.fixture
def fake_tf(monkeypatch):
    mod = types.ModuleType("tensorflow")
    mod._vars = []
    mod.global_variables = lambda: list(mod._vars)
    monkeypatch.setitem(sys.modules, "tensorflow", mod)
    return mod


def _register(tf, values):
    tf._vars = [_Var(n) for n in values]


def test_dynamics_reader_reference_names(fake_tf):
    rs = np.random.RandomState(0)
    S, A, h = 20, 6, 32
    vals = {}
    shapes = [(S + A, h), (h, h), (h, S)]
    for i, (fi, fo) in enumerate(shapes):
        sfx = "" if i == 0 else f"_{i}"
        vals[f"NNDynamicsModel/dense{sfx}/kernel:0"] = rs.randn(fi, fo).astype(np.float32)
        vals[f"NNDynamicsModel/dense{sfx}/bias:0"] = rs.randn(fo).astype(np.float32)
        vals[f"NNDynamicsModel/dense{sfx}/kernel/Adam:0"] = np.zeros((fi, fo), np.float32)
        vals[f"NNDynamicsModel/dense{sfx}/kernel/Adam_1:0"] = np.zeros((fi, fo), np.float32)
    for i in range(2):
        sfx = "" if i == 0 else f"_{i}"
        vals[f"NNDynamicsModel/LayerNorm{sfx}/gamma:0"] = rs.randn(h).astype(np.float32)
        vals[f"NNDynamicsModel/LayerNorm{sfx}/beta:0"] = rs.randn(h).astype(np.float32)
    vals["beta1_power:0"] = np.float32(0.9)
    _register(fake_tf, vals)
    ops = [_Op("NNDynamicsModel/dense/Relu", "Relu"), _Op("NNDynamicsModel/dense/MatMul", "MatMul")]
    sess = _Sess(vals, ops)
    fits = []

    class RefModel:                      # dynamics.NNDynamicsModel's attributes (dynamics.py:31-48)
        def __init__(self):
            self.sess = sess
            self.scope = "NNDynamicsModel"
            (self.mean_obs, self.std_obs, self.mean_action, self.std_action, self.mean_reward, self.std_reward,
             self.mean_nxt_state, self.std_nxt_state, self.mean_deltas, self.std_deltas) = (
                np.zeros(S), np.ones(S), np.zeros(A), np.ones(A), np.zeros(1), np.ones(1),
                np.zeros(S), np.ones(S), np.zeros(S), np.ones(S))

        def fit(self, data):
            fits.append(data)

    m = RefModel()
    spec, norm, v0 = bw.extract(m)
    assert spec.model == "delta" and spec.activation == "relu" and spec.n_layers == 2 and spec.hidden == h
    for i in range(3):
        sfx = "" if i == 0 else f"_{i}"
        assert np.array_equal(spec.kernels[i], vals[f"NNDynamicsModel/dense{sfx}/kernel:0"])
        assert np.array_equal(spec.biases[i], vals[f"NNDynamicsModel/dense{sfx}/bias:0"])
    assert spec.layer_norm and np.array_equal(spec.ln_gamma[1], vals["NNDynamicsModel/LayerNorm_1/gamma:0"])
    assert not any("Adam" in n or "power" in n for n in sess.fetched[-1])     # slots are not fetched
    # cached per version: a second call reads nothing; a refit bumps the version and re-reads
    spec2, _, v1 = bw.extract(m)
    assert v1 == v0 and len(sess.fetched) == 1 and spec2 is spec
    m.fit("buffer")
    assert fits == ["buffer"]
    _, _, v2 = bw.extract(m)
    assert v2 != v0 and len(sess.fetched) == 2


def _policy_values(rs, prefix, S, A, ph, L):
    vals = {}
    dims = [S] + [ph] * L
    for i in range(L):
        for part in ("pol", "vf"):
            vals[f"{prefix}/{part}/fc{i + 1}/kernel:0"] = rs.randn(dims[i], ph).astype(np.float32)
            vals[f"{prefix}/{part}/fc{i + 1}/bias:0"] = rs.randn(ph).astype(np.float32)
    vals[f"{prefix}/pol/final/kernel:0"] = rs.randn(ph, A).astype(np.float32)
    vals[f"{prefix}/pol/final/bias:0"] = rs.randn(A).astype(np.float32)
    vals[f"{prefix}/vf/final/kernel:0"] = rs.randn(ph, 1).astype(np.float32)
    vals[f"{prefix}/pol/logstd:0"] = rs.randn(1, A).astype(np.float32)
    vals[f"{prefix}/obfilter/runningsum:0"] = rs.randn(S) * 50.0              # f64, as RunningMeanStd
    vals[f"{prefix}/obfilter/runningsumsq:0"] = np.abs(rs.randn(S)) * 900.0 + 500.0
    vals[f"{prefix}/obfilter/count:0"] = np.float64(377.0)
    vals[f"{prefix}/pol/fc1/kernel/Adam:0"] = np.zeros((S, ph), np.float32)
    return vals


def test_policy_reader_reference_names(fake_tf):
    rs = np.random.RandomState(1)
    S, A, ph, L = 20, 6, 16, 2
    vals = _policy_values(rs, "pi/pi", S, A, ph, L)
    vals.update(_policy_values(rs, "old_pi/old_pi", S, A, ph, L))
    _register(fake_tf, vals)
    sess = _Sess(vals)
    pnet = types.SimpleNamespace(sess=sess, pi_scope="pi", num_hid_layers=L)
    spec, ver = bpol.extract(pnet)
    p = "pi/pi"
    assert [k.shape for k in spec.kernels] == [(S, ph), (ph, ph), (ph, A)]
    assert np.array_equal(spec.kernels[0], vals[f"{p}/pol/fc1/kernel:0"])
    assert np.array_equal(spec.kernels[2], vals[f"{p}/pol/final/kernel:0"])
    assert np.array_equal(spec.biases[1], vals[f"{p}/pol/fc2/bias:0"])
    assert np.array_equal(spec.logstd, vals[f"{p}/pol/logstd:0"].reshape(-1))
    # RunningMeanStd (baselines): mean = to_float(sum / count), std = sqrt(max(to_float(sumsq / count) - mean^2, 1e-2))
    cnt = vals[f"{p}/obfilter/count:0"]
    mean = (vals[f"{p}/obfilter/runningsum:0"] / cnt).astype(np.float32)
    std = np.sqrt(np.maximum((vals[f"{p}/obfilter/runningsumsq:0"] / cnt).astype(np.float32) - np.square(mean),
                             np.float32(1e-2)))
    assert np.array_equal(spec.ob_mean, mean) and np.array_equal(spec.ob_std, std.astype(np.float32))
    fetched = sess.fetched[-1]
    assert all(n.startswith("pi/pi/pol/") or n.startswith("pi/pi/obfilter/") for n in fetched)
    assert not any("Adam" in n or "/vf/" in n for n in fetched)
    # the digest changes with the weights
    vals[f"{p}/pol/fc1/bias:0"] = vals[f"{p}/pol/fc1/bias:0"] + np.float32(1.0)
    _, ver2 = bpol.extract(pnet)
    assert ver2 != ver


def test_policy_reader_rejects_missing_scope(fake_tf):
    vals = _policy_values(np.random.RandomState(2), "other/other", 20, 6, 8, 1)
    _register(fake_tf, vals)
    pnet = types.SimpleNamespace(sess=_Sess(vals), pi_scope="pi", num_hid_layers=1)
    with pytest.raises(KeyError, match="pi/pi/pol/fc1/kernel:0"):
        bpol.extract(pnet)
