"""Weight magnitudes far from the synthetic glorot range, against the oracle.

The reference's trained weights (saved_data/ppo-mpc/vars.pkl) cannot be read with an allowed loader
(tests/golden/PROVENANCE.json records both refusals), so the kernels' power-of-two operand scaling is
exercised here by rescaling the synthetic nets instead:

* relu + LayerNorm (train_mpc_ppo.py:52,74-75,539's 2x256 net) on the team kernel, whose last LayerNorm
  is deferred behind the output layer (rollout_team.hip DEFER): dense_1 and its bias scaled by s.  relu
  is homogeneous and LayerNorm divides the scale out again, so the costs barely move while the
  activations the kernel splits into hi / lo f16 halves span 1e-3 .. 1e3 (the centred
  activations now carry the wave's column power of two, as the relu path's do);
* the same without LayerNorm (the DYN column scale);
* the 2x500 tanh net on the split (rollout_x3) and fp32 (rollout_grp) slab kernels with per-layer scale
  patterns: saturated tanh layers, a small hidden kernel, a large / small output kernel.

Same tolerance and envelope as test_gpu_team.py / test_gpu_parity.py (the envelope times the output
kernel's scale where that scale exceeds 1: the cost is linear in it)."""
import numpy as np
import pytest

from conftest import envelope
from oracle import mpc_oracle as orc

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-4, 1e-5


def _check(costs, want, near, best_index, label, env):
    d = np.abs(costs - want)
    tol = np.minimum(ATOL + RTOL * np.abs(want), env)
    bad = d > tol
    bad &= ~(near & (np.abs(d - 10.0 * np.round(d / 10.0)) <= tol))
    print(f"[{label}] max|dcost|={np.nanmax(d):.2e} max|cost|={np.nanmax(np.abs(want)):.3g}")
    assert not bad.any(), f"{label}: {int(bad.sum())} candidates outside the tolerance, worst {np.nanmax(d):.3e}"
    assert best_index == int(np.argmin(costs))
    order = np.sort(want)
    i = int(np.argmin(want))
    if order[1] - order[0] > 2 * (ATOL + RTOL * abs(order[0])) and not near[i]:
        assert best_index == i


def _scaled(hidden, act, ln, scales, seed_base):
    w = orc.synthetic_weights(20, 6, hidden, 2, act, ln, seed_base=seed_base)
    ks = [(k * np.float32(s)).astype(np.float32) for k, s in zip(w.kernels, scales)]
    bs = [(b * np.float32(s)).astype(np.float32) for b, s in zip(w.biases, scales)]
    return orc.MLPWeights(ks, bs, act, w.ln_gamma, w.ln_beta)


def _run(w, K, H, kernel, label, env):
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    norm = orc.synthetic_normalization(seed=3)
    eng = RolloutEngine(20, 6, w.hidden, 2, w.activation, w.ln_gamma is not None, H, K, kernel=kernel)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), norm, 1)
    state = orc.synthetic_state(norm, seed=4)
    res = eng.get_action(state, None, seed=77, return_costs=True)
    ap = orc.device_rng_actions(77, 0, K, H, -np.ones(6), np.ones(6))
    want, paths = orc.rollout(orc.NumpyDynamics(w, norm), state, ap)
    layout = eng.info()["layout"]
    eng.close()
    _check(res.costs, want, orc.near_threshold_mask(paths), res.best_index, f"{label} {layout}", env)
    return layout


@pytest.mark.parametrize("s", [1e-3, 1e-2, 1e2, 1e3])
@pytest.mark.parametrize("K,H,hidden", [(400, 7, 256), (77, 5, 200)])
def test_team_relu_ln_deferred_layernorm_any_scale(K, H, hidden, s):
    w = _scaled(hidden, "relu", True, [1.0, s, 1.0], seed_base=41 + hidden)
    layout = _run(w, K, H, "team", f"team relu+LN h{hidden} dense_1 x{s:g}", envelope(True, 2, hidden, H))
    assert layout.startswith("rollout_team")


@pytest.mark.parametrize("s", [1e-3, 10.0])
def test_team_relu_column_scale_any_scale(s):
    # (no LayerNorm: the deltas, and so the cost, scale with s -- the envelope with them)
    w = _scaled(256, "relu", False, [1.0, s, 1.0], seed_base=297)
    _run(w, 400, 7, "team", f"team relu h256 dense_1 x{s:g}", envelope(False, 2, 256, 7) * max(1.0, s))


PATTERNS = [  # (dense, dense_1, dense_2) scale factors
    (4.0, 0.25, 8.0),      # saturated first tanh layer, small hidden kernel, large output kernel
    (0.25, 4.0, 0.125),    # near-linear first layer, saturated second, small output kernel
]


@pytest.mark.parametrize("kernel", ["split4", "group4"])
@pytest.mark.parametrize("pattern", PATTERNS)
def test_slab_kernels_tanh_2x500_scaled_layers(kernel, pattern):
    w = _scaled(500, "tanh", False, list(pattern), seed_base=541)
    # (the absolute envelope grows with the output kernel's scale: the cost is linear in it)
    _run(w, 2048, 20, kernel, f"{kernel} 2x500 tanh x{pattern}", envelope(False, 2, 500, 20) * max(1.0, pattern[2]))
