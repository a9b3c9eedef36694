"""Shape sweep of the split-f16 kernel against the oracle: odd K (partial columns and
workgroups), H = 1..7, every padded width the kernel instantiates (64..1024), L = 1..3, each
candidate-group width (split1/2/4), with and without the fused policy / reward heads.  Same
tolerance as test_gpu_parity.py (|dcost| <= 1e-4 + 1e-5 |cost|, a +-10 flip only on the
oracle's near-threshold candidates); the argmin and its first action must match whenever the
oracle's top-2 gap decides them.  Device Philox actions (no [H, K, A] upload), oracle replays
of the same draws (oracle.device_rng_actions)."""
import numpy as np
import pytest

from conftest import ENV_PLAIN, envelope
from oracle import mpc_oracle as orc

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-4, 1e-5

DELTA = [  # (K, H, hidden, L, kernel)
    (1, 1, 64, 1, "split1"), (17, 3, 64, 2, "split2"), (65, 2, 100, 2, "split1"), (200, 4, 128, 3, "split4"),
    (129, 5, 200, 2, "split2"), (300, 3, 256, 2, "split4"), (97, 2, 300, 1, "split1"), (257, 4, 500, 2, "split4"),
    (130, 3, 512, 3, "split2"), (70, 2, 600, 2, "split1"), (150, 2, 768, 2, "split2"), (90, 2, 1000, 3, "split2"),
    # the one-column layout at hidden 512 keeps its own layer-1 k-steps resident (X3_RES): L = 1 (no hidden
    # layer, nothing resident), L = 2, L = 3 (layer 2 streamed from k-step kown as before)
    (33, 2, 480, 1, "split1"), (70, 4, 500, 2, "split1"), (130, 3, 512, 3, "split1"),
]


def _check(costs, want, near, best_index, first, actions_h0, label, env=ENV_PLAIN):
    """The stated tolerance AND the achieved envelope ``env`` (conftest.envelope)."""
    d = np.abs(costs - want)
    tol = np.minimum(ATOL + RTOL * np.abs(want), env)
    bad = d > tol
    bad &= ~(near & (np.abs(d - 10.0 * np.round(d / 10.0)) <= tol))
    print(f"[{label}] max|dcost|={np.nanmax(d) if d.size else 0:.2e}")
    assert np.array_equal(np.isnan(costs), np.isnan(want)) and not bad.any()
    assert best_index == int(np.argmin(costs))
    order = np.sort(want[~np.isnan(want)])
    i = int(np.argmin(want))
    if len(order) < 2 or order[1] - order[0] > 2 * (ATOL + RTOL * abs(order[0])) and not near[i]:
        assert best_index == i and np.array_equal(first, actions_h0[i])


@pytest.mark.parametrize("K,H,hidden,L,kernel", DELTA)
def test_split_delta_shapes(K, H, hidden, L, kernel):
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    norm = orc.synthetic_normalization(seed=3)
    w = orc.synthetic_weights(20, 6, hidden, L, "tanh", False, seed_base=31 + hidden)
    state = orc.synthetic_state(norm, seed=4)
    try:
        eng = RolloutEngine(20, 6, hidden, L, "tanh", False, H, K, kernel=kernel)
    except ValueError as e:                                  # a width this NC does not instantiate
        pytest.skip(str(e))
    eng.set_weights(MLPSpec(w.kernels, w.biases, "tanh"), norm, 1)
    res = eng.get_action(state, None, seed=1234, cand_offset=5, return_costs=True)
    ap = orc.device_rng_actions(1234, 5, K, H, -np.ones(6), np.ones(6))
    dyn = orc.NumpyDynamics(w, norm)
    want, paths = orc.rollout(dyn, state, ap)
    near = orc.near_threshold_mask(paths)
    _check(res.costs, want, near, res.best_index - 5, res.first_action, ap[0], f"{kernel} K{K} H{H} {L}x{hidden}",
           env=envelope(False, L, hidden, H))
    eng.close()


@pytest.mark.parametrize("K,H,hidden,kernel", [(33, 3, 64, "split1"), (140, 2, 200, "split2"),
                                               (300, 4, 500, "split4"), (77, 2, 256, "split4")])
def test_split_reward_shapes(K, H, hidden, kernel):
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    norm = orc.synthetic_normalization(20, 6, seed=5, reward=True)
    w = orc.synthetic_reward_weights(20, 6, hidden, False, seed_base=7 + hidden)
    state = orc.synthetic_state(norm, seed=6)
    try:
        eng = RolloutEngine(20, 6, hidden, 2, "tanh", False, H, K, cost="reward", model="reward", kernel=kernel)
    except ValueError as e:
        pytest.skip(str(e))
    eng.set_weights(MLPSpec(w.kernels, w.biases, "tanh", model="reward"), norm, 1)
    eng.set_discount(0.95)
    res = eng.get_action(state, None, seed=99, return_costs=True)
    ap = orc.device_rng_actions(99, 0, K, H, -np.ones(6), np.ones(6))
    want, _ = orc.reward_rollout(orc.NumpyRewardDynamics(w, norm), state, ap, 0.95)
    d = np.abs(res.costs - want)
    print(f"[reward {kernel} K{K} H{H} {hidden}] max|dr|={d.max():.2e}")
    assert (d <= ATOL + RTOL * np.abs(want)).all()
    assert res.best_index == int(np.argmax(res.costs))


ACTLN = [  # (K, H, hidden, L, activation, layer_norm, kernel): the relu / LayerNorm split variants
    (65, 3, 64, 2, "relu", False, "split1"), (300, 2, 128, 1, "relu", False, "split4"),
    (200, 4, 256, 2, "relu", True, "split4"), (97, 3, 200, 3, "relu", True, "split2"),
    (130, 3, 500, 2, "relu", False, "split2"), (70, 5, 500, 2, "relu", True, "split1"),
    (257, 2, 512, 2, "tanh", True, "split2"), (150, 2, 256, 2, "tanh", True, "split4"),
    (90, 2, 100, 2, "tanh", True, "split1"),
]


@pytest.mark.parametrize("K,H,hidden,L,act,ln,kernel", ACTLN)
def test_split_relu_layernorm_shapes(K, H, hidden, L, act, ln, kernel):
    """relu hidden layers (per-column power-of-two scales exchanged across the workgroup) and
    LayerNorm (column statistics exchanged, dynamics.py:68-69) in the split kernel vs the oracle."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    norm = orc.synthetic_normalization(seed=8)
    w = orc.synthetic_weights(20, 6, hidden, L, act, ln, seed_base=57 + hidden)
    state = orc.synthetic_state(norm, seed=9)
    eng = RolloutEngine(20, 6, hidden, L, act, ln, H, K, kernel=kernel)
    assert eng.precision == "split"
    eng.set_weights(MLPSpec(w.kernels, w.biases, act, w.ln_gamma, w.ln_beta), norm, 1)
    res = eng.get_action(state, None, seed=77, cand_offset=3, return_costs=True)
    ap = orc.device_rng_actions(77, 3, K, H, -np.ones(6), np.ones(6))
    want, paths = orc.rollout(orc.NumpyDynamics(w, norm), state, ap)
    near = orc.near_threshold_mask(paths)
    _check(res.costs, want, near, res.best_index - 3, res.first_action, ap[0],
           f"{kernel} {act}{'+LN' if ln else ''} K{K} H{H} {L}x{hidden}", env=envelope(ln, L, hidden, H))
    eng.close()
