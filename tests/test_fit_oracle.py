"""CPU checks of the fit restatement (oracle.fit_*, dynamics.py:44-52, 81-104) and of the
batch sampler (bc_mpc_amd.fit.sample_batches vs DataBufferGeneral.sample, data_buffer.py:45-57)."""
import random
from collections import deque

import numpy as np
import pytest

from oracle import mpc_oracle as orc


@pytest.mark.parametrize("act,ln", [("tanh", False), ("relu", True), ("tanh", True), ("relu", False)])
def test_fit_grads_match_finite_differences(act, ln):
    """The hand-written backward (incl. the LayerNorm autodiff with TF1's stop_gradient on the
    mean inside the variance) against central differences of the same forward, in f64."""
    w = orc.synthetic_weights(5, 3, 12, 2, act, ln, seed_base=3)
    ps = [p.astype(np.float64) for p in orc.fit_params(w)]
    rs = np.random.RandomState(0)
    x0, t = rs.standard_normal((7, 8)), rs.standard_normal((7, 5))
    _, g = orc.fit_grads(ps, 2, act, ln, x0, t, dtype=np.float64)
    worst = 0.0
    for pi in range(len(ps)):
        for k in range(0, ps[pi].size, max(1, ps[pi].size // 7)):
            e = 1e-6
            p2 = [q.copy() for q in ps]
            p2[pi].flat[k] += e
            lp, _ = orc.fit_grads(p2, 2, act, ln, x0, t, dtype=np.float64)
            p2[pi].flat[k] -= 2 * e
            lm, _ = orc.fit_grads(p2, 2, act, ln, x0, t, dtype=np.float64)
            num = (lp - lm) / (2 * e)
            worst = max(worst, abs(num - g[pi].flat[k]) / (abs(num) + 1e-5))
    assert worst < 1e-4, worst


def test_adam_first_step_matches_closed_form():
    """TF1 ApplyAdam step 1: m = (1-b1) g, v = (1-b2) g^2, lr_t = lr sqrt(1-b2)/(1-b1) =>
    w' = w - lr_t m / (sqrt(v) + eps) ~ w - lr sign(g)."""
    p = [np.array([1.0, -2.0, 0.5], np.float32)]
    g = [np.array([0.3, -4.0, 1e-3], np.float32)]
    st = orc.AdamState.zeros_like(p)
    orc.adam_apply(p, g, st, 1e-3)
    assert np.allclose(p[0], [1.0 - 1e-3, -2.0 + 1e-3, 0.5 - 1e-3], atol=2e-6)
    assert st.beta1_power == np.float32(0.9) * np.float32(0.9)


def test_sample_batches_draws_the_reference_rows():
    """DataBufferGeneral.sample = random.sample(deque, min(size, num)): same RNG draws as
    random.sample(range(size), k) -> the same rows in the same order."""
    from bc_mpc_amd.fit import sample_batches
    items = deque([[np.full(3, i, float), np.zeros(2), 0.0, np.zeros(3), np.zeros(3)] for i in range(50)])
    for size, num in [(50, 16), (50, 64)]:
        random.seed(123)
        ref = []
        for _ in range(4):                       # data_buffer.py:45-52
            batch = random.sample(items, size) if size < num else random.sample(items, num)
            ref.append([int(b[0][0]) for b in batch])
        random.seed(123)
        got = sample_batches(size, num, 4)
        assert [list(map(int, g)) for g in got] == ref


@pytest.mark.parametrize("ln", [False, True])
def test_fit_reward_grads_match_finite_differences(ln):
    """NNDynamicsRewardModel's loss_dynamic + loss_reward (dynamics.py:153-157) over the two-head net
    (dynamics.py:165-177): the hand-written backward (both heads' gradients summed into the trunk, each
    head's and the trunk's LayerNorm autodiff) against central differences of the same forward, f64."""
    w = orc.synthetic_reward_weights(5, 3, 12, ln, seed_base=21)
    ps = [p.astype(np.float64) for p in orc.fit_reward_params(w)]
    assert len(ps) == (16 if ln else 10)
    rs = np.random.RandomState(1)
    x0, t, r = rs.standard_normal((7, 8)), rs.standard_normal((7, 5)), rs.standard_normal((7, 1))
    _, _, g = orc.fit_reward_grads(ps, ln, x0, t, r, dtype=np.float64)

    def loss(p2):
        ld, lr_, _ = orc.fit_reward_grads(p2, ln, x0, t, r, dtype=np.float64)
        return ld + lr_
    worst = 0.0
    for pi in range(len(ps)):
        for k in range(0, ps[pi].size, max(1, ps[pi].size // 7)):
            e = 1e-6
            p2 = [q.copy() for q in ps]
            p2[pi].flat[k] += e
            lp = loss(p2)
            p2[pi].flat[k] -= 2 * e
            lm = loss(p2)
            num = (lp - lm) / (2 * e)
            worst = max(worst, abs(num - g[pi].flat[k]) / (abs(num) + 1e-5))
    assert worst < 1e-4, worst


def test_fit_reward_batch_normalises_like_the_reference():
    """dynamics.py:201-210: (x - mean) / (std + 1e-10) in f64 for states, actions, rewards and deltas,
    fed as f32, the reward as a [-1, 1] column."""
    norm = orc.synthetic_normalization(4, 2, reward=True)
    rs = np.random.RandomState(3)
    s, a, d = rs.standard_normal((5, 4)), rs.standard_normal((5, 2)), rs.standard_normal((5, 4))
    rw = rs.standard_normal(5)
    x0, t, r = orc.fit_reward_batch(norm, s, a, rw, d)
    assert x0.dtype == t.dtype == r.dtype == np.float32 and r.shape == (5, 1)
    want = ((rw - np.float64(np.asarray(norm[4]).reshape(-1)[0])) /
            (np.float64(np.asarray(norm[5]).reshape(-1)[0]) + 1e-10)).astype(np.float32)
    assert np.array_equal(r[:, 0], want)
