"""GPU NNDynamicsModel.fit (csrc/fit.hip) against the oracle restatement (oracle.fit, dynamics.py:81-104).

Tolerance (stated): the GPU and the oracle run the same f32 ops in different
summation orders, so per-step losses agree to rtol 1e-4.  Adam moves every
parameter by ~lr * sign(m) early on, so a gradient within rounding of 0 may
step the other way: parameters are compared as max |dw| <= 2.5 lr (one flipped
step) with the median |dw| <= 1e-6.
"""
import numpy as np
import pytest

from oracle import mpc_oracle as orc

pytestmark = pytest.mark.gpu


def _data(n, S=20, A=6, seed=5):
    rs = np.random.RandomState(seed)
    norm = orc.synthetic_normalization(S, A)
    states = norm[0] + norm[1] * rs.standard_normal((n, S))
    actions = rs.uniform(-1, 1, (n, A))
    deltas = norm[8] + norm[9] * rs.standard_normal((n, S))
    return norm, states, actions, deltas


@pytest.mark.parametrize("hidden,L,act,ln,B", [(64, 2, "tanh", False, 128), (256, 2, "relu", True, 512),
                                              (500, 2, "tanh", False, 512), (96, 3, "tanh", True, 77)])
@pytest.mark.parametrize("fused", ["1", "0"])
def test_fit_matches_oracle(hidden, L, act, ln, B, fused, monkeypatch):
    """fused: the two-launch iteration (fit_rows_kernel + fit_params_kernel, the default);
    "0": the per-op kernels (BCMPC_FIT_FUSED=0)."""
    monkeypatch.setenv("BCMPC_FIT_FUSED", fused)
    from bc_mpc_amd.engine import MLPSpec
    from bc_mpc_amd.fit import GPUFitter
    lr, iters = 1e-3, 6
    w = orc.synthetic_weights(20, 6, hidden, L, act, ln, seed_base=11)
    norm, states, actions, deltas = _data(2000)
    rs = np.random.RandomState(9)
    batches = [rs.choice(2000, B, replace=False) for _ in range(iters)]
    f = GPUFitter(20, 6, hidden, L, act, ln, B, lr, device=0)
    f.set_params(MLPSpec(w.kernels, w.biases, act, w.ln_gamma, w.ln_beta), norm)
    f.set_data(states, actions, deltas)
    got = f.run(batches)
    ps = orc.fit_params(w)
    st = orc.AdamState.zeros_like(ps)
    want = orc.fit(ps, st, L, act, ln, norm, states, actions, deltas, batches, lr)
    print(f"[{hidden}x{L} {act} ln={ln}] losses gpu {got} oracle {np.array(want)}")
    assert np.allclose(got, want, rtol=1e-4, atol=0)
    ks, bs, gs, bes = f.get_params()
    mine = []
    for k, b in zip(ks, bs):
        mine += [k, b]
    if ln:
        for g, be in zip(gs, bes):
            mine += [g, be]
    d = np.concatenate([np.abs(a - b).ravel() for a, b in zip(mine, ps)])
    print(f"   params max|dw|={d.max():.3e} median={np.median(d):.3e}")
    assert d.max() <= 2.5 * lr and np.median(d) <= 1e-6
    # a second run continues the Adam state (beta powers, m, v) like the reference's optimizer
    got2 = f.run(batches[:2])
    want2 = orc.fit(ps, st, L, act, ln, norm, states, actions, deltas, batches[:2], lr)
    assert np.allclose(got2, want2, rtol=1e-4, atol=0)
    f.close()


def test_model_fit_dropin_updates_weights_and_engine():
    """bc_mpc_amd.dynamics.NNDynamicsModel.fit(DataBufferGeneral-like) -> (loss, 0); the weights
    change, the version bumps, and predict (the rollout kernel) uses the new weights."""
    import random
    from collections import deque
    from bc_mpc_amd.dynamics import NNDynamicsModel

    class Space:
        def __init__(self, n):
            self.shape = (n,)

    class Env:
        observation_space, action_space = Space(20), Space(6)

    norm, states, actions, deltas = _data(600)

    class Buf:                                   # DataBufferGeneral(.., 5) (data_buffer.py:29-57)
        buffer = deque([[states[i], actions[i], 0.0, states[i] + deltas[i], deltas[i]] for i in range(600)])
        size = 600

    m = NNDynamicsModel(Env(), 2, 64, "relu", None, norm, batch_size=128, iterations=20, learning_rate=1e-3,
                        layer_norm=True, device=0)
    before = [k.clone() for k in m.kernels]
    v0 = m.version
    random.seed(7)
    p0 = m.predict(states[:32], actions[:32])
    loss, zero = m.fit(Buf())
    assert zero == 0 and np.isfinite(loss) and m.version > v0
    assert any(not np.array_equal(a.numpy(), b.numpy()) for a, b in zip(before, m.kernels))
    p1 = m.predict(states[:32], actions[:32])
    assert not np.array_equal(p0, p1)
    # the oracle on the same batches (random.sample stream) reproduces the loss
    from bc_mpc_amd.fit import sample_batches
    random.seed(7)
    batches = sample_batches(600, 128, 20)
    w = orc.MLPWeights([k.numpy() for k in before], [np.zeros_like(b.numpy()) for b in m.biases], "relu",
                       [np.ones(64, np.float32)] * 2, [np.zeros(64, np.float32)] * 2)
    ps = orc.fit_params(w)
    want = orc.fit(ps, orc.AdamState.zeros_like(ps), 2, "relu", True, norm, states, actions, deltas, batches, 1e-3)
    assert np.isclose(loss, want[-1], rtol=1e-3)


def test_fit_graph_and_launch_paths_identical(monkeypatch):
    """A uniform-batch run executes as one captured graph; ragged batches (and BCMPC_FIT_GRAPH=0)
    launch per iteration.  Same kernels, same device iteration state: bit-identical results."""
    from bc_mpc_amd.engine import MLPSpec
    from bc_mpc_amd.fit import GPUFitter
    w = orc.synthetic_weights(20, 6, 128, 2, "relu", True, seed_base=3)
    norm, states, actions, deltas = _data(1500)
    rs = np.random.RandomState(4)
    batches = [rs.choice(1500, 256, replace=False) for _ in range(12)]
    out = []
    for graph in ("1", "0"):
        monkeypatch.setenv("BCMPC_FIT_GRAPH", graph)
        f = GPUFitter(20, 6, 128, 2, "relu", True, 256, 1e-3, device=0)
        f.set_params(MLPSpec(w.kernels, w.biases, "relu", w.ln_gamma, w.ln_beta), norm)
        f.set_data(states, actions, deltas)
        l1 = f.run(batches[:8])
        l2 = f.run(batches[8:])                   # a second run continues the Adam state
        out.append((np.concatenate([l1, l2]), f.get_params()))
        f.close()
    assert np.array_equal(out[0][0], out[1][0])
    for a, b in zip(out[0][1], out[1][1]):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    # ragged batches take the launch path and still match the oracle
    ps = orc.fit_params(w)
    ragged = [rs.choice(1500, n, replace=False) for n in (256, 100, 256, 7)]
    monkeypatch.setenv("BCMPC_FIT_GRAPH", "1")
    f = GPUFitter(20, 6, 128, 2, "relu", True, 256, 1e-3, device=0)
    f.set_params(MLPSpec(w.kernels, w.biases, "relu", w.ln_gamma, w.ln_beta), norm)
    f.set_data(states, actions, deltas)
    got = f.run(ragged)
    want = orc.fit(ps, orc.AdamState.zeros_like(ps), 2, "relu", True, norm, states, actions, deltas, ragged, 1e-3)
    assert np.allclose(got, want, rtol=1e-4, atol=0)
    f.close()


def _reward_data(n, S=20, A=6, seed=6):
    norm = orc.synthetic_normalization(S, A, reward=True)
    _, states, actions, deltas = _data(n, S, A, seed)
    rs = np.random.RandomState(seed + 1)
    mr, sr = float(np.asarray(norm[4]).reshape(-1)[0]), float(np.asarray(norm[5]).reshape(-1)[0])
    rewards = mr + sr * rs.standard_normal(n)
    return norm, states, actions, rewards, deltas


@pytest.mark.parametrize("hidden,ln,B", [(500, True, 512), (500, False, 512), (64, True, 77)])
def test_fit_reward_matches_oracle(hidden, ln, B):
    """NNDynamicsRewardModel.fit on the GPU (GPUFitter model="reward": loss_dynamic + loss_reward over the
    two-head net, dynamics.py:153-160, 195-219) against oracle.fit_reward on the same batches: both
    losses of every step (rtol 1e-4) and the parameters (one flipped Adam step), then a second run
    continuing the Adam state.  hidden 500 with LayerNorm is run.sh's model (train_mpc_ppo.py:52)."""
    from bc_mpc_amd.engine import MLPSpec
    from bc_mpc_amd.fit import GPUFitter
    lr, iters = 1e-3, 6
    w = orc.synthetic_reward_weights(20, 6, hidden, ln, seed_base=31)
    norm, states, actions, rewards, deltas = _reward_data(2000)
    rs = np.random.RandomState(10)
    batches = [rs.choice(2000, B, replace=False) for _ in range(iters)]
    f = GPUFitter(20, 6, hidden, 2, "tanh", ln, B, lr, device=0, model="reward")
    f.set_params(MLPSpec(w.kernels, w.biases, "tanh", w.ln_gamma, w.ln_beta, model="reward"), norm)
    f.set_data(states, actions, deltas)
    f.set_rewards(rewards)
    got_d = f.run(batches)
    got_r = f.reward_losses(iters)
    ps = orc.fit_reward_params(w)
    st = orc.AdamState.zeros_like(ps)
    want = orc.fit_reward(ps, st, ln, norm, states, actions, rewards, deltas, batches, lr)
    want_d, want_r = np.array([x[0] for x in want]), np.array([x[1] for x in want])
    print(f"[reward fit h{hidden} ln={ln}] dyn gpu {got_d} oracle {want_d}; rew gpu {got_r} oracle {want_r}")
    assert np.allclose(got_d, want_d, rtol=1e-4, atol=0)
    assert np.allclose(got_r, want_r, rtol=1e-4, atol=0)
    ks, bs, gs, bes = f.get_params()
    mine = []
    for k, b in zip(ks, bs):
        mine += [k, b]
    if ln:
        for g, be in zip(gs, bes):
            mine += [g, be]
    assert len(mine) == len(ps)
    d = np.concatenate([np.abs(a - b).ravel() for a, b in zip(mine, ps)])
    print(f"   params max|dw|={d.max():.3e} median={np.median(d):.3e}")
    assert d.max() <= 2.5 * lr and np.median(d) <= 1e-6
    got2 = f.run(batches[:2])
    want2 = orc.fit_reward(ps, st, ln, norm, states, actions, rewards, deltas, batches[:2], lr)
    assert np.allclose(got2, [x[0] for x in want2], rtol=1e-4, atol=0)
    assert np.allclose(f.reward_losses(2), [x[1] for x in want2], rtol=1e-4, atol=0)
    f.close()


def test_reward_model_fit_dropin():
    """bc_mpc_amd.dynamics.NNDynamicsRewardModel.fit(DataBufferGeneral-like) returns the last step's
    (model_loss, reward_loss) like dynamics.py:219, bumps the version, and predict uses the new weights;
    the losses are the oracle's on the same random.sample batches."""
    import random
    from collections import deque
    from bc_mpc_amd.dynamics import NNDynamicsRewardModel
    from bc_mpc_amd.fit import sample_batches

    class Space:
        def __init__(self, n):
            self.shape = (n,)

    class Env:
        observation_space, action_space = Space(20), Space(6)

    norm, states, actions, rewards, deltas = _reward_data(700)

    class Buf:                                   # DataBufferGeneral(.., 5): [ob, ac, rew, nxt_ob, nxt_ob - ob]
        buffer = deque([[states[i], actions[i], rewards[i], states[i] + deltas[i], deltas[i]] for i in range(700)])
        size = 700

    m = NNDynamicsRewardModel(Env(), norm, 128, 15, 1e-3, layer_norm=True, size=96, device=0)
    w0 = orc.RewardMLPWeights([k.numpy().copy() for k in m.kernels], [b.numpy().copy() for b in m.biases],
                              [g.numpy().copy() for g in m.ln_gamma], [b.numpy().copy() for b in m.ln_beta])
    v0 = m.version
    p0 = m.predict(states[:16], actions[:16])
    random.seed(11)
    model_loss, reward_loss = m.fit(Buf())
    assert np.isfinite(model_loss) and np.isfinite(reward_loss) and m.version > v0
    p1 = m.predict(states[:16], actions[:16])
    assert not np.array_equal(p0[1], p1[1])
    random.seed(11)
    batches = sample_batches(700, 128, 15)
    ps = orc.fit_reward_params(w0)
    want = orc.fit_reward(ps, orc.AdamState.zeros_like(ps), True, norm, states, actions, rewards, deltas, batches,
                          1e-3)
    assert np.isclose(model_loss, want[-1][0], rtol=1e-3) and np.isclose(reward_loss, want[-1][1], rtol=1e-3)
