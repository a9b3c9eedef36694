"""GPU parity of MCTScontrollerPolicyNetReward (controllers.py:365-457) on the engine.

The first-stage actions are pinned to their restatement: the stochastic policy's
``mean + exp(logstd) * N(0, 1)`` with the engine's Philox normals
(``oracle.device_rng_normals``), the deterministic policy's mean (``NumpyPolicy.mean``), or the
env's own ``action_space.sample()`` draws (bit-identical).  Given those actions, the rest of the
search -- one ``predict`` from the root, R tiled follow-up paths under the deterministic policy,
the reward sums, their mean, the argmax -- is compared with ``oracle.mcts_get_action``, the NumPy
restatement of controllers.py:397-457.  Tolerance as test_gpu_reward.py: totals within
1e-4 + 1e-5 |r|; the argmax exact when the top-2 gap exceeds twice that.  Parity against TF itself
is unpinned (TF1 is absent; the stochastic draws are TF's in the reference).
"""
import numpy as np
import pytest

from test_gpu_reward import ATOL, RTOL, _Env, assert_rewards_close

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("hidden", [64, 500])
@pytest.mark.parametrize("mode", ["stochastic", "mean", "env"])
def test_mcts_matches_oracle(mode, hidden):
    from bc_mpc_amd import MCTScontrollerPolicyNetReward
    from oracle import mpc_oracle as orc
    S, A, N, R, H = 20, 6, 12, 5, 6
    norm = orc.synthetic_normalization(S, A, seed=5, reward=True)
    w = orc.synthetic_reward_weights(S, A, hidden, False, seed_base=321)
    p = orc.synthetic_policy(S, A, 128, 2, seed=9)
    state = orc.synthetic_state(norm, seed=6)
    dyn, pol = orc.NumpyRewardDynamics(w, norm), orc.NumpyPolicy(p)
    ctrl = MCTScontrollerPolicyNetReward(_Env(S, A, seed=3), dyn, pol, explore=0.3, self_exp=(mode == "stochastic"),
                                         horizon=H, num_first_stage_actions=N, random_path_per_action=R,
                                         random_first_stage_action=(mode == "env"), seed=77)
    a = ctrl.get_action(state)
    assert a.shape == (1, A) and a.dtype == np.float32
    first = ctrl.last_first_actions
    mean = pol.mean(state)[0].astype(np.float64)
    if mode == "env":
        probe = _Env(S, A, seed=3)
        action_1s = [np.expand_dims(probe.action_space.sample(), axis=0) for _ in range(N)]
        assert np.array_equal(first, np.concatenate(action_1s).astype(np.float64))   # U exactly (explore = 1)
    else:
        if mode == "stochastic":
            want = mean + np.exp(p.logstd.astype(np.float64)) * orc.device_rng_normals(ctrl.last_seeds[0], 0, N, 0, A)
        else:
            want = np.tile(mean, (N, 1))
        err = np.abs(first - want)
        print(f"[mcts {mode} h{hidden}] max|dfirst|={err.max():.3e}")
        assert (err <= 2e-5 + 2e-5 * np.abs(want)).all()
        action_1s = [first[i:i + 1].astype(np.float32) for i in range(N)]
    best, total, r1, rall = orc.mcts_get_action(dyn, pol, state, H, action_1s, R)
    assert np.allclose(rall, rall[:, :1], rtol=1e-6, atol=1e-6)   # R follow-ups per first action (BLAS rounding)
    assert_rewards_close(ctrl.last_total_rewards, total, f"mcts {mode} h{hidden}")
    srt = np.sort(total)[::-1]
    gap = srt[0] - srt[1] if N > 1 else np.inf
    if mode == "mean":                                     # N identical first actions: a tie, lowest index
        assert np.all(ctrl.last_total_rewards == ctrl.last_total_rewards[0]) and ctrl.last_index == 0
    elif gap > 2 * (ATOL + RTOL * abs(srt[0])):
        assert ctrl.last_index == best
        assert np.array_equal(a, action_1s[best])
    ctrl.close()


def test_mcts_reference_quirks():
    """sample_random_actions reads num_simulated_paths, which __init__ never sets (controllers.py:390-395):
    an AttributeError there as in the reference; an empty first stage is an argmax of nothing."""
    from bc_mpc_amd import MCTScontrollerPolicyNetReward
    from oracle import mpc_oracle as orc
    S, A = 20, 6
    norm = orc.synthetic_normalization(S, A, seed=5, reward=True)
    w = orc.synthetic_reward_weights(S, A, 64, False, seed_base=321)
    ctrl = MCTScontrollerPolicyNetReward(_Env(S, A), orc.NumpyRewardDynamics(w, norm),
                                         orc.NumpyPolicy(orc.synthetic_policy(S, A, 128, 2, seed=9)),
                                         num_first_stage_actions=0)
    with pytest.raises(AttributeError):
        ctrl.sample_random_actions()
    with pytest.raises(ValueError):
        ctrl.get_action(orc.synthetic_state(norm, seed=6))
