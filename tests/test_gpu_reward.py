"""GPU parity of the learned-reward paths: MPCcontrollerReward (controllers.py:90-158)
and MPCcontrollerPolicyNetReward (controllers.py:289-363) on the two-head
NNDynamicsRewardModel net (dynamics.py:121-238), against the reference-made
fixtures (tests/golden/gen_golden.py REWARD_CASES / POLICY_REWARD_CASES).

Tolerance (stated, fp32 MLP, same reasoning as test_gpu_parity.py): per-candidate
discounted reward sums agree to |r_gpu - r_ref| <= ATOL + RTOL*|r_ref| with
ATOL = 1e-4, RTOL = 1e-5 (there are no penalty thresholds in this objective);
NaN patterns are identical; the ARGMAX is exact whenever the reference's top-2
gap exceeds twice that tolerance, and the returned first action is then the
reference's.
"""
import numpy as np
import pytest

from conftest import ENV_PLAIN, RewardGolden, envelope, golden_names

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-4, 1e-5
REWARD = [n for n in golden_names("reward") if n.startswith("reward_")]
POLREW = [n for n in golden_names("reward") if n.startswith("polrew_")]


def _spec(g):
    from bc_mpc_amd.engine import MLPSpec
    w = g.weights
    return MLPSpec(w.kernels, w.biases, "tanh", w.ln_gamma, w.ln_beta, model="reward")


def assert_rewards_close(got, want, label="", env=ENV_PLAIN):
    """The stated tolerance AND the achieved envelope ``env`` (conftest.envelope)."""
    assert got.shape == want.shape
    assert np.array_equal(np.isnan(got), np.isnan(want)), f"{label}: NaN pattern differs"
    ok = ~np.isnan(want)
    diff = np.abs(got[ok] - want[ok])
    tol = np.minimum(ATOL + RTOL * np.abs(want[ok]), env)
    print(f"[{label}] max|dreward|={diff.max() if diff.size else 0:.3e} n={ok.sum()}")
    assert (diff <= tol).all(), f"{label}: {int((diff > tol).sum())} rewards outside tolerance; worst {diff.max():.3e}"


def decidable(g) -> bool:
    best = g.rewards[g.argmax]
    return bool(np.isnan(best)) or g.top2_gap > 2 * (ATOL + RTOL * abs(best))


def assert_tie_rule(g, rewards, best_index):
    """Exact ties (duplicated action paths, or explore=0 where every path is the policy's):
    when the GPU also ties them at its maximum, the LOWEST index wins (np.argmax)."""
    if np.isnan(g.rewards[g.argmax]):
        return
    tied = np.flatnonzero(g.rewards == g.rewards[g.argmax])
    if tied.size > 1 and np.all(rewards[tied] == np.nanmax(rewards)):
        assert best_index == tied[0]


class _Box:
    def __init__(self, A, seed=0):
        self.low = -np.ones(A, dtype=np.float32)
        self.high = np.ones(A, dtype=np.float32)
        self.shape = (A,)
        self.np_random = np.random.RandomState(seed)

    def sample(self):   # gym.spaces.Box.sample for a float32 Box
        return self.np_random.uniform(low=self.low, high=self.high, size=self.shape).astype(np.float32)


class _Env:
    def __init__(self, S, A, seed=0):
        self.action_space = _Box(A, seed)

        class obs:
            shape = (S,)
        self.observation_space = obs


def _skip_split(g, kernel):
    if kernel.startswith("split"):
        if g.weights.layer_norm:
            pytest.skip("split precision: nets without LayerNorm")
        if kernel == "split4" and g.weights.hidden <= 64:
            pytest.skip("split4 needs >= 4 waves (hidden > 64)")


@pytest.mark.parametrize("kernel", ["group4", "group8", "split1", "split2", "split4", "team"])
@pytest.mark.parametrize("name", REWARD)
def test_reward_engine_matches_reference_fixture(name, kernel):
    from bc_mpc_amd.engine import RolloutEngine
    g = RewardGolden(name)
    _skip_split(g, kernel)
    if kernel == "team" and not (448 < g.weights.hidden <= 512 and 0 < g.K <= 512):
        pytest.skip("team kernel, reward net: hidden 449..512, K <= 512")
    eng = RolloutEngine(g.S, g.A, g.weights.hidden, 2, "tanh", g.weights.layer_norm, g.H, g.K, device=0,
                        cost="reward", model="reward", kernel=kernel)
    assert eng.info()["kernel"] == kernel
    eng.set_weights(_spec(g), g.norm, 1)
    eng.set_discount(g.gamma)
    if g.meta.get("inject") == "philox":
        res = eng.get_action(g.state, None, seed=g.meta["rng_seed"], cand_offset=g.meta["cand_offset"],
                             return_costs=True)
        off = g.meta["cand_offset"]
    else:
        res = eng.get_action(g.state, g.env_actions(), return_costs=True)
        off = 0
    assert_rewards_close(res.costs, g.rewards, f"{name}/{kernel}", env=envelope(g.weights.layer_norm, 2,
                                                                             g.weights.hidden, g.H))
    assert res.best_index - off == int(np.argmax(res.costs))           # device argmax == np.argmax
    assert_tie_rule(g, res.costs, res.best_index - off)
    if decidable(g):
        assert res.best_index - off == g.argmax
        assert np.array_equal(res.first_action, g.opt_action, equal_nan=True)


@pytest.mark.parametrize("name", [n for n in REWARD if "device_rng" not in n])
def test_reward_controller_dropin(name):
    """MPCcontrollerReward with the reference's env-sampled actions: same action, same dtype."""
    from bc_mpc_amd import MPCcontrollerReward
    g = RewardGolden(name)
    if g.meta.get("inject"):
        pytest.skip("injected actions replace the env samples; covered by the engine test")
    env = _Env(g.S, g.A, seed=g.meta["seed"])
    ctrl = MPCcontrollerReward(env, g.dyn(), horizon=g.H, num_simulated_paths=g.K, gamma=g.gamma)
    ctrl.keep_costs = True
    a = ctrl.get_action(g.state)
    assert a.dtype == np.float32 and a.shape == (g.A,)          # copy of the float32 env samples
    assert_rewards_close(ctrl.last_rewards, g.rewards, name, env=envelope(g.weights.layer_norm, 2, g.weights.hidden, g.H))
    if decidable(g):
        assert ctrl.last_index == g.argmax
        assert np.array_equal(a.astype(np.float64), g.opt_action)
    # the env RNG advanced by exactly K*H samples (controllers.py:112-114)
    want_next = np.random.RandomState(g.meta["seed"]).uniform(-1, 1, size=(g.K * g.H + 1, g.A))[-1]
    assert np.array_equal(env.action_space.np_random.uniform(-1, 1, size=g.A), want_next)


@pytest.mark.parametrize("kernel", ["group4", "group8", "team"])
@pytest.mark.parametrize("name", POLREW)
def test_policy_reward_engine_matches_reference_fixture(name, kernel):
    from bc_mpc_amd.engine import PolicySpec, RolloutEngine
    g = RewardGolden(name)
    p = g.policy
    if kernel == "team" and not (448 < g.weights.hidden <= 512 and 0 < g.K <= 512
                                 and p.hidden <= 128 and p.n_layers <= 2):
        pytest.skip("team kernel, reward net + policy: hidden 449..512, policy <= 2 x 128, K <= 512")
    eng = RolloutEngine(g.S, g.A, g.weights.hidden, 2, "tanh", g.weights.layer_norm, g.H, g.K, device=0,
                        cost="reward", model="reward", kernel=kernel, policy_hidden=p.hidden,
                        policy_layers=p.n_layers, policy_mode="explore")
    if kernel == "team":
        assert eng.info()["kernel"] == "team"
    eng.set_weights(_spec(g), g.norm, 1)
    eng.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), g.explore, 1)
    expl = np.random.RandomState(g.meta["seed"]).uniform(g.low, g.high, size=[g.H, g.K, g.A])
    res = eng.get_action(g.state, expl, return_costs=True)
    assert_rewards_close(res.costs, g.rewards, f"{name}/{kernel}", env=envelope(g.weights.layer_norm, 2,
                                                                             g.weights.hidden, g.H))
    fa = eng.first_actions()
    err = np.abs(fa - g.z["first_actions"])
    print(f"[{name}/{kernel}] max|dfirst_action|={err.max():.3e}")
    assert (err <= 1e-6).all()
    assert res.best_index == int(np.argmax(res.costs))
    assert_tie_rule(g, res.costs, res.best_index)
    if decidable(g):
        assert res.best_index == g.argmax
        assert np.allclose(res.first_action, g.opt_action, rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", POLREW)
def test_policy_reward_controller_dropin(name):
    from bc_mpc_amd import MPCcontrollerPolicyNetReward
    from oracle import mpc_oracle as orc
    g = RewardGolden(name)
    env = _Env(g.S, g.A)
    ctrl = MPCcontrollerPolicyNetReward(env, g.dyn(), orc.NumpyPolicy(g.policy), explore=g.explore,
                                        self_exp=False, horizon=g.H, num_simulated_paths=g.K)
    np.random.seed(g.meta["seed"])
    a = ctrl.get_action(g.state)
    assert a.dtype == np.float64 and a.shape == (g.A,)
    if decidable(g):
        assert ctrl.last_index == g.argmax
        assert np.allclose(a, g.opt_action, rtol=0, atol=1e-6)
    assert np.random.random() == float(g.z["next_draw"])        # same global-RNG side effect


def test_reward_predict_container_matches_oracle():
    """bc_mpc_amd.dynamics.NNDynamicsRewardModel.predict (one kernel step, per-candidate
    states) vs the NumPy restatement of dynamics.py:225-238."""
    from bc_mpc_amd.dynamics import NNDynamicsRewardModel
    from oracle import mpc_oracle as orc
    S, A, K = 20, 6, 333
    norm = orc.synthetic_normalization(S, A, seed=3, reward=True)
    w = orc.synthetic_reward_weights(S, A, 500, True, seed_base=77)
    m = NNDynamicsRewardModel(_Env(S, A), norm, 512, 10, 1e-3, layer_norm=True, size=500)
    m.load_weights(w.kernels, w.biases, w.ln_gamma, w.ln_beta)
    rs = np.random.RandomState(9)
    s = orc.synthetic_state(norm)[None] + 0.1 * rs.standard_normal((K, S))
    a = rs.uniform(-1, 1, (K, A))
    ns, r = m.predict(s, a)
    ns_ref, r_ref = orc.NumpyRewardDynamics(w, norm).predict(s, a)
    assert ns.shape == (K, S) and r.shape == (K, 1)
    print(f"[predict] max|dstate|={np.abs(ns - ns_ref).max():.3e} max|dreward|={np.abs(r - r_ref).max():.3e}")
    assert np.allclose(ns, ns_ref, rtol=1e-5, atol=1e-6)
    assert np.allclose(r, r_ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize("kernel", ["auto", "group4"])
def test_reward_full_size_properties(kernel):
    """cfg3 shape on the learned-reward net (K=65536, H=20, 500-wide heads, device RNG):
    argmax agrees with np.argmax of the returned rewards, results are deterministic and
    shard-invariant, and a sample of candidates matches the oracle."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    S, A, K, H, h = 20, 6, 65536, 20, 500
    norm = orc.synthetic_normalization(S, A, seed=5, reward=True)
    w = orc.synthetic_reward_weights(S, A, h, False, seed_base=123)
    state = orc.synthetic_state(norm, seed=6)
    spec = MLPSpec(w.kernels, w.biases, "tanh", model="reward")

    def mk(k):
        e = RolloutEngine(S, A, h, 2, "tanh", False, H, k, cost="reward", model="reward", kernel=kernel)
        e.set_weights(spec, norm, 1)
        e.set_discount(0.99)
        return e
    full = mk(K)
    r1 = full.get_action(state, None, seed=2024, return_costs=True)
    r2 = full.get_action(state, None, seed=2024, return_costs=True)
    assert np.array_equal(r1.costs, r2.costs)
    assert r1.best_index == int(np.argmax(r1.costs)) and r1.best_cost == r1.costs.max()
    half = mk(K // 2)
    ra = half.get_action(state, None, seed=2024, cand_offset=0, return_costs=True)
    rb = half.get_action(state, None, seed=2024, cand_offset=K // 2, return_costs=True)
    assert np.array_equal(np.concatenate([ra.costs, rb.costs]), r1.costs)
    idx = np.random.RandomState(1).choice(K, 64, replace=False)
    idx[0] = r1.best_index
    for i in idx[:8]:                                      # a few single-candidate oracle replays
        ap = orc.device_rng_actions(2024, int(i), 1, H, -np.ones(A), np.ones(A))
        want, _ = orc.reward_rollout(orc.NumpyRewardDynamics(w, norm), state, ap, 0.99)
        assert abs(r1.costs[i] - want[0]) <= ATOL + RTOL * abs(want[0]), (i, r1.costs[i], want[0])
    first = orc.device_rng_actions(2024, r1.best_index, 1, 1, -np.ones(A), np.ones(A))[0, 0]
    assert np.array_equal(r1.first_action, first)


def test_reward_errors():
    from bc_mpc_amd import MPCcontroller
    from bc_mpc_amd.engine import RolloutEngine
    from oracle import mpc_oracle as orc
    g = RewardGolden(REWARD[0])
    with pytest.raises(TypeError):
        MPCcontroller(_Env(g.S, g.A), g.dyn(), horizon=2, num_simulated_paths=8).get_action(g.state)
    with pytest.raises(ValueError):
        RolloutEngine(20, 6, 128, 2, "tanh", False, 3, 64, cost="cheetah", model="reward")
    with pytest.raises(ValueError):
        RolloutEngine(20, 6, 128, 2, "relu", False, 3, 64, cost="reward", model="reward")
    with pytest.raises(ValueError):
        RolloutEngine(20, 6, 128, 3, "tanh", False, 3, 64, cost="reward", model="reward")
    delta = RolloutEngine(20, 6, 64, 2, "tanh", False, 3, 64)
    with pytest.raises(Exception):
        delta.set_discount(0.9)
    del orc


@pytest.mark.parametrize("mode", ["explore", "stochastic"])
def test_split_policy_reward_matches_fp32_engine(mode):
    """MPCcontrollerPolicyNetReward at hidden 500 (the run.sh recipe's net): the split kernel
    (reward heads + fused policy in split-f16) against the fp32 group kernel on the same draws."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    from oracle import mpc_oracle as orc
    S, A, K, H, h = 20, 6, 3000, 8, 500
    norm = orc.synthetic_normalization(S, A, seed=5, reward=True)
    w = orc.synthetic_reward_weights(S, A, h, False, seed_base=123)
    p = orc.synthetic_policy(S, A, 128, 2, seed=9)
    state = orc.synthetic_state(norm, seed=6)
    expl = np.random.RandomState(4).uniform(-1, 1, (H, K, A))
    out = {}
    for prec in ("fp32", "split"):
        e = RolloutEngine(S, A, h, 2, "tanh", False, H, K, cost="reward", model="reward", precision=prec,
                          policy_hidden=128, policy_layers=2, policy_mode=mode)
        e.set_weights(MLPSpec(w.kernels, w.biases, "tanh", model="reward"), norm, 1)
        e.set_discount(0.99)
        e.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), 0.5, 1)
        if prec == "split":
            assert e.info()["kernel"].startswith("split")
        r = e.get_action(state, expl, seed=13, return_costs=True)
        out[prec] = (r, e.first_actions())
        e.close()
    (r32, a32), (rsp, asp) = out["fp32"], out["split"]
    err = np.abs(asp - a32)
    print(f"[split polrew {mode}] max|dfirst|={err.max():.3e}")
    assert (err <= 2e-6).all()
    assert_rewards_close(rsp.costs, r32.costs, f"split polrew {mode}")
    assert rsp.best_index == int(np.argmax(rsp.costs))


@pytest.mark.parametrize("ln", [False, True], ids=["noln", "ln"])
@pytest.mark.parametrize("mode", ["explore", "stochastic", "none"])
def test_team_policy_reward_matches_fp32_engine(mode, ln):
    """The run.sh recipe's shape on the small-K team kernel (rollout_team.hip: reward-head and
    delta-head waves, fused policy, 8 workgroups per 16-candidate column, one exchange per step)
    against the fp32 group kernel on the same draws: K = 400 (train_mpc_ppo.py:71), hidden 500;
    ln=True is the recipe as run.sh:31 runs it (LAYER_NORM defaults to True, train_mpc_ppo.py:52:
    the trunk and both heads LayerNorm'd, dynamics.py:165-177)."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    from oracle import mpc_oracle as orc
    S, A, K, H, h = 20, 6, 400, 12, 500
    norm = orc.synthetic_normalization(S, A, seed=5, reward=True)
    w = orc.synthetic_reward_weights(S, A, h, ln, seed_base=123)
    p = orc.synthetic_policy(S, A, 128, 2, seed=9)
    state = orc.synthetic_state(norm, seed=6)
    expl = np.random.RandomState(4).uniform(-1, 1, (H, K, A))
    out = {}
    for kern in ("fp32", "team"):
        kw = dict(precision="fp32") if kern == "fp32" else dict(kernel="team")
        pol = dict(policy_hidden=128, policy_layers=2, policy_mode=mode) if mode != "none" else {}
        e = RolloutEngine(S, A, h, 2, "tanh", ln, H, K, cost="reward", model="reward", **pol, **kw)
        e.set_weights(MLPSpec(w.kernels, w.biases, "tanh", w.ln_gamma, w.ln_beta, model="reward"), norm, 1)
        e.set_discount(0.99)
        if mode != "none":
            e.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), 0.5, 1)
        if kern == "team":
            assert e.info()["kernel"] == "team"
        rs = [e.get_action(state, expl if mode != "stochastic" else None, seed=13, return_costs=True)
              for _ in range(3)]
        for r in rs[1:]:                                   # repeated launches: bit-identical
            assert np.array_equal(r.costs, rs[0].costs)
        out[kern] = (rs[0], e.first_actions() if mode != "none" else None)
        e.close()
    (r32, a32), (rt, at) = out["fp32"], out["team"]
    if mode != "none":
        err = np.abs(at - a32)
        print(f"[team polrew {mode}] max|dfirst|={err.max():.3e}")
        assert (err <= 2e-6).all()
    assert_rewards_close(rt.costs, r32.costs, f"team polrew {mode} ln={ln}", env=envelope(ln, 2, h, H))
    assert rt.best_index == int(np.argmax(rt.costs))
