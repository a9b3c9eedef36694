"""GPU parity: libbcmpc (HIP, gfx950) against the oracle and the reference-made fixtures.

Tolerance (stated, fp32 MLP): the engine carries state, normalisation, cost
and the trajectory sum in f64 exactly as the reference does; only the f32
MLP's summation order differs (MFMA k-ordered fma chain vs BLAS sgemm), so
per-candidate costs must agree to
    |cost_gpu - cost_ref| <= ATOL + RTOL * |cost_ref|,  ATOL = 1e-4, RTOL = 1e-5
except candidates the oracle flags as near a +-10 penalty threshold
(|s5 - 0.2|, |s6|, |s7| < 1e-4 at some step), whose cost may differ by an
exact multiple of 10 plus that tolerance.  The argmin must be bit-exact
whenever the oracle's top-2 gap exceeds 2*(ATOL + RTOL*|best|) and the
winner is not near a threshold; the returned first action is then
bit-identical (it is copied from the same f64 action array).
"""
import ctypes

import numpy as np
import pytest

from conftest import ENV_PLAIN, ENV_WIDE, Golden, envelope, golden_names

pytestmark = pytest.mark.gpu

ATOL, RTOL = 1e-4, 1e-5


KERNELS = ["solo", "group4", "group8", "split1", "split2", "split4", "team"]


def team_ok(hidden, ln, n_layers, K, S=20, A=6):
    """Shapes the small-K team kernel takes (capi.cpp bcmpc_create): the 2-layer delta net, hidden <= 512
    (LayerNorm: <= 256), the whole grid resident (ceil(K/128)*8 workgroups x members <= 256 CUs)."""
    hp = next(p for p in (64, 128, 256, 512, 768, 1024) if hidden <= p)
    members = 4 if hp == 512 else 1
    blocks = -(-(-(-K // 16)) // 8) * 8 * members
    return (n_layers == 2 and hp <= 512 and not (ln and members > 1) and S + A <= 32 and 0 < K
            and blocks <= 256)


def _skip_unsupported(g: Golden, kernel: str):
    if kernel == "group8" and g.meta["hidden"] <= 64:
        pytest.skip("group8 needs >= 8 hidden tiles")
    if kernel == "solo" and g.meta["hidden"] > 512:
        pytest.skip("solo: hidden <= 512")
    if kernel == "split4" and g.meta["hidden"] > 512:
        pytest.skip("split kernel at hidden > 512: 32-candidate groups at most (the hi + lo slab, 160-KiB LDS)")
    if kernel == "team" and not team_ok(g.meta["hidden"], g.meta["ln"], g.weights.n_layers, g.K, g.S, g.A):
        pytest.skip("team: the 2-layer delta net at small K (grid resident)")
    if kernel.startswith("split"):
        if (g.meta["act"] != "tanh" or g.meta["ln"]) and g.meta["hidden"] > 512:
            pytest.skip("split precision: relu / LayerNorm nets up to hidden 512")
        if kernel == "split4" and g.meta["hidden"] <= 64:
            pytest.skip("split4 needs >= 4 waves (hidden > 64)")


def _engine(g: Golden, K=None, H=None, cost="cheetah", kernel="auto"):
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    w = g.weights
    eng = RolloutEngine(g.S, g.A, w.hidden, w.n_layers, w.activation, w.layer_norm,
                        H or g.H, K if K is not None else g.K, device=0, cost=cost, kernel=kernel)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), g.norm, version=1)
    return eng


# multiples of a fixture's conditioning (its rounding spread, conftest.Golden.cond) added to the tolerance: the
# kernels' deviation on the relu + LayerNorm H = 20 fixture reaches 4.3x it at worst (the f32 solo kernel's
# sequential k chains; group4 2.2x, split4 2.3x, team 2.9x: profiles/r06_cond_ratios.txt)
COND_K = 6.0


def assert_costs_close(got, want, near=None, label="", env=ENV_PLAIN, cond=None):
    """The stated tolerance AND the achieved envelope ``env`` (conftest.envelope), except exact +-10
    flips of near-threshold candidates.  ``cond`` (fixtures that hold it): per candidate, the spread between
    the reference's f32 costs and the same net in f64 arithmetic -- where the dynamics amplify rounding
    that much, no other rounding order can be held closer, so COND_K times it widens that candidate's bar."""
    assert got.shape == want.shape
    nan_g, nan_w = np.isnan(got), np.isnan(want)
    assert np.array_equal(nan_g, nan_w), f"{label}: NaN pattern differs"
    ok = ~nan_w
    diff = np.abs(got[ok] - want[ok])
    tol = np.minimum(ATOL + RTOL * np.abs(want[ok]), env)
    if cond is not None:
        tol = tol + COND_K * cond[ok]
    bad = diff > tol
    if near is not None:
        nr = near[ok]
        flip = np.abs(diff - 10.0 * np.round(diff / 10.0)) <= tol
        bad &= ~(nr & flip)
    print(f"[{label}] max|dcost|={diff.max() if diff.size else 0:.3e} "
          f"n={ok.sum()} over_tol={int(bad.sum())}")
    assert not bad.any(), f"{label}: {int(bad.sum())} costs outside tolerance; worst {diff.max():.3e}"


def argmin_is_decidable(g: Golden) -> bool:
    best = g.costs[g.argmin]
    if np.isnan(best):
        return True
    return g.top2_gap > 2 * (ATOL + RTOL * abs(best) + COND_K * float(np.max(g.cond))) and not g.near[g.argmin]


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", golden_names("mpc"))
def test_engine_matches_reference_fixture(name, kernel):
    g = Golden(name)
    _skip_unsupported(g, kernel)
    eng = _engine(g, kernel=kernel)
    assert eng.info()["kernel"] == kernel
    if g.meta.get("inject") == "philox":
        res = eng.get_action(g.state, None, seed=g.meta["rng_seed"], cand_offset=g.meta["cand_offset"],
                             return_costs=True)
        offset = g.meta["cand_offset"]
    else:
        res = eng.get_action(g.state, g.actions(), return_costs=True)
        offset = 0
    assert_costs_close(res.costs, g.costs, g.near, f"{name}/{kernel}",
                       env=envelope(g.meta["ln"], g.weights.n_layers, g.meta["hidden"], g.H), cond=g.cond)
    assert res.best_index - offset == int(np.argmin(res.costs))
    if argmin_is_decidable(g):
        assert res.best_index - offset == g.argmin
        assert np.array_equal(res.first_action, g.opt_action)
        if not np.isnan(g.costs[g.argmin]):
            assert res.best_cost == res.costs[g.argmin]
    eng.close()


@pytest.mark.parametrize("name", ["tiny_tanh", "small_relu", "cfg1_2x500_tanh", "ppo_defaults_2x256_relu_ln"])
def test_mpccontroller_dropin_bitexact(name):
    """The drop-in class: same constructor/get_action signature, same RNG side
    effect, bit-identical float64 action (controllers.py:57-88)."""
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    g = Golden(name)

    class Box:
        low, high = g.low, g.high
        shape = (g.A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (g.S,)

    ctrl = MPCcontroller(env=Env(), dyn_model=g.dyn(), horizon=g.H, cost_fn=cheetah_cost_fn,
                         num_simulated_paths=g.K)
    np.random.seed(g.meta["seed"])
    a = ctrl.get_action(g.state)
    assert isinstance(a, np.ndarray) and a.dtype == np.float64 and a.shape == (g.A,)
    if argmin_is_decidable(g):
        assert np.array_equal(a, g.opt_action)
    assert np.random.random() == float(g.z["next_draw"])


@pytest.mark.parametrize("kernel", KERNELS)
@pytest.mark.parametrize("name", ["tiny_tanh", "small_relu", "small_ln_relu", "deep3_tanh", "one_layer_tanh",
                                  "nan_candidates", "ragged_k1", "ragged_k17_h1"])
def test_trajectory_states_match(name, kernel):
    """states_paths_all (controllers.py:65-74) from the kernel vs the reference's."""
    import torch
    g = Golden(name)
    if "states" not in g.z.files:
        pytest.skip("fixture holds no states")
    _skip_unsupported(g, kernel)
    eng = _engine(g, cost="none", kernel=kernel)
    dev = torch.device("cuda", 0)
    st = torch.from_numpy(g.state).to(dev)
    act = torch.from_numpy(np.ascontiguousarray(g.actions())).to(dev)
    traj = torch.full((g.H + 1, g.K, g.S), np.nan, dtype=torch.float64, device=dev)
    eng.rollout_async(st.data_ptr(), 0, act.data_ptr(), 0, 0, None, traj.data_ptr(), None,
                      torch.cuda.current_stream(dev).cuda_stream)
    got = traj.cpu().numpy()
    want = g.z["states"]
    assert np.array_equal(np.isnan(got), np.isnan(want))
    ok = ~np.isnan(want)
    err = np.abs(got[ok] - want[ok])
    print(f"[{name}] max|dstate|={err.max():.3e}")
    assert np.array_equal(got[0], want[0])               # tiled initial state is exact
    assert (err <= 1e-6 + 1e-6 * np.abs(want[ok])).all()
    eng.close()


def test_predict_per_candidate_states():
    """NNDynamicsModel.predict (dynamics.py:106-119) on [K, S] states via the kernel."""
    import torch
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    w = orc.synthetic_weights(20, 6, 256, 2, "relu", True)
    norm = orc.synthetic_normalization()
    rs = np.random.RandomState(0)
    K = 300
    s = norm[0] + norm[1] * rs.standard_normal((K, 20))
    a = rs.uniform(-1, 1, (K, 6))
    want = orc.NumpyDynamics(w, norm).predict(s, a)
    eng = RolloutEngine(20, 6, 256, 2, "relu", True, 1, K, cost="none")
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), norm, 1)
    dev = torch.device("cuda", 0)
    ds, da = torch.from_numpy(s).to(dev), torch.from_numpy(a).to(dev)
    traj = torch.empty((2, K, 20), dtype=torch.float64, device=dev)
    eng.rollout_async(ds.data_ptr(), 20, da.data_ptr(), 0, 0, None, traj.data_ptr(), None,
                      torch.cuda.current_stream(dev).cuda_stream)
    got = traj.cpu().numpy()
    assert np.array_equal(got[0], s)
    err = np.abs(got[1] - want)
    print(f"max|dpredict|={err.max():.3e}")
    assert (err <= 1e-6 + 1e-6 * np.abs(want)).all()


def test_non_fused_cost_goes_through_trajectory_mode():
    from bc_mpc_amd import MPCcontroller
    from oracle import mpc_oracle as orc
    g = Golden("small_relu")

    def my_cost(state, action, next_state):     # not the cheetah cost -> host scoring of GPU states
        return -(next_state[:, 0] - state[:, 0]) + 0.1 * np.sum(action ** 2, axis=1)

    class Box:
        low, high = g.low, g.high
        shape = (g.A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (g.S,)

    ctrl = MPCcontroller(Env(), g.dyn(), horizon=g.H, cost_fn=my_cost, num_simulated_paths=g.K)
    np.random.seed(123)
    a = ctrl.get_action(g.state)
    np.random.seed(123)
    want, i, costs = orc.get_action(g.dyn(), g.state, g.H, g.K, g.low, g.high, cost_fn=my_cost)
    assert_costs_close(ctrl.last_costs, costs, label="traj-mode")
    assert ctrl.last_index == i and np.array_equal(a, want)


@pytest.mark.parametrize("kernel", ["splitr", "group2"])
def test_retired_kernels_are_refused(kernel):
    """The resident-column kernel (rollout_rr.hip, opt-in only, slower than the slab kernel at every K: DESIGN.md
    6.5) and the 2-wave f32 group layout (A/B only, never chosen by auto) were retired in round 6: asking for
    either fails loudly instead of running another layout."""
    from bc_mpc_amd.engine import RolloutEngine
    with pytest.raises(ValueError, match="retired"):
        RolloutEngine(20, 6, 500, 2, "tanh", False, 20, 4096, kernel=kernel)


@pytest.mark.parametrize("kernel", ["auto", "solo", "group8", "split4", "split1"])
def test_full_size_cfg3_properties(kernel):
    """K=65536, H=20, 2x500 tanh (BASELINE cfg3 dims) at full size: shard
    invariance (bitwise), argmin consistency, determinism, and a 256-candidate
    oracle sample within tolerance -- device-RNG and host-action modes."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    K, H = 65536, 20
    w = orc.synthetic_weights(20, 6, 500, 2, "tanh", False)
    norm = orc.synthetic_normalization()
    state = orc.synthetic_state(norm)
    spec = MLPSpec(w.kernels, w.biases, w.activation)

    def mk(k):
        e = RolloutEngine(20, 6, 500, 2, "tanh", False, H, k, kernel=kernel)
        e.set_weights(spec, norm, 1)
        return e

    full = mk(K)
    seed = 0xC0FFEE
    r1 = full.get_action(state, None, seed=seed, return_costs=True)
    r2 = full.get_action(state, None, seed=seed, return_costs=True)
    assert np.array_equal(r1.costs, r2.costs) and r1.best_index == r2.best_index    # deterministic
    assert r1.best_index == int(np.argmin(r1.costs)) and r1.best_cost == r1.costs[r1.best_index]
    half = mk(K // 2)
    a = half.get_action(state, None, seed=seed, cand_offset=0, return_costs=True)
    b = half.get_action(state, None, seed=seed, cand_offset=K // 2, return_costs=True)
    assert np.array_equal(np.concatenate([a.costs, b.costs]), r1.costs)            # shard invariance
    # oracle sample: 256 candidates incl. the winner
    rs = np.random.RandomState(1)
    idx = np.unique(np.concatenate([rs.choice(K, 255, replace=False), [r1.best_index]]))
    acts = orc.device_rng_actions(seed, 0, K, H, -np.ones(6), np.ones(6))[:, idx, :]
    want, states = orc.rollout(orc.NumpyDynamics(w, norm), state, acts)
    assert_costs_close(r1.costs[idx], want, orc.near_threshold_mask(states), "cfg3-sample")
    assert np.array_equal(r1.first_action, acts[0, np.searchsorted(idx, r1.best_index)])
    # host-action mode on the same sampled actions reproduces the same costs bitwise
    host = np.random.RandomState(2).uniform(-1, 1, (H, K, 6))
    host[:, idx, :] = orc.device_rng_actions(seed, 0, K, H, -np.ones(6), np.ones(6))[:, idx, :]
    r3 = full.get_action(state, host, return_costs=True)
    assert np.array_equal(r3.costs[idx], r1.costs[idx])
    for e in (full, half):
        e.close()


def test_errors_are_python_exceptions():
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    e = RolloutEngine(20, 6, 64, 2, "tanh", False, 3, 0)
    w = orc.synthetic_weights(20, 6, 64, 2)
    e.set_weights(MLPSpec(w.kernels, w.biases), orc.synthetic_normalization(), 1)
    with pytest.raises(ValueError):                 # np.argmin of an empty sequence
        e.get_action(np.zeros(20))
    e2 = RolloutEngine(20, 6, 64, 2, "tanh", False, 3, 16)
    with pytest.raises(RuntimeError):               # rollout before set_weights
        e2.get_action(np.zeros(20))
    with pytest.raises(ValueError):
        e2.set_weights(MLPSpec(w.kernels[:2], w.biases[:2]), orc.synthetic_normalization(), 1)


@pytest.mark.parametrize("kernel", ["auto", "group4", "group8", "split1", "split2"])
@pytest.mark.parametrize("hidden,L,act,ln", [(1024, 3, "tanh", False), (768, 2, "tanh", False),
                                             (1000, 3, "relu", True), (600, 2, "tanh", False)])
def test_large_hidden_vs_oracle(hidden, L, act, ln, kernel):
    """cfg5-class networks (3x1024) and odd widths on the group kernels."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    if kernel.startswith("split") and (act != "tanh" or ln):
        pytest.skip("split precision: relu / LayerNorm nets up to hidden 512")
    K, H = 96, 4
    w = orc.synthetic_weights(20, 6, hidden, L, act, ln, seed_base=77)
    norm = orc.synthetic_normalization()
    state = orc.synthetic_state(norm)
    acts = np.random.RandomState(5).uniform(-1, 1, (H, K, 6))
    eng = RolloutEngine(20, 6, hidden, L, act, ln, H, K, kernel=kernel)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), norm, 1)
    res = eng.get_action(state, acts, return_costs=True)
    want, states = orc.rollout(orc.NumpyDynamics(w, norm), state, acts)
    assert_costs_close(res.costs, want, orc.near_threshold_mask(states), f"h{hidden}xL{L}/{kernel}",
                       env=envelope(ln, L, hidden, H))
    assert res.best_index == int(np.argmin(res.costs))


def _policy_env(g):
    class Box:
        low, high = g.low, g.high
        shape = (g.A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (g.S,)
    return Env()


def _split_policy_ok(hidden, act, ln):
    return act == "tanh" and not ln and 448 < hidden <= 1024


def team_policy_ok(hidden, act, ln, K, ph, pl):
    """Shapes the team kernel takes with a fused policy (capi.cpp bcmpc_create): <= 2 x 128 policy; dynamics
    hidden 65..256 with any activation / LayerNorm (one workgroup per column: ceil(K/128)*8 <= 256 CUs) or
    449..512 tanh without LayerNorm (4 members per column)."""
    if ph > 128 or pl > 2 or K < 1:
        return False
    blocks = -(-(-(-K // 16)) // 8) * 8
    if 64 < hidden <= 256:
        return blocks <= 256
    return 448 < hidden <= 512 and act == "tanh" and not ln and 4 * blocks <= 256


@pytest.mark.parametrize("kernel", ["fp32", "split1", "split2", "split4", "team"])
@pytest.mark.parametrize("name", golden_names("policy"))
def test_policy_engine_matches_reference_fixture(name, kernel):
    """MPCcontrollerPolicyNet (self_exp=False) fused into the group kernel (fp32) or the split
    kernel (policy MLP in split-f16 too) vs the reference run; same tolerances."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    g = Golden(name)
    w, p = g.weights, g.policy
    if kernel.startswith("split") and not _split_policy_ok(w.hidden, w.activation, w.layer_norm):
        pytest.skip("split kernel with a policy: tanh dynamics without LayerNorm, hidden 449..1024")
    if kernel == "team" and not team_policy_ok(w.hidden, w.activation, w.layer_norm, g.K, p.hidden, p.n_layers):
        pytest.skip("team kernel with a policy: hidden 65..256 (any net) or 449..512 tanh, policy <= 2 x 128, small K")
    kw = dict(precision="fp32") if kernel == "fp32" else dict(kernel=kernel)
    eng = RolloutEngine(g.S, g.A, w.hidden, w.n_layers, w.activation, w.layer_norm, g.H, g.K,
                        policy_hidden=p.hidden, policy_layers=p.n_layers, policy_mode="explore", **kw)
    if kernel != "fp32":
        assert eng.info()["kernel"] == kernel
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), g.norm, 1)
    eng.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), g.meta["explore"], 1)
    rs = np.random.RandomState(g.meta["seed"])
    expl = rs.uniform(g.low, g.high, size=[g.H, g.K, g.A])
    res = eng.get_action(g.state, expl, return_costs=True)
    assert_costs_close(res.costs, g.costs, g.near, f"{name}/{kernel}",
                       env=envelope(w.layer_norm, w.n_layers, w.hidden, g.H))
    fa = eng.first_actions()
    err = np.abs(fa - g.z["first_actions"])
    print(f"[{name}] max|dfirst_action|={err.max():.3e}")
    assert (err <= 1e-6).all()
    assert res.best_index == int(np.argmin(res.costs))
    if argmin_is_decidable(g):
        assert res.best_index == g.argmin
        assert np.allclose(res.first_action, g.opt_action, rtol=0, atol=1e-6)


@pytest.mark.parametrize("name", golden_names("policy"))
def test_policy_controller_dropin(name):
    from bc_mpc_amd import MPCcontrollerPolicyNet, cheetah_cost_fn
    from oracle import mpc_oracle as orc
    g = Golden(name)
    ctrl = MPCcontrollerPolicyNet(_policy_env(g), g.dyn(), orc.NumpyPolicy(g.policy), explore=g.meta["explore"],
                                  self_exp=False, horizon=g.H, cost_fn=cheetah_cost_fn, num_simulated_paths=g.K)
    np.random.seed(g.meta["seed"])
    a = ctrl.get_action(g.state)
    assert a.dtype == np.float64 and a.shape == (g.A,)
    if argmin_is_decidable(g):
        assert np.allclose(a, g.opt_action, rtol=0, atol=1e-6)
    assert np.random.random() == float(g.z["next_draw"])        # same RNG side effect as the reference


@pytest.mark.parametrize("kernel", ["fp32", "split2", "team", "team_relu_ln"])
def test_policy_stochastic_mode_pinned_every_step(kernel):
    """self_exp=True (run.sh's recipe, controllers.py:202-203): at EVERY horizon step the action the
    kernel rolled out equals mean(s_h) + exp(logstd) * z_h, where s_h is the GPU's own trajectory
    state, mean the oracle's policy MLP (ppo_bc_policy.py:64-80) and z_h the oracle's restatement of
    the device Philox normals (oracle.device_rng_normals) -- within the f32 tolerance (the kernel
    evaluates mean, exp and Box-Muller in f32); and s_{h+1} = predict(s_h, a_h) (dynamics.py:106-119).
    Then the same call is deterministic and shard-invariant."""
    import torch
    from bc_mpc_amd import _lib
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    from oracle import mpc_oracle as orc
    K, H, S, A, seed = 512, 8, 20, 6, 42
    if kernel == "fp32":
        w = orc.synthetic_weights(S, A, 256, 2, "relu", False)
        kw = dict(precision="fp32")
    elif kernel == "team_relu_ln":      # train_mpc_ppo.py's own dynamics net (:52, :74-75, :539)
        w = orc.synthetic_weights(S, A, 256, 2, "relu", True)
        kw = dict(kernel="team")
    else:
        w = orc.synthetic_weights(S, A, 500, 2, "tanh", False)
        kw = dict(kernel=kernel)
    p = orc.synthetic_policy(S, A, 128, 2)
    norm = orc.synthetic_normalization()
    state = orc.synthetic_state(norm)
    dyn, pol = orc.NumpyDynamics(w, norm), orc.NumpyPolicy(p)

    def mk(k):
        e = RolloutEngine(S, A, w.hidden, 2, w.activation, w.layer_norm, H, k, policy_hidden=128,
                          policy_layers=2, policy_mode="stochastic", **kw)
        e.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), norm, 1)
        e.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), 0.5, 1)
        return e
    full = mk(K)
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)
    d_state = torch.from_numpy(state).to(dev)
    d_traj, d_out = torch.empty((H + 1, K, S), **f64), torch.empty((H, K, A), **f64)
    d_costs = torch.empty(K, **f64)
    d_res = torch.zeros(ctypes.sizeof(_lib.Result), dtype=torch.uint8, device=dev)
    full.rollout_policy_async(d_state.data_ptr(), None, seed, 0, d_costs.data_ptr(), d_traj.data_ptr(),
                              d_out.data_ptr(), d_res.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
    traj, acts, costs = d_traj.cpu().numpy(), d_out.cpu().numpy(), d_costs.cpu().numpy()
    sd = np.exp(p.logstd.astype(np.float64))
    worst_a = worst_s = 0.0
    for h in range(H):
        mean = pol.mean(traj[h]).astype(np.float64)
        want = mean + sd * orc.device_rng_normals(seed, 0, K, h, A)
        da = np.abs(acts[h] - want)
        assert (da <= 1e-5 + 1e-5 * np.abs(want)).all(), f"step {h}: action off by {da.max():.3e}"
        nxt = dyn.predict(traj[h], acts[h])
        ds = np.abs(traj[h + 1] - nxt)
        assert (ds <= 1e-6 * (1 + np.abs(nxt))).all(), f"step {h}: state off by {ds.max():.3e}"
        worst_a, worst_s = max(worst_a, da.max()), max(worst_s, ds.max())
    print(f"[stochastic policy {kernel}] max|da|={worst_a:.2e} max|ds|={worst_s:.2e}")
    raw = d_res.cpu().numpy()
    best = int(raw[:8].view(np.int64)[0])
    assert best == int(np.argmin(costs)) and np.array_equal(raw[16:16 + 8 * A].view(np.float64), acts[0, best])
    # the synchronous call: the same normals -> bit-identical costs; halves concatenate to the whole
    r1 = full.get_action(state, None, seed=seed, return_costs=True)
    assert np.array_equal(r1.costs, costs)
    half = mk(K // 2)
    ra = half.get_action(state, None, seed=seed, cand_offset=0, return_costs=True)
    rb = half.get_action(state, None, seed=seed, cand_offset=K // 2, return_costs=True)
    assert np.array_equal(np.concatenate([ra.costs, rb.costs]), costs)
    full.close(), half.close()


@pytest.mark.parametrize("mode", ["explore", "stochastic"])
@pytest.mark.parametrize("hidden,PL,ph", [(500, 2, 128), (1000, 2, 64), (512, 1, 100)])
def test_split_policy_matches_fp32_engine(hidden, PL, ph, mode):
    """The split kernel's fused policy against the fp32 group/solo kernel at scale: same f64
    explore draws / Philox normals, costs and step-0 actions within the f32 tolerance
    (the two engines differ only in the f32 summation order / split rounding)."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    from oracle import mpc_oracle as orc
    K, H = 3000, 8
    w = orc.synthetic_weights(20, 6, hidden, 2, "tanh", False, seed_base=77)
    p = orc.synthetic_policy(20, 6, ph, PL, seed=5)
    norm = orc.synthetic_normalization()
    state = orc.synthetic_state(norm)
    expl = np.random.RandomState(3).uniform(-1, 1, (H, K, 6))
    out = {}
    if hidden > 512:                     # the fp32 kernels fuse a policy up to hidden 512: the oracle
        if mode == "stochastic":
            pytest.skip("device Philox normals: no host restatement beyond the fp32 engine")
        dyn, pol = orc.NumpyDynamics(w, norm), orc.NumpyPolicy(p)
        a0, i0, c0 = orc.policy_get_action(dyn, pol, state, H, K, -np.ones(6), np.ones(6), 0.3,
                                           rng=np.random.RandomState(3))
        e = RolloutEngine(20, 6, hidden, 2, "tanh", False, H, K, policy_hidden=ph, policy_layers=PL,
                          policy_mode=mode, precision="split")
        e.set_weights(MLPSpec(w.kernels, w.biases, "tanh"), norm, 1)
        e.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), 0.3, 1)
        r = e.get_action(state, expl, return_costs=True)
        first = (1 - 0.3) * pol.act(np.tile(state, [K, 1]), stochastic=False)[0] + 0.3 * expl[0]
        err = np.abs(e.first_actions() - first)
        print(f"[split policy {hidden}/{PL}x{ph} vs oracle] max|dfirst|={err.max():.3e}")
        assert (err <= 2e-6).all()
        d = np.abs(r.costs - c0)
        tol = 10 * (ATOL + RTOL * np.abs(c0))
        flip = np.abs(d - 10.0 * np.round(d / 10.0)) <= tol
        print(f"   max|dcost|={d.max():.3e} over_tol={(d > tol).sum()} flips={(flip & (d > tol)).sum()}")
        assert ((d <= tol) | flip).all() and (flip & (d > tol)).sum() <= K // 500
        e.close()
        return
    for prec in ("fp32", "split"):
        e = RolloutEngine(20, 6, hidden, 2, "tanh", False, H, K, policy_hidden=ph, policy_layers=PL,
                          policy_mode=mode, precision=prec)
        e.set_weights(MLPSpec(w.kernels, w.biases, "tanh"), norm, 1)
        e.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), 0.3, 1)
        if prec == "split":
            assert e.info()["kernel"].startswith("split")
        r = e.get_action(state, expl, seed=9, return_costs=True)
        out[prec] = (r, e.first_actions())
        e.close()
    (r32, a32), (rsp, asp) = out["fp32"], out["split"]
    err = np.abs(asp - a32)
    print(f"[split policy {hidden}/{PL}x{ph} {mode}] max|dfirst|={err.max():.3e}")
    assert (err <= 2e-6).all()
    d = np.abs(rsp.costs - r32.costs)
    tol = 10 * (ATOL + RTOL * np.abs(r32.costs))
    flip = np.abs(d - 10.0 * np.round(d / 10.0)) <= tol          # a +-10 penalty threshold crossed
    print(f"   max|dcost|={d.max():.3e} over_tol={(d > tol).sum()} flips={(flip & (d > tol)).sum()}")
    assert ((d <= tol) | flip).all() and (flip & (d > tol)).sum() <= K // 500
    assert rsp.best_index == int(np.argmin(rsp.costs))


def test_split_policy_shard_invariant():
    """Candidate sharding (cand_offset) leaves the split kernel's stochastic policy bit-identical."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    from oracle import mpc_oracle as orc
    K, H = 2048, 5
    w = orc.synthetic_weights(20, 6, 500, 2, "tanh", False)
    p = orc.synthetic_policy(20, 6, 128, 2)
    norm = orc.synthetic_normalization()
    state = orc.synthetic_state(norm)

    def mk(k):
        e = RolloutEngine(20, 6, 500, 2, "tanh", False, H, k, policy_hidden=128, policy_layers=2,
                          policy_mode="stochastic", kernel="split2")
        e.set_weights(MLPSpec(w.kernels, w.biases, "tanh"), norm, 1)
        e.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), 0.5, 1)
        return e
    full = mk(K)
    r1 = full.get_action(state, None, seed=42, return_costs=True)
    r2 = full.get_action(state, None, seed=42, return_costs=True)
    assert np.array_equal(r1.costs, r2.costs)
    half = mk(K // 2)
    ra = half.get_action(state, None, seed=42, cand_offset=0, return_costs=True)
    rb = half.get_action(state, None, seed=42, cand_offset=K // 2, return_costs=True)
    assert np.array_equal(np.concatenate([ra.costs, rb.costs]), r1.costs)


@pytest.mark.parametrize("model", ["delta", "policy", "reward"])
def test_fused_argmin_tail_matches_launches(model, monkeypatch):
    """BCMPC_FUSED_ARGMIN=1 (the split kernel reduces np.argmin in its own tail) returns exactly
    what the two argmin launches return: index, cost, first action (policy: the mixed action)."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    from oracle import mpc_oracle as orc
    K, H = 5000, 6
    rew = model == "reward"
    norm = orc.synthetic_normalization(20, 6, seed=5, reward=rew)
    w = orc.synthetic_reward_weights(20, 6, 500, False, seed_base=9) if rew else orc.synthetic_weights(20, 6, 500, 2)
    state = orc.synthetic_state(norm, seed=6)
    expl = np.random.RandomState(8).uniform(-1, 1, (H, K, 6))
    out = []
    for fused in ("0", "1"):
        monkeypatch.setenv("BCMPC_FUSED_ARGMIN", fused)
        kw = dict(cost="reward", model="reward") if rew else {}
        if model == "policy":
            kw.update(policy_hidden=128, policy_layers=2)
        e = RolloutEngine(20, 6, 500, 2, "tanh", False, H, K, precision="split", **kw)
        e.set_weights(MLPSpec(w.kernels, w.biases, "tanh", model="reward" if rew else "delta"), norm, 1)
        if rew:
            e.set_discount(0.99)
        if model == "policy":
            p = orc.synthetic_policy(20, 6, 128, 2)
            e.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), 0.5, 1)
        r1 = e.get_action(state, expl, return_costs=True)
        r2 = e.get_action(state, None, seed=77, cand_offset=123, return_costs=True)   # device RNG, offset
        out.append((r1, r2))
        e.close()
    for a, b in zip(out[0], out[1]):
        assert a.best_index == b.best_index and a.best_cost == b.best_cost
        assert np.array_equal(a.first_action, b.first_action) and np.array_equal(a.costs, b.costs)


def test_dropin_numpy_stream_path_equals_host_array_path():
    """MPCcontroller draws the reference's [H, K, A] array with the library's MT19937 restatement
    straight into pinned memory; a subclass that overrides sample_random_actions takes the host-
    array path.  Same costs, same action, same global-stream position afterwards."""
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    g = Golden("cfg2_2x500_tanh")

    class Box:
        low, high = g.low, g.high
        shape = (g.A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (g.S,)

    class Slow(MPCcontroller):
        def sample_random_actions(self):
            return super().sample_random_actions()

    out = []
    for cls in (MPCcontroller, Slow):
        ctrl = cls(env=Env(), dyn_model=g.dyn(), horizon=g.H, cost_fn=cheetah_cost_fn, num_simulated_paths=g.K)
        ctrl.keep_costs = True
        np.random.seed(g.meta["seed"])
        a = ctrl.get_action(g.state)
        out.append((a, ctrl.last_costs.copy(), np.random.random()))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert out[0][2] == out[1][2] == float(g.z["next_draw"])
    assert_costs_close(out[0][1], g.costs, g.near, "numpy-stream path")


@pytest.mark.parametrize("pre_draws", [0, 1, 313])
def test_dropin_threaded_numpy_stream_equals_host_array_path(pre_draws):
    """Large draws split over host threads by MT19937 jump-ahead (csrc/mt_jump.cpp), each thread
    uploading its own slice: the same costs, action and global-stream position as the host-array
    path (NumPy's own draw) at K = 65536, H = 6 (4.7M generator words: 4 threads)."""
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    g = Golden("cfg2_2x500_tanh")

    class Box:
        low, high = g.low, g.high
        shape = (g.A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (g.S,)

    class Slow(MPCcontroller):
        def sample_random_actions(self):
            return super().sample_random_actions()

    out = []
    for cls in (MPCcontroller, Slow):
        ctrl = cls(env=Env(), dyn_model=g.dyn(), horizon=6, cost_fn=cheetah_cost_fn, num_simulated_paths=65536)
        ctrl.keep_costs = True
        np.random.seed(99)
        np.random.random(pre_draws)
        a = ctrl.get_action(g.state)
        out.append((a, ctrl.last_costs.copy(), np.random.get_state()))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    assert np.array_equal(out[0][2][1], out[1][2][1]) and out[0][2][2] == out[1][2][2]


def test_numpy_stream_shards_equal_whole_draw():
    """Multi-GPU parity mode on one card: two engines own the halves of K_global = 65536 (H = 6) and each
    draws only its own rows of every step (jump-ahead over the other half, csrc/mt_jump.cpp).  Their cost
    vectors concatenate to the single engine's, and every engine leaves the global stream where NumPy's
    one draw leaves it."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    S, A, H, KG = 20, 6, 6, 65536
    w = orc.synthetic_weights(S, A, 128, 2, "tanh", False)
    norm = orc.synthetic_normalization(S, A)
    state = orc.synthetic_state(norm)
    low, high = -np.ones(A), np.ones(A)
    np.random.seed(2024)
    np.random.random(3)
    st0 = np.random.get_state()
    np.random.uniform(low, high, [H, KG, A])
    st_want = np.random.get_state()
    costs, states = [], []
    for off, k in ((0, KG), (0, KG // 2), (KG // 2, KG // 2)):
        eng = RolloutEngine(S, A, 128, 2, "tanh", False, H, k, device=0)
        eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, 1)
        np.random.set_state(st0)
        res = eng.get_action_numpy_stream(state, low, high, KG, cand_offset=off, return_costs=True)
        costs.append(res.costs.copy())
        states.append(np.random.get_state())
        eng.close()
    assert np.array_equal(np.concatenate(costs[1:]), costs[0])
    for st in states:
        assert np.array_equal(st[1], st_want[1]) and st[2] == st_want[2]


def test_dropin_repeat_fast_path_tracks_changes():
    """MPCcontroller.get_action's repeat-call fast path (controllers.py fast path: the checks of the last
    call reused): consecutive calls, a weight reload (version bump), a replaced normalisation object and a
    changed horizon each return exactly what a fresh controller returns from the same NumPy state, and
    leave NumPy's stream where it leaves it."""
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    from bc_mpc_amd.dynamics import NNDynamicsModel
    from oracle import mpc_oracle as orc
    S, A, K, H = 20, 6, 400, 7

    class Box:
        low, high = -np.ones(A), np.ones(A)
        shape = (A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (S,)

    norm = orc.synthetic_normalization(S, A)
    w = orc.synthetic_weights(S, A, 256, 2, "relu", True)
    w2 = orc.synthetic_weights(S, A, 256, 2, "relu", True, seed_base=5)

    def model(wt):
        m = NNDynamicsModel(Env(), 2, 256, "relu", None, list(norm), 512, 1, 1e-3, layer_norm=True, device=0)
        m.load_weights(wt.kernels, wt.biases, wt.ln_gamma, wt.ln_beta)
        return m

    state = orc.synthetic_state(norm)
    dm = model(w)
    ctrl = MPCcontroller(Env(), dm, horizon=H, cost_fn=cheetah_cost_fn, num_simulated_paths=K)

    def fresh(wt, h, nrm=None):
        m = model(wt)
        if nrm is not None:
            m.std_obs = nrm
        return MPCcontroller(Env(), m, horizon=h, cost_fn=cheetah_cost_fn, num_simulated_paths=K)

    def same(step, ref_ctrl):
        st = np.random.get_state()
        want = ref_ctrl.get_action(state)
        want_next = np.random.get_state()
        np.random.set_state(st)
        got = ctrl.get_action(state)
        got_next = np.random.get_state()
        assert np.array_equal(got, want), step
        assert np.array_equal(got_next[1], want_next[1]) and got_next[2] == want_next[2], step
        ref_ctrl._engine.close()

    np.random.seed(11)
    for i in range(3):
        same(f"repeat {i}", fresh(w, H))
    assert ctrl._fast is not None                      # the repeat path is the one under test
    dm.load_weights(w2.kernels, w2.biases, w2.ln_gamma, w2.ln_beta)
    same("weights reloaded", fresh(w2, H))
    dm.std_obs = np.asarray(norm[1]) * 1.5
    same("normalisation replaced", fresh(w2, H, dm.std_obs))
    ctrl.horizon = 5
    same("horizon changed", fresh(w2, 5, dm.std_obs))
    ctrl._engine.close()


def test_policy_dropin_repeat_fast_path_tracks_changes():
    """MPCcontrollerPolicyNet's repeat-call fast path (train_mpc_ppo's default MPC-aug controller: explore 0.5
    over the 2x256 relu + LN net): repeated calls, a new policy (integer version bumped), a changed explore
    and a reloaded dynamics net each return exactly what a fresh controller returns from the same NumPy state
    (and the same private seed stream), and leave NumPy's stream where it leaves it."""
    from bc_mpc_amd import MPCcontrollerPolicyNet, cheetah_cost_fn
    from bc_mpc_amd.dynamics import NNDynamicsModel
    from bc_mpc_amd.engine import PolicySpec
    from oracle import mpc_oracle as orc
    S, A, K, H = 20, 6, 400, 7

    class Box:
        low, high = -np.ones(A), np.ones(A)
        shape = (A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (S,)

    class Pol:                                          # a versioned policy container (policy.extract)
        def __init__(self, p, version):
            self._spec = PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd)
            self.version = version

        def policy_spec(self):
            return self._spec

    norm = orc.synthetic_normalization(S, A)
    w, w2 = orc.synthetic_weights(S, A, 256, 2, "relu", True), orc.synthetic_weights(S, A, 256, 2, "relu", True, seed_base=9)
    p1, p2 = orc.synthetic_policy(S, A), orc.synthetic_policy(S, A, seed=77)

    def model(wt):
        m = NNDynamicsModel(Env(), 2, 256, "relu", None, list(norm), 512, 1, 1e-3, layer_norm=True, device=0)
        m.load_weights(wt.kernels, wt.biases, wt.ln_gamma, wt.ln_beta)
        return m

    state = orc.synthetic_state(norm)
    dm, pol = model(w), Pol(p1, 1)
    ctrl = MPCcontrollerPolicyNet(Env(), dm, pol, explore=0.5, self_exp=False, horizon=H, cost_fn=cheetah_cost_fn,
                                  num_simulated_paths=K, seed=3)

    def same(step, wt, pp, explore):
        ref = MPCcontrollerPolicyNet(Env(), model(wt), Pol(pp, 1), explore=explore, self_exp=False, horizon=H,
                                     cost_fn=cheetah_cost_fn, num_simulated_paths=K, seed=3)
        ref._seed_rng.set_state(ctrl._seed_rng.get_state())
        st = np.random.get_state()
        want = ref.get_action(state)
        want_next = np.random.get_state()
        np.random.set_state(st)
        got = ctrl.get_action(state)
        got_next = np.random.get_state()
        assert np.array_equal(got, want), step
        assert np.array_equal(got_next[1], want_next[1]) and got_next[2] == want_next[2], step
        ref._engine.close()

    np.random.seed(5)
    for i in range(3):
        same(f"repeat {i}", w, p1, 0.5)
    assert ctrl._fast is not None                      # the repeat path is the one under test
    ctrl.policy_net = Pol(p2, 2)
    same("new policy", w, p2, 0.5)
    ctrl.explore = 0.3
    same("explore changed", w, p2, 0.3)
    dm.load_weights(w2.kernels, w2.biases, w2.ln_gamma, w2.ln_beta)
    same("dynamics reloaded", w2, p2, 0.3)
    ctrl._engine.close()
