"""Forward progress of the small-K team kernel (rollout_team.hip).

The team kernel's workgroups wait for each other once per step, so a team needs all its members
resident.  These tests pin what happens when that does not hold:

* a team that gives up (forced here with BCMPC_TEAM_SPINS=-1: every member gives up at its first
  exchange) makes the synchronous entry points rerun the call on the engine's fallback engine (split
  slab kernel, or the fp32 group kernel for nets only the team kernel takes in split precision) --
  the result is the reference's (fixtures) and NumPy's stream advances exactly once;
* a stream-ordered launch that gave up is reported by bcmpc_engine_status (Python: check_status);
* a team launched while another stream's kernels hold the CUs waits for them and is correct;
* team launches of two engines on two streams are serialised by the library and both correct.

Plus the device select of the library's multi-rank exchange (bcmpc_select_results_async) against its
host twin on 2, 3 and 8 records (NaN, cross-rank ties, argmax).
"""
import ctypes

import numpy as np
import pytest

from conftest import ENV_WIDE, Golden, RewardGolden

pytestmark = pytest.mark.gpu


@pytest.fixture
def forced_giveup(monkeypatch):
    monkeypatch.setenv("BCMPC_TEAM_SPINS", "-1")
    yield
    monkeypatch.delenv("BCMPC_TEAM_SPINS", raising=False)


def _cfg1_engine(kernel="team"):
    from test_gpu_parity import _engine
    g = Golden("cfg1_2x500_tanh")
    eng = _engine(g, kernel=kernel)
    return g, eng


def test_team_giveup_reruns_on_fallback(forced_giveup, monkeypatch):
    """cfg1 (K=1000, 4 members per column): every member gives up; get_action reruns on the fallback
    engine and returns the reference's answer; with the spin limit restored the team runs again."""
    from test_gpu_parity import argmin_is_decidable, assert_costs_close
    g, eng = _cfg1_engine()
    assert eng.info()["kernel"] == "team"
    res = eng.get_action(g.state, g.actions(), return_costs=True)
    assert eng.team_reruns == 1
    assert_costs_close(res.costs, g.costs, g.near, "cfg1 fallback")
    if argmin_is_decidable(g):
        assert res.best_index == g.argmin and np.array_equal(res.first_action, g.opt_action)
    monkeypatch.delenv("BCMPC_TEAM_SPINS")
    res2 = eng.get_action(g.state, g.actions(), return_costs=True)
    assert eng.team_reruns == 1                                   # the team met this time
    assert_costs_close(res2.costs, g.costs, g.near, "cfg1 team")
    assert res2.best_index == res.best_index
    eng.close()


def test_team_giveup_dropin_numpy_stream(forced_giveup):
    """The drop-in MPCcontroller.get_action (NumPy's stream, controllers.py:53) on a team engine that
    gives up: the rerun draws the same rows, and the global stream advances exactly once."""
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    from test_gpu_parity import _policy_env, argmin_is_decidable
    g = Golden("cfg1_2x500_tanh")

    class Env:
        action_space = _policy_env(g).action_space
        observation_space = _policy_env(g).observation_space
    ctrl = MPCcontroller(Env(), g.dyn(), horizon=g.H, cost_fn=cheetah_cost_fn, num_simulated_paths=g.K)
    np.random.seed(g.meta["seed"])
    a = ctrl.get_action(g.state)
    assert ctrl._engine.info()["kernel"] == "team" and ctrl._engine.team_reruns == 1
    if argmin_is_decidable(g):
        assert np.array_equal(a, g.opt_action)
    assert np.random.random() == float(g.z["next_draw"])


def test_team_giveup_reward_ln_policy(forced_giveup):
    """run.sh's net (LayerNorm reward net + fused policy, 8 members): the fallback is the fp32 group
    kernel (only the team kernel takes this net in split precision); reference fixture."""
    from bc_mpc_amd.engine import MLPSpec, PolicySpec, RolloutEngine
    from test_gpu_reward import assert_rewards_close, decidable
    g = RewardGolden("polrew_explore05_ln")
    p, w = g.policy, g.weights
    eng = RolloutEngine(g.S, g.A, w.hidden, 2, "tanh", True, g.H, g.K, cost="reward", model="reward",
                        kernel="team", policy_hidden=p.hidden, policy_layers=p.n_layers, policy_mode="explore")
    eng.set_weights(MLPSpec(w.kernels, w.biases, "tanh", w.ln_gamma, w.ln_beta, model="reward"), g.norm, 1)
    eng.set_policy(PolicySpec(p.kernels, p.biases, p.ob_mean, p.ob_std, p.logstd), g.explore, 1)
    expl = np.random.RandomState(g.meta["seed"]).uniform(g.low, g.high, size=[g.H, g.K, g.A])
    res = eng.get_action(g.state, expl, return_costs=True)
    assert eng.team_reruns == 1
    assert_rewards_close(res.costs, g.rewards, "polrew LN fallback", env=ENV_WIDE)
    if decidable(g):
        assert res.best_index == g.argmax
    eng.close()


def test_team_giveup_async_reported(forced_giveup, monkeypatch):
    """bcmpc_rollout_async on a team engine that gives up: check_status raises once, then clears."""
    import torch
    from bc_mpc_amd import _lib
    g, eng = _cfg1_engine()
    dev = torch.device("cuda", 0)
    d_state = torch.from_numpy(g.state).to(dev)
    d_act = torch.from_numpy(np.ascontiguousarray(g.actions())).to(dev)
    d_costs = torch.empty(g.K, dtype=torch.float64, device=dev)
    eng.rollout_async(d_state.data_ptr(), 0, d_act.data_ptr(), 0, 0, d_costs.data_ptr(), None, None,
                      torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    with pytest.raises(_lib.BcmpcError):
        eng.check_status()
    eng.check_status()                                            # read once: cleared
    monkeypatch.delenv("BCMPC_TEAM_SPINS")
    eng.rollout_async(d_state.data_ptr(), 0, d_act.data_ptr(), 0, 0, d_costs.data_ptr(), None, None,
                      torch.cuda.current_stream(dev).cuda_stream)
    torch.cuda.synchronize(dev)
    eng.check_status()
    from test_gpu_parity import assert_costs_close
    assert_costs_close(d_costs.cpu().numpy(), g.costs, g.near, "cfg1 async team")
    eng.close()


def test_team_waits_while_another_stream_holds_the_cus():
    """A team launched while a chain of large GEMMs on another stream occupies the CUs: its members
    become resident as the GEMMs' workgroups drain, the team meets, the answer is the reference's."""
    import torch
    from test_gpu_parity import argmin_is_decidable, assert_costs_close
    g, eng = _cfg1_engine()
    dev = torch.device("cuda", 0)
    side = torch.cuda.Stream(dev)
    a = torch.randn(4096, 4096, device=dev)
    b = torch.randn(4096, 4096, device=dev)
    torch.cuda.synchronize(dev)
    with torch.cuda.stream(side):
        for _ in range(24):
            a = torch.tanh(a @ b * 1e-2)
    res = eng.get_action(g.state, g.actions(), return_costs=True)
    torch.cuda.synchronize(dev)
    assert_costs_close(res.costs, g.costs, g.near, "cfg1 team under load")
    if argmin_is_decidable(g):
        assert res.best_index == g.argmin
    print(f"[team under load] reruns={eng.team_reruns}")
    eng.close()


def test_team_launches_on_two_streams_are_serialised():
    """Two team engines (4 members per column each, 128 + 128 workgroups > half the chip each) launched
    back to back on two streams: the library orders the second behind the first; both correct."""
    import torch
    from test_gpu_parity import _engine, assert_costs_close
    g = Golden("cfg1_2x500_tanh")
    dev = torch.device("cuda", 0)
    e1, e2 = _engine(g, kernel="team"), _engine(g, kernel="team")
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    d_state = torch.from_numpy(g.state).to(dev)
    d_act = torch.from_numpy(np.ascontiguousarray(g.actions())).to(dev)
    c1 = torch.empty(g.K, dtype=torch.float64, device=dev)
    c2 = torch.empty(g.K, dtype=torch.float64, device=dev)
    torch.cuda.synchronize(dev)
    for _ in range(5):
        e1.rollout_async(d_state.data_ptr(), 0, d_act.data_ptr(), 0, 0, c1.data_ptr(), None, None, s1.cuda_stream)
        e2.rollout_async(d_state.data_ptr(), 0, d_act.data_ptr(), 0, 0, c2.data_ptr(), None, None, s2.cuda_stream)
    torch.cuda.synchronize(dev)
    e1.check_status()
    e2.check_status()
    r1, r2 = c1.cpu().numpy(), c2.cpu().numpy()
    assert np.array_equal(r1, r2)
    assert_costs_close(r1, g.costs, g.near, "two streams")
    e1.close(), e2.close()


def _records(n, seed, nan_at=None, tie=False):
    from bc_mpc_amd import _lib
    rs = np.random.RandomState(seed)
    recs = (_lib.Result * n)()
    for r in range(n):
        recs[r].best_index = int(r * 1000 + rs.randint(0, 1000))
        recs[r].best_cost = float(rs.uniform(-50, 50))
        for j in range(6):
            recs[r].first_action[j] = float(rs.uniform(-1, 1))
    if tie:                                  # exact cost ties across ranks: the lowest global index wins
        for r in range(n):
            recs[r].best_cost = -7.25
        recs[n - 1].best_index, recs[0].best_index = recs[0].best_index, recs[n - 1].best_index
    if nan_at is not None:
        recs[nan_at].best_cost = float("nan")
    return recs


@pytest.mark.parametrize("n", [2, 3, 8])
@pytest.mark.parametrize("case", ["plain", "nan", "tie", "argmax", "argmax_nan"])
def test_select_results_async_matches_host(n, case):
    """The exchange's device select (comm.hip select_records_kernel through bcmpc_select_results_async)
    applies np.argmin's rule exactly as the host twin: first NaN, smallest cost, lowest global index on
    ties; np.argmax for the learned reward."""
    import torch
    from bc_mpc_amd import _lib
    lib = _lib.load()
    recs = _records(n, seed=n * 7 + len(case), nan_at=(n - 1 if "nan" in case else None), tie=(case == "tie"))
    maximize = 1 if case.startswith("argmax") else 0
    want = _lib.Result()
    _lib.check(lib.bcmpc_select_results(recs, n, maximize, ctypes.byref(want)))
    dev = torch.device("cuda", 0)
    raw = np.frombuffer(bytes(recs), dtype=np.uint8).copy()
    d_in = torch.from_numpy(raw).to(dev)
    d_out = torch.zeros(ctypes.sizeof(_lib.Result), dtype=torch.uint8, device=dev)
    st = torch.cuda.current_stream(dev)
    _lib.check(lib.bcmpc_select_results_async(ctypes.c_void_p(d_in.data_ptr()), n, maximize,
                                              ctypes.c_void_p(d_out.data_ptr()), ctypes.c_void_p(st.cuda_stream)))
    got = d_out.cpu().numpy().tobytes()
    assert got == bytes(want)
    best = int(np.frombuffer(got[:8], dtype=np.int64)[0])
    costs = np.array([recs[r].best_cost for r in range(n)])
    idx = np.array([recs[r].best_index for r in range(n)])
    sg = -1.0 if maximize else 1.0
    if np.isnan(costs).any():
        assert best == idx[np.isnan(costs)].min()
    else:
        m = (sg * costs).min()
        assert best == idx[sg * costs == m].min()
    with pytest.raises(ValueError):                               # overlapping output is refused
        _lib.check(lib.bcmpc_select_results_async(ctypes.c_void_p(d_in.data_ptr()), n, maximize,
                                                  ctypes.c_void_p(d_in.data_ptr()), ctypes.c_void_p(st.cuda_stream)))
