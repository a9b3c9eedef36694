"""The multi-column team kernel (rollout_mc.hip) on the GPU box.

Same arithmetic and summation orders as the one-column team kernel (rollout_team.hip, T = 4 at hidden
512), so where both run (K small enough for the one-column team) their cost vectors must be
bit-identical; against the reference-run fixtures and the oracle it must meet the fp32 bar of
test_gpu_parity.py.  Also: shard invariance (bitwise), ragged K / H, HBM action arrays, the NumPy-stream
drop-in, and the forced give-up path (the call reruns on the fallback engine)."""
import numpy as np
import pytest

from conftest import ENV_PLAIN, Golden, envelope

pytestmark = pytest.mark.gpu


def _weights(seed_base=7):
    from oracle import mpc_oracle as orc
    w = orc.synthetic_weights(20, 6, 500, 2, "tanh", False, seed_base=seed_base)
    norm = orc.synthetic_normalization()
    return w, norm, orc.synthetic_state(norm)


def _engine(w, norm, H, K, mc=True, monkeypatch=None, kernel="auto"):
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    if monkeypatch is not None:
        monkeypatch.setenv("BCMPC_MC", "1" if mc else "0")
    eng = RolloutEngine(20, 6, w.hidden, w.n_layers, w.activation, False, H, K, device=0, kernel=kernel)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, version=1)
    if monkeypatch is not None:
        monkeypatch.delenv("BCMPC_MC")
    lay = eng.info()["layout"]
    assert lay.startswith("rollout_mc") == mc, lay
    return eng


@pytest.mark.parametrize("K,H", [(1000, 15), (64, 3), (1, 1), (900, 1)])
def test_mc_bitwise_equal_to_one_column_team(K, H, monkeypatch):
    """Where the one-column team fits, the multi-column kernel (forced) computes the same bits."""
    w, norm, state = _weights()
    team = _engine(w, norm, H, K, mc=False, monkeypatch=monkeypatch, kernel="team")
    mc = _engine(w, norm, H, K, mc=True, monkeypatch=monkeypatch)
    for seed in (3, 4):
        a = team.get_action(state, None, seed=seed, return_costs=True)
        b = mc.get_action(state, None, seed=seed, return_costs=True)
        assert np.array_equal(a.costs, b.costs, equal_nan=True)
        assert (a.best_index, a.best_cost) == (b.best_index, b.best_cost)
        assert np.array_equal(a.first_action, b.first_action)
    acts = np.random.RandomState(5).uniform(-1, 1, (H, K, 6))
    a = team.get_action(state, acts, return_costs=True)
    b = mc.get_action(state, acts, return_costs=True)
    assert np.array_equal(a.costs, b.costs, equal_nan=True)
    assert b.best_index == int(np.argmin(b.costs)) and np.array_equal(b.first_action, acts[0, b.best_index])
    team.close(), mc.close()


def test_mc_cfg2_reference_fixture():
    """BASELINE configs[1] (K = 4096, H = 20, 2x500 tanh) through the reference-run fixture on the
    multi-column team kernel (kernel "team" beyond the one-column team's reach takes it): the fp32 bar,
    argmin and first action exact."""
    from test_gpu_parity import argmin_is_decidable, assert_costs_close
    g = Golden("cfg2_2x500_tanh")
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    wt = g.weights
    eng = RolloutEngine(g.S, g.A, wt.hidden, wt.n_layers, wt.activation, False, g.H, g.K, device=0, kernel="team")
    eng.set_weights(MLPSpec(wt.kernels, wt.biases, wt.activation), g.norm, version=1)
    assert eng.info()["layout"].startswith("rollout_mc"), eng.info()["layout"]
    res = eng.get_action(g.state, g.actions(), return_costs=True)
    assert_costs_close(res.costs, g.costs, g.near, "cfg2/mc", env=envelope(False, 2, wt.hidden, g.H))
    if argmin_is_decidable(g):
        assert res.best_index == g.argmin and np.array_equal(res.first_action, g.opt_action)
    eng.close()


@pytest.mark.parametrize("K,H", [(4096, 20), (4100, 7), (5000, 1), (8192, 3), (2049, 20)])
def test_mc_vs_oracle_and_shards(K, H, monkeypatch):
    """Ragged K and H against the oracle (Philox actions, the fp32 bar); two half shards reproduce the
    full engine's cost vector bitwise; deterministic."""
    from oracle import mpc_oracle as orc
    from test_gpu_parity import assert_costs_close
    w, norm, state = _weights(seed_base=11)
    full = _engine(w, norm, H, K, monkeypatch=monkeypatch)
    r = full.get_action(state, None, seed=21, return_costs=True)
    r2 = full.get_action(state, None, seed=21, return_costs=True)
    assert np.array_equal(r.costs, r2.costs, equal_nan=True)
    n = min(K, 512)
    idx = np.linspace(0, K - 1, n).astype(np.int64)
    acts = orc.device_rng_actions(21, 0, K, H, -np.ones(6), np.ones(6))[:, idx]
    want, states = orc.rollout(orc.NumpyDynamics(w, norm), state, acts)
    assert_costs_close(r.costs[idx], want, orc.near_threshold_mask(states), f"mc K{K} H{H}",
                       env=envelope(False, 2, 500, H))
    assert r.best_index == int(np.argmin(r.costs))
    half = K // 2
    lo = _engine(w, norm, H, half, monkeypatch=monkeypatch)
    hi = _engine(w, norm, H, K - half, monkeypatch=monkeypatch)
    a = lo.get_action(state, None, seed=21, cand_offset=0, return_costs=True)
    b = hi.get_action(state, None, seed=21, cand_offset=half, return_costs=True)
    assert np.array_equal(np.concatenate([a.costs, b.costs]), r.costs, equal_nan=True)
    full.close(), lo.close(), hi.close()


def test_mc_numpy_stream_dropin(monkeypatch):
    """The drop-in's NumPy-stream call on the multi-column engine: the same pick as the engine on
    np.random.uniform's own array, NumPy's stream advanced exactly as the reference's one draw."""
    w, norm, state = _weights()
    K, H = 4096, 20
    eng = _engine(w, norm, H, K, monkeypatch=monkeypatch)
    low, high = -np.ones(6), np.ones(6)
    for seed in (1, 2):
        np.random.seed(seed)
        st = np.random.get_state()
        r = eng.get_action_numpy_stream(state, low, high, K)
        after = np.random.get_state()
        np.random.set_state(st)
        acts = np.random.uniform(low, high, (H, K, 6))
        assert np.array_equal(after[1], np.random.get_state()[1]) and after[2] == np.random.get_state()[2]
        ref = eng.get_action(state, acts, return_costs=True)
        assert (r.best_index, r.best_cost) == (ref.best_index, ref.best_cost)
        assert np.array_equal(r.first_action, acts[0, r.best_index])
    eng.close()


def test_mc_forced_giveup_reruns_on_fallback(monkeypatch):
    """BCMPC_TEAM_SPINS=-1 skips the team launch and reports it as given up: the synchronous call reruns
    on the fallback (split slab) engine -- same argmin within the fp32 bar."""
    w, norm, state = _weights()
    K, H = 4096, 10
    eng = _engine(w, norm, H, K, monkeypatch=monkeypatch)
    ok = eng.get_action(state, None, seed=9, return_costs=True)
    monkeypatch.setenv("BCMPC_TEAM_SPINS", "-1")
    rr = eng.get_action(state, None, seed=9, return_costs=True)
    monkeypatch.delenv("BCMPC_TEAM_SPINS")
    assert eng.team_reruns == 1
    assert np.max(np.abs(rr.costs - ok.costs)) <= ENV_PLAIN
    assert rr.best_index == ok.best_index
    eng.close()
