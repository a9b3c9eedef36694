"""BASELINE cfg4 and cfg5 as whole workloads on one MI355X.

cfg4 (K=262144, H=20, 2x500 tanh, "sharded 8x MI355X with RCCL min-loc"): the eight 32768-candidate
shards a node would run (cand_offset = g * 32768) run one after another on this card, in device-RNG
mode and in the drop-in's NumPy-stream mode (each shard draws only its own rows of the global
[H, 262144, 6] array on the GPU).  The concatenated shard cost vectors equal one K=262144 engine's
bit for bit, the min-loc over the eight shard records equals np.argmin of the full vector (with the
first action of the winning row), every shard leaves NumPy's stream where the full draw leaves it,
and a 256-candidate sample is within the fp32 tolerance of the oracle.

cfg5 (K=65536, H=50, 3x1024 tanh, CEM x4): every iteration on the split kernel checked like
tests/test_gpu_cem.py at full size -- a 256-candidate oracle sample of the costs, the elite set equal
to oracle.cem_select of the GPU's costs, the refit mu / sigma bit-identical to oracle.cem_refit --
and the fused bcmpc_cem_get_action equal to the step-by-step launches.
"""
import ctypes

import numpy as np
import pytest

from conftest import ENV_WIDE
from test_gpu_parity import assert_costs_close

pytestmark = pytest.mark.gpu

S, A = 20, 6
ELITE = np.dtype([("cost", "<f8"), ("index", "<i8")])


def _delta_problem(hidden, L, seed_base=1000):
    from bc_mpc_amd.engine import MLPSpec
    from oracle import mpc_oracle as orc
    w = orc.synthetic_weights(S, A, hidden, L, "tanh", False, seed_base=seed_base)
    norm = orc.synthetic_normalization(S, A)
    return MLPSpec(w.kernels, w.biases, "tanh"), orc.NumpyDynamics(w, norm), norm, orc.synthetic_state(norm)


@pytest.mark.parametrize("mode", ["device", "numpy"])
def test_cfg4_eight_shards_equal_one_engine(mode):
    from bc_mpc_amd import _lib
    from bc_mpc_amd import distributed as bd
    from bc_mpc_amd.engine import RolloutEngine
    from oracle import mpc_oracle as orc
    KG, G, H = 262144, 8, 20
    KS = KG // G
    low, high = -np.ones(A), np.ones(A)
    spec, dyn, norm, state = _delta_problem(500, 2)
    full = RolloutEngine(S, A, 500, 2, "tanh", False, H, KG, device=0)
    full.set_weights(spec, norm, 1)
    shard = RolloutEngine(S, A, 500, 2, "tanh", False, H, KS, device=0)
    shard.set_weights(spec, norm, 1)
    assert shard.precision == "split" and full.precision == "split"
    seed = 77
    np.random.seed(2026)
    np.random.random(5)                               # an odd position in the key block
    st0 = np.random.get_state()
    if mode == "device":
        ref = full.get_action(state, None, seed=seed, return_costs=True)
    else:
        ref = full.get_action_numpy_stream(state, low, high, KG, 0, return_costs=True)
        st_full = np.random.get_state()
        np.random.set_state(st0)
        actions = np.random.uniform(low, high, [H, KG, A])   # the reference's own draw (controllers.py:53)
        st_want = np.random.get_state()
        assert np.array_equal(st_full[1], st_want[1]) and st_full[2] == st_want[2]
    costs, recs = [], []
    for g in range(G):
        if mode == "device":
            r = shard.get_action(state, None, seed=seed, cand_offset=g * KS, return_costs=True)
        else:
            np.random.set_state(st0)
            r = shard.get_action_numpy_stream(state, low, high, KG, g * KS, return_costs=True)
            st = np.random.get_state()
            assert np.array_equal(st[1], st_want[1]) and st[2] == st_want[2], f"shard {g} left another state"
        costs.append(r.costs.copy())
        rec = _lib.Result()
        rec.best_index, rec.best_cost = r.best_index, r.best_cost
        rec.first_action[:A] = r.first_action
        recs.append(rec)
    full.close(), shard.close()
    cat = np.concatenate(costs)
    assert np.array_equal(cat, ref.costs), "8 shards != one K=262144 engine"
    cost, index, first = bd.select_results_host(recs)
    assert index == int(np.argmin(cat)) == ref.best_index and cost == ref.best_cost
    if mode == "device":
        want_first = orc.device_rng_actions(seed, index, 1, 1, low, high)[0, 0]
    else:
        want_first = actions[0, index]
    assert np.array_equal(first[:A], want_first) and np.array_equal(ref.first_action, want_first)
    # a 256-candidate oracle sample straddling the boundary of shards 3 and 4
    lo = 4 * KS - 128
    if mode == "device":
        acts = orc.device_rng_actions(seed, lo, 256, H, low, high)
    else:
        acts = np.ascontiguousarray(actions[:, lo:lo + 256])
    want, states = orc.rollout(dyn, state, acts)
    assert_costs_close(cat[lo:lo + 256], want, orc.near_threshold_mask(states), f"cfg4 {mode} sample")


def test_cfg5_cem_full_size_pinned_to_oracle():
    import torch
    from bc_mpc_amd import _lib
    from bc_mpc_amd.engine import RolloutEngine
    from oracle import mpc_oracle as orc
    K, H, iters, alpha, seed = 65536, 50, 4, 0.1, 0xCF5
    E = int(round(0.1 * K))
    low, high = -np.ones(A), np.ones(A)
    spec, dyn, norm, state = _delta_problem(1024, 3)
    eng = RolloutEngine(S, A, 1024, 3, "tanh", False, H, K, device=0)
    eng.set_weights(spec, norm, 1)
    assert eng.precision == "split"
    dev = torch.device("cuda", 0)
    f64 = dict(dtype=torch.float64, device=dev)
    d_costs = torch.empty(K, **f64)
    d_res = torch.zeros(ctypes.sizeof(_lib.Result), dtype=torch.uint8, device=dev)
    d_el = torch.empty(E * 16, dtype=torch.uint8, device=dev)
    d_cnt = torch.zeros(1, dtype=torch.int32, device=dev)
    mu0, sd0 = np.zeros((H, A)), np.full((H, A), 0.5)
    d_state = torch.from_numpy(state).to(dev)
    d_mu, d_sd = torch.from_numpy(mu0.copy()).to(dev), torch.from_numpy(sd0.copy()).to(dev)
    st = torch.cuda.current_stream(dev).cuda_stream
    sample = np.sort(np.random.RandomState(5).choice(K, 256, replace=False))
    all_costs = []
    for it in range(iters):
        mu_in, sd_in = d_mu.cpu().numpy(), d_sd.cpu().numpy()
        eng.cem_rollout_async(d_state.data_ptr(), d_mu.data_ptr(), d_sd.data_ptr(), seed, it, 0, K,
                              d_costs.data_ptr(), d_res.data_ptr(), it > 0, st)
        costs = d_costs.cpu().numpy()
        acts = orc.cem_actions(seed, it, 0, K, H, mu_in, sd_in, low, high, index=sample)
        want, states = orc.rollout(dyn, state, acts)
        assert_costs_close(costs[sample], want, orc.near_threshold_mask(states), f"cfg5 it{it}", env=ENV_WIDE)
        all_costs.append(costs)
        eng.select_async(None, d_costs.data_ptr(), K, 0, E, d_el.data_ptr(), d_cnt.data_ptr(), st)
        rec = d_el.cpu().numpy().view(ELITE)
        want_el = orc.cem_select(costs, np.arange(K), E)
        assert int(d_cnt.cpu()[0]) == E and np.array_equal(rec["index"][:E], want_el)
        eng.cem_refit_async(d_el.data_ptr(), d_cnt.data_ptr(), seed, it, alpha, d_mu.data_ptr(), d_sd.data_ptr(), st)
        m2, s2 = orc.cem_refit(want_el, seed, it, mu_in, sd_in, low, high, alpha)
        assert np.array_equal(d_mu.cpu().numpy(), m2), f"it{it}: refit mean not bit-identical"
        assert np.array_equal(d_sd.cpu().numpy(), s2), f"it{it}: refit std not bit-identical"
    flat = np.concatenate(all_costs)
    raw = d_res.cpu().numpy()
    pos, cost = int(raw[:8].view(np.int64)[0]), float(raw[8:16].view(np.float64)[0])
    assert pos == int(np.argmin(flat)) and cost == flat[pos]
    res, mu, sd = eng.cem_get_action(state, mu0, sd0, iters, E, alpha, seed)
    assert res.best_index == pos and res.best_cost == cost
    assert np.array_equal(mu, d_mu.cpu().numpy()) and np.array_equal(sd, d_sd.cpu().numpy())
    eng.close()
