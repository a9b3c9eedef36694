"""CEM outer loop (BASELINE cfg5) on CPU: the oracle restatement's own invariants and
the multi-rank orchestration (bc_mpc_amd.cem.cem_multi_rank) on 2 gloo ranks.

The reference has no CEM, so these pin the engine's DEFINED semantics (DESIGN.md
"CEM"): the sampler, the elite rule, the refit reduction order and the
"best over all iterations" answer.  Kernel parity against this oracle is in
tests/test_gpu_cem.py.
"""
import ctypes
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO
from oracle import mpc_oracle as orc

ELITE = np.dtype([("cost", "<f8"), ("index", "<i8")])


def test_irwin_hall_normals_are_exact_and_standard():
    z = orc.cem_normals(77, 2, 1000, 4096, 3, 6)
    assert z.shape == (3, 4096, 6)
    assert np.array_equal(z, np.round(z * 2**24) / 2**24)           # exact multiples of 2^-24
    assert z.min() >= -6 and z.max() < 6
    assert abs(z.mean()) < 0.02 and abs(z.std() - 1.0) < 0.02        # Irwin-Hall(12) - 6: mean 0, var 1
    # keyed by the global candidate: a shard reproduces its slice of the full draw
    full = orc.cem_normals(77, 2, 0, 5096, 3, 6)
    assert np.array_equal(full[:, 1000:], z)
    # iterations draw independent streams
    assert not np.array_equal(orc.cem_normals(77, 3, 1000, 16, 3, 6), z[:, :16])


def test_cem_actions_clip_like_numpy():
    mu = np.full((2, 6), 0.9)
    sd = np.full((2, 6), 0.5)
    a = orc.cem_actions(5, 0, 0, 512, 2, mu, sd, -np.ones(6), np.ones(6))
    assert a.max() == 1.0 and a.min() >= -1.0 and (a == 1.0).mean() > 0.2


def test_select_rule():
    costs = np.array([3.0, np.nan, 1.0, 1.0, -0.0, 0.0, 2.0, np.nan, -5.0])
    idx = np.arange(costs.size) + 100
    # stable: -5 (108), -0 (104) == +0 (105) tie -> both, 1.0 (102, 103) ...
    assert orc.cem_select(costs, idx, 4).tolist() == [102, 104, 105, 108]
    assert orc.cem_select(costs, idx, 3).tolist() == [104, 105, 108]
    assert orc.cem_select(costs, idx, 5).tolist() == [102, 103, 104, 105, 108]
    # NaN last: asking for everything returns everything, NaNs included
    assert orc.cem_select(costs, idx, 9).tolist() == idx.tolist()
    # maximize: largest first, NaN still last
    assert orc.cem_select(costs, idx, 2, maximize=True).tolist() == [100, 106]
    # empty records (index < 0) never selected
    assert orc.cem_select(np.array([0.0, -1.0]), np.array([-1, 7]), 2).tolist() == [7]


def test_select_of_local_selects_equals_global_select():
    rs = np.random.RandomState(0)
    K, E = 1000, 37
    costs = np.round(rs.standard_normal(K), 1)            # many exact ties
    costs[rs.choice(K, 20, replace=False)] = np.nan
    glob = orc.cem_select(costs, np.arange(K), E)
    parts = []
    for lo, hi in [(0, 333), (333, 700), (700, 1000)]:
        sel = orc.cem_select(costs[lo:hi], np.arange(lo, hi), E)
        parts.append((costs[sel], sel))
    c = np.concatenate([p[0] for p in parts])
    i = np.concatenate([p[1] for p in parts])
    assert np.array_equal(orc.cem_select(c, i, E), glob)


def test_refit_matches_numpy_statistics():
    low, high = -np.ones(6), np.ones(6)
    mu = np.zeros((3, 6))
    sd = np.full((3, 6), 0.5)
    el = np.sort(np.random.RandomState(1).choice(5000, 300, replace=False))
    m1, s1 = orc.cem_refit(el, 9, 1, mu, sd, low, high, alpha=0.0)
    acts = orc.cem_actions(9, 1, 0, 5000, 3, mu, sd, low, high)[:, el, :]
    assert np.allclose(m1, acts.mean(axis=1), rtol=0, atol=1e-15)
    assert np.allclose(s1, acts.std(axis=1), rtol=0, atol=1e-15)
    m2, s2 = orc.cem_refit(el, 9, 1, mu, sd, low, high, alpha=0.25)
    assert np.array_equal(m2, 0.25 * mu + 0.75 * m1) and np.array_equal(s2, 0.25 * sd + 0.75 * s1)


def test_cem_loop_improves_and_answers_best_of_all_iterations():
    w = orc.synthetic_weights(20, 6, 64, 2, "tanh", False)
    norm = orc.synthetic_normalization()
    dyn = orc.NumpyDynamics(w, norm)
    state = orc.synthetic_state(norm)
    H, K = 5, 400
    mu0, sd0 = np.zeros((H, 6)), np.full((H, 6), 0.5)
    first, pos, flat, mu, sd, hist = orc.cem_get_action(lambda s, a: orc.rollout(dyn, s, a)[0], state, H, K,
                                                        -np.ones(6), np.ones(6), 4, 40, 0.1, 123, mu0, sd0)
    assert pos == int(np.argmin(flat)) and flat.shape == (4 * K,)
    it_best = flat.reshape(4, K).min(axis=1)
    assert it_best[-1] <= it_best[0]                          # the distribution moved towards low cost
    assert (sd < sd0).all()                                   # and contracted
    it, i = divmod(pos, K)
    acts = orc.cem_actions(123, it, 0, K, H, *hist[it], -np.ones(6), np.ones(6))
    assert np.array_equal(first, acts[0, i])


# ------------------------------------------------------------------ 2 gloo ranks
class ShardDouble:
    """NumPy stand-in for cem._EngineShard (CPU tensors, oracle math)."""

    def __init__(self, dyn, K_local, H, A):
        self.dyn, self.K, self.H, self.A = dyn, K_local, H, A
        self.device = torch.device("cpu")
        self.low, self.high = -np.ones(A), np.ones(A)

    def rollout(self, d_state, d_mu, d_sigma, seed, it, lo, k_global, d_costs, d_res, merge):
        mu, sd = d_mu.numpy(), d_sigma.numpy()
        acts = orc.cem_actions(seed, it, lo, self.K, self.H, mu, sd, self.low, self.high)
        costs, _ = orc.rollout(self.dyn, d_state.numpy(), acts)
        d_costs[: self.K] = torch.from_numpy(costs)
        i = int(np.argmin(costs))
        raw = d_res.numpy()
        pos = it * k_global + lo + i
        if merge:
            pc, pp = float(raw[8:16].view(np.float64)[0]), int(raw[:8].view(np.int64)[0])
            if not (np.isnan(costs[i]) and not np.isnan(pc)) and not (costs[i] < pc):
                return                                      # np.argmin keeps the earlier position on ties
        raw[:8].view(np.int64)[0] = pos
        raw[8:16].view(np.float64)[0] = costs[i]
        raw[16:16 + 8 * self.A].view(np.float64)[:] = acts[0, i]

    def _write(self, d_out, d_count, sel_idx, cost_of, n_elite):
        rec = np.zeros(n_elite, dtype=ELITE)
        rec["cost"], rec["index"] = np.nan, -1
        rec["cost"][: sel_idx.size] = [cost_of[g] for g in sel_idx]
        rec["index"][: sel_idx.size] = sel_idx
        d_out.copy_(torch.from_numpy(rec.view(np.uint8)))
        d_count[0] = sel_idx.size

    def select(self, d_pairs, d_costs, m, index_base, n_elite, d_out, d_count):
        if d_pairs is not None:
            rec = d_pairs.numpy().view(ELITE)[:m]
            costs, idx = rec["cost"], rec["index"]
        else:
            costs = d_costs.numpy()[:m]
            idx = np.arange(m) + index_base
        sel = orc.cem_select(costs, idx, n_elite)
        self._write(d_out, d_count, sel, dict(zip(idx.tolist(), costs.tolist())), n_elite)

    def refit(self, d_elite, d_count, seed, it, alpha, d_mu, d_sigma):
        n = int(d_count[0])
        el = d_elite.numpy().view(ELITE)["index"][:n]
        mu, sd = orc.cem_refit(el, seed, it, d_mu.numpy(), d_sigma.numpy(), self.low, self.high, alpha)
        d_mu.copy_(torch.from_numpy(mu))
        d_sigma.copy_(torch.from_numpy(sd))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _problem():
    w = orc.synthetic_weights(20, 6, 64, 2, "tanh", False)
    norm = orc.synthetic_normalization()
    return orc.NumpyDynamics(w, norm), orc.synthetic_state(norm)


def _worker(rank, world, port, q, K, H, E):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bc_mpc_amd import distributed as bdist
    from bc_mpc_amd.cem import cem_multi_rank
    dyn, state = _problem()
    lo, hi = bdist.shard_range(K, rank, world)
    shard = ShardDouble(dyn, hi - lo, H, 6)
    mu0, sd0 = np.zeros((H, 6)), np.full((H, 6), 0.5)
    cost, pos, first, mu, sd = cem_multi_rank(shard, state, mu0, sd0, 3, E, 0.1, 4242, lo, hi, K, 6, False)
    q.put((rank, cost, pos, first.tolist(), mu.tolist(), sd.tolist()))
    dist.destroy_process_group()


def test_two_rank_cem_matches_single_process_oracle():
    K, H, E = 301, 4, 29
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, K, H, E)) for r in range(2)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(2):
        r, *rest = q.get(timeout=180)
        out[r] = rest
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1], "ranks disagree"
    dyn, state = _problem()
    first, pos, flat, mu, sd, _ = orc.cem_get_action(lambda s, a: orc.rollout(dyn, s, a)[0], state, H, K,
                                                     -np.ones(6), np.ones(6), 3, E, 0.1, 4242,
                                                     np.zeros((H, 6)), np.full((H, 6), 0.5))
    cost_g, pos_g, first_g, mu_g, sd_g = out[0]
    assert pos_g == pos and cost_g == flat[pos]
    assert first_g == first.tolist()
    assert np.array_equal(np.array(mu_g), mu) and np.array_equal(np.array(sd_g), sd)   # bit-identical refits


def test_elite_record_layout_matches_c_struct():
    from bc_mpc_amd import _lib
    assert ctypes.sizeof(_lib.Elite) == ELITE.itemsize == 16
    assert _lib.Elite.index.offset == ELITE.fields["index"][1] == 8
