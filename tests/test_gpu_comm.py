"""The library-owned min-loc exchange (bcmpc_comm_*, csrc/comm.hip) on the GPU box.

One rank: the RCCL all-gather + device selection leave the engine's own result unchanged (the
path every multi-GPU get_action takes, exercised end to end on one card).  Two ranks on one card:
RCCL refuses two ranks on the same GPU on most builds; when it accepts them, the two half-shard
engines must both return the single engine's global argmin.  Multi-GPU scaling is measured by
the driver's 8-GPU bench, not here."""
import ctypes
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _setup(K, H=6):
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    w = orc.synthetic_weights(20, 6, 128, 2, "tanh", False)
    norm = orc.synthetic_normalization(20, 6)
    state = orc.synthetic_state(norm)

    def make(k):
        eng = RolloutEngine(20, 6, 128, 2, "tanh", False, H, k, device=0)
        eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, 1)
        return eng
    return make, state


class _Comm:
    """bcmpc_comm for tests (bootstrap by hand)."""

    def __init__(self, idbuf, n, r):
        from bc_mpc_amd import _lib
        self._lib = _lib.load()
        h = ctypes.c_void_p()
        self.rc = self._lib.bcmpc_comm_init(idbuf, n, r, 0, ctypes.byref(h))
        self.err = self._lib.bcmpc_last_error().decode()
        self.handle = h

    def close(self):
        if self.handle:
            self._lib.bcmpc_comm_destroy(self.handle)
            self.handle = None


def test_single_rank_exchange_is_identity():
    from bc_mpc_amd import _lib
    lib = _lib.load()
    make, state = _setup(3000)
    idbuf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    _lib.check(lib.bcmpc_comm_unique_id(idbuf))
    comm = _Comm(idbuf, 1, 0)
    assert comm.rc == 0, comm.err
    plain, shared = make(3000), make(3000)
    shared.set_comm(comm)
    for seed in (1, 2, 3):
        a = plain.get_action(state, None, seed=seed, cand_offset=500)
        b = shared.get_action(state, None, seed=seed, cand_offset=500)
        assert (a.best_index, a.best_cost) == (b.best_index, b.best_cost)
        assert np.array_equal(a.first_action, b.first_action)
    np.random.seed(4)
    st = np.random.get_state()
    a = plain.get_action_numpy_stream(state, -np.ones(6), np.ones(6), 3000)
    np.random.set_state(st)
    b = shared.get_action_numpy_stream(state, -np.ones(6), np.ones(6), 3000)
    assert (a.best_index, a.best_cost) == (b.best_index, b.best_cost)
    shared.set_comm(None)
    plain.close(), shared.close()
    comm.close()


def test_single_rank_exchange_team_giveup_reruns_collectively(monkeypatch):
    """A team that gives up while a communicator is attached: the exchange carries the rank's status
    flag (comm.hip wire record), every rank sees the OR of the flags, and every rank reruns the step on
    its fallback engine with the communicator attached (one rank here: the whole path on one card).
    Forced with BCMPC_TEAM_SPINS=-1; the answer is the reference fixture's, NumPy's stream advances once."""
    from bc_mpc_amd import _lib
    from conftest import Golden
    from test_gpu_parity import _engine, argmin_is_decidable, assert_costs_close
    lib = _lib.load()
    idbuf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    _lib.check(lib.bcmpc_comm_unique_id(idbuf))
    comm = _Comm(idbuf, 1, 0)
    assert comm.rc == 0, comm.err
    g = Golden("cfg1_2x500_tanh")
    eng = _engine(g, kernel="team")
    assert eng.info()["kernel"] == "team"
    eng.set_comm(comm)
    monkeypatch.setenv("BCMPC_TEAM_SPINS", "-1")
    res = eng.get_action(g.state, g.actions(), return_costs=True)
    assert eng.team_reruns == 1
    assert_costs_close(res.costs, g.costs, g.near, "cfg1 collective rerun")
    if argmin_is_decidable(g):
        assert res.best_index == g.argmin and np.array_equal(res.first_action, g.opt_action)
    # the NumPy-stream drop-in path: the rerun draws again from the same state, the stream advances once
    np.random.seed(9)
    st = np.random.get_state()
    low, high = -np.ones(g.A), np.ones(g.A)
    r1 = eng.get_action_numpy_stream(g.state, low, high, g.K)
    after = np.random.get_state()
    assert eng.team_reruns == 2
    monkeypatch.delenv("BCMPC_TEAM_SPINS")
    np.random.set_state(st)
    r2 = eng.get_action_numpy_stream(g.state, low, high, g.K)       # the team meets: no rerun
    assert eng.team_reruns == 2
    # (the rerun ran the fallback's split slab kernel, r2 the team kernel: same arithmetic, another
    #  summation order of the output partials -- the stated tolerance, same argmin)
    assert r1.best_index == r2.best_index and abs(r1.best_cost - r2.best_cost) <= 1e-4 + 1e-5 * abs(r2.best_cost)
    assert np.array_equal(np.random.get_state()[1], after[1]) and np.random.get_state()[2] == after[2]
    eng.set_comm(None)
    eng.close()
    comm.close()


def test_single_rank_non_team_engine_joins_a_collective_rerun(monkeypatch):
    """With a communicator attached, a flag that ANOTHER rank's team raised (the exchange carries the OR
    of every rank's flags) makes every rank rerun the step together.  A rank whose own kernel is not the
    team kernel reruns the same call on its own engine -- joining the rerun's exchange -- instead of
    building a fallback from host weight copies it does not keep.  The other rank's flag is
    simulated with the test hook BCMPC_COMM_FORCE_FLAGS=n (the first n exchanges carry a set flag)."""
    from bc_mpc_amd import _lib
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    lib = _lib.load()
    w = orc.synthetic_weights(20, 6, 500, 2, "tanh", False)
    norm = orc.synthetic_normalization(20, 6)
    state = orc.synthetic_state(norm)

    def make():
        eng = RolloutEngine(20, 6, 500, 2, "tanh", False, 6, 3000, device=0, kernel="split4")
        eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, 1)
        return eng
    idbuf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    _lib.check(lib.bcmpc_comm_unique_id(idbuf))
    monkeypatch.setenv("BCMPC_COMM_FORCE_FLAGS", "2")
    comm = _Comm(idbuf, 1, 0)
    monkeypatch.delenv("BCMPC_COMM_FORCE_FLAGS")
    assert comm.rc == 0, comm.err
    plain, shared = make(), make()
    assert shared.info()["kernel"] == "split4"
    shared.set_comm(comm)
    a = plain.get_action(state, None, seed=5, cand_offset=500)
    b = shared.get_action(state, None, seed=5, cand_offset=500)    # flagged exchange -> rerun -> clean one
    assert (a.best_index, a.best_cost) == (b.best_index, b.best_cost)
    assert np.array_equal(a.first_action, b.first_action)
    np.random.seed(4)
    st = np.random.get_state()
    a = plain.get_action_numpy_stream(state, -np.ones(6), np.ones(6), 3000)
    after = np.random.get_state()
    np.random.set_state(st)
    b = shared.get_action_numpy_stream(state, -np.ones(6), np.ones(6), 3000)   # flagged again: rerun
    assert (a.best_index, a.best_cost) == (b.best_index, b.best_cost)
    assert np.array_equal(np.random.get_state()[1], after[1]) and np.random.get_state()[2] == after[2]
    c = shared.get_action(state, None, seed=6, cand_offset=500)     # the hook is spent: plain exchange
    d = plain.get_action(state, None, seed=6, cand_offset=500)
    assert (c.best_index, c.best_cost) == (d.best_index, d.best_cost)
    assert shared.team_reruns == 0
    shared.set_comm(None)
    plain.close(), shared.close()
    comm.close()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _two_rank_worker(rank, port, q):
    import sys
    import torch.distributed as dist
    from conftest import REPO
    sys.path.insert(0, REPO)
    from bc_mpc_amd import _lib
    import torch
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    lib = _lib.load()
    idbuf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    if rank == 0:
        _lib.check(lib.bcmpc_comm_unique_id(idbuf))
    t = torch.frombuffer(bytearray(bytes(idbuf)), dtype=torch.uint8)
    dist.broadcast(t, 0)
    ctypes.memmove(idbuf, bytes(t.numpy()), _lib.COMM_ID_BYTES)
    comm = _Comm(idbuf, 2, rank)
    if comm.rc != 0:
        q.put((rank, "init-failed", comm.err))
        dist.destroy_process_group()
        return
    make, state = _setup(2000)
    eng = make(1000)
    eng.set_comm(comm)
    res = eng.get_action(state, None, seed=11, cand_offset=1000 * rank)
    q.put((rank, "ok", (res.best_index, res.best_cost, res.first_action.tolist())))
    eng.set_comm(None)
    eng.close()
    comm.close()
    dist.destroy_process_group()


def test_two_ranks_one_card_agree_on_the_global_argmin():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_two_rank_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(2):
        r, status, val = q.get(timeout=100)
        out[r] = (status, val)
    for p in ps:
        p.join(timeout=60)
    if any(s == "init-failed" for s, _ in out.values()):
        pytest.skip(f"RCCL refuses two ranks on one GPU here: {out[0][1]}")
    make, state = _setup(2000)
    eng = make(2000)
    want = eng.get_action(state, None, seed=11, cand_offset=0)
    eng.close()
    for r in (0, 1):
        idx, cost, first = out[r][1]
        assert (idx, cost) == (want.best_index, want.best_cost)
        assert first == want.first_action.tolist()
