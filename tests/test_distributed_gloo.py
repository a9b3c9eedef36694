"""N>1 path on CPU: world_size-2 gloo ranks run MPCcontroller SPMD.

The HIP engine is replaced by a test double (``ShardEngine``) that scores its
candidate shard with the oracle -- this exercises only the multi-rank host
logic (sharding, RNG stream consumption on every rank, the one all-gather
min-loc per step, first-action recovery); kernel parity is tested on the GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import REPO


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class ShardEngine:
    """Test double for RolloutEngine (CPU, oracle-backed)."""

    def __init__(self, S, A, hidden, n_layers, activation, layer_norm, horizon, num_paths, device=0, cost="cheetah"):
        self.K, self.H, self.A, self.device = num_paths, horizon, A, device

    def set_action_bounds(self, low, high):
        self.low, self.high = low, high

    def set_weights(self, spec, norm, version):
        from oracle import mpc_oracle as orc
        w = orc.MLPWeights(spec.kernels, spec.biases, spec.activation, spec.ln_gamma, spec.ln_beta)
        self.dyn = orc.NumpyDynamics(w, norm)

    def get_action(self, state, actions, seed=0, cand_offset=0, return_costs=False):
        from bc_mpc_amd.engine import StepResult
        from oracle import mpc_oracle as orc
        if actions is None:
            actions = orc.device_rng_actions(seed, cand_offset, self.K, self.H, self.low, self.high)
        costs, _ = orc.rollout(self.dyn, state, actions)
        i = int(np.argmin(costs))
        return StepResult(cand_offset + i, float(costs[i]), actions[0, i].copy(), costs)

    def numpy_stream_available(self, low, high):
        return True

    def get_action_numpy_stream(self, state, low, high, k_global, cand_offset=0, return_costs=False, seed=0):
        """The engine's NumPy-stream path: the full [H, k_global, A] from the library's MT19937
        restatement (host-only, bcmpc_mt19937_uniform), this shard's slice rolled out."""
        import ctypes
        from bc_mpc_amd import _lib
        lib = _lib.load()
        st = np.random.get_state()
        key = np.array(st[1], dtype=np.uint32)
        pos = ctypes.c_int32(int(st[2]))
        lo, hi = np.asarray(low, np.float64), np.asarray(high, np.float64)
        full = np.empty((self.H * k_global, self.A))
        dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
        assert lib.bcmpc_mt19937_uniform(key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos),
                                         dp(lo), dp(hi), self.A, self.H * k_global, dp(full)) == 0
        np.random.set_state((st[0], key, pos.value, st[3], st[4]))
        actions = np.ascontiguousarray(full.reshape(self.H, k_global, self.A)[:, cand_offset:cand_offset + self.K])
        return self.get_action(state, actions, cand_offset=cand_offset, return_costs=return_costs)

    def close(self):
        pass


def _worker(rank, world, port, q, rng_mode):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bc_mpc_amd import controllers as C
    from bc_mpc_amd.cost_functions import cheetah_cost_fn
    from oracle import mpc_oracle as orc
    C.RolloutEngine = ShardEngine
    env = _Env()
    w = orc.synthetic_weights(20, 6, 64, 2, "tanh", False)
    dyn = orc.NumpyDynamics(w, orc.synthetic_normalization())
    state = orc.synthetic_state(orc.synthetic_normalization())
    ctrl = C.MPCcontroller(env, dyn, horizon=4, cost_fn=cheetah_cost_fn,
                           num_simulated_paths=37, rng=rng_mode, seed=5 if rng_mode == "device" else None)
    np.random.seed(99)
    acts = [ctrl.get_action(state) for _ in range(3)]
    q.put((rank, [a.tolist() for a in acts], float(np.random.random())))
    dist.destroy_process_group()


class _Box:
    def __init__(self, n, lo, hi):
        self.low = np.full(n, lo, dtype=np.float32)
        self.high = np.full(n, hi, dtype=np.float32)
        self.shape = (n,)


class _Env:
    action_space = _Box(6, -1, 1)
    observation_space = _Box(20, -np.inf, np.inf)


@pytest.mark.parametrize("rng_mode", ["numpy", "device"])
def test_two_rank_controller_matches_single_process(rng_mode):
    from oracle import mpc_oracle as orc
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, rng_mode)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict()
    for _ in range(2):
        r, acts, nxt = q.get(timeout=180)
        out[r] = (acts, nxt)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[0] == out[1], "ranks disagree"
    # single-process reference of the same three steps
    w = orc.synthetic_weights(20, 6, 64, 2, "tanh", False)
    dyn = orc.NumpyDynamics(w, orc.synthetic_normalization())
    state = orc.synthetic_state(orc.synthetic_normalization())
    np.random.seed(99)
    seed_rng = np.random.RandomState(5)
    want = []
    for _ in range(3):
        if rng_mode == "numpy":
            a, _, _ = orc.get_action(dyn, state, 4, 37, -np.ones(6, np.float32), np.ones(6, np.float32))
        else:
            seed = int(seed_rng.randint(0, 2**62, dtype=np.int64))
            ap = orc.device_rng_actions(seed, 0, 37, 4, -np.ones(6), np.ones(6))
            costs, _ = orc.rollout(dyn, state, ap)
            a = ap[0, int(np.argmin(costs))]
        want.append(a.tolist())
    assert out[0][0] == want
    assert out[0][1] == float(np.random.random())   # both ranks consumed the stream like one process


def _result_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, REPO)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bc_mpc_amd import distributed as bd
    # bcmpc_result layout: int64 index, f64 cost, f64 first_action[16]
    costs = {0: 3.5, 1: 1.25, 2: 1.25}                  # tie between ranks 1 and 2: the lower index wins
    raw = np.zeros(144, dtype=np.uint8)
    raw[0:8] = np.frombuffer(np.int64(100 * rank + 7).tobytes(), np.uint8)
    raw[8:16] = np.frombuffer(np.float64(costs[rank]).tobytes(), np.uint8)
    raw[16:64] = np.frombuffer(np.full(6, float(rank)).tobytes(), np.uint8)
    got = bd.allgather_result(torch.from_numpy(raw), 6)
    got_max = bd.allgather_result(torch.from_numpy(raw), 6, maximize=True)
    q.put((rank, got[0], got[1], got[2].tolist(), got_max[0], got_max[1]))
    dist.destroy_process_group()


def test_allgather_result_minloc_gloo():
    """The device-record exchange (bench / multi-rank path): min-loc with the lowest-index tie-break,
    argmax for the learned reward, identical on every rank."""
    world, port = 3, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_result_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
    for rank, c, i, fa, cmax, imax in res:
        assert (c, i, fa) == (1.25, 107, [1.0] * 6)
        assert (cmax, imax) == (3.5, 7)
