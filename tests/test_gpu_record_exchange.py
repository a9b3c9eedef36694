"""distributed.RecordExchange (the bench's N > 1 exchange: torch all-gather of the 144-byte result records +
the library's device select + one D2H) over a REAL RCCL communicator: a 1-rank "nccl" process group on the box's
one GPU, in a child process (so no process group leaks into the other tests).  The gathered-and-selected
winner must equal the synchronous get_action's on the same shard, seeds and offset (the select of one
record is the identity), and the reward engine's argmax rule must hold the same way.  The 2-rank form of the
same exchange runs through gloo in tests/test_gpu_bench_contract.py (RCCL refuses two ranks on one card)."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import sys, numpy as np, torch, torch.distributed as dist
sys.path.insert(0, REPO)
dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
from bc_mpc_amd import distributed as bd
from bc_mpc_amd.engine import MLPSpec, RolloutEngine
from oracle import mpc_oracle as orc
for model in ("delta", "reward"):
    K, H = 3000, 6
    if model == "delta":
        w = orc.synthetic_weights(20, 6, 128, 2, "tanh", False)
        spec = MLPSpec(w.kernels, w.biases, "tanh")
        norm = orc.synthetic_normalization(20, 6)
        eng = RolloutEngine(20, 6, 128, 2, "tanh", False, H, K, device=0)
    else:
        w = orc.synthetic_reward_weights(20, 6, 128, False)
        spec = MLPSpec(w.kernels, w.biases, "tanh", model="reward")
        norm = orc.synthetic_normalization(20, 6, reward=True)
        eng = RolloutEngine(20, 6, 128, 2, "tanh", False, H, K, device=0, cost="reward", model="reward")
    eng.set_weights(spec, norm, 1)
    state = orc.synthetic_state(norm)
    ex = bd.RecordExchange(0, maximize=(model == "reward"))
    assert ex.collective and ex.backend == "nccl", (ex.collective, ex.backend)
    stream = torch.cuda.current_stream(0)
    d_state = torch.from_numpy(state).cuda(0)
    d_costs = torch.empty(K, dtype=torch.float64, device="cuda:0")
    for seed in (1, 2, 3):
        want = eng.get_action(state, None, seed=seed, cand_offset=700)
        eng.rollout_async(d_state.data_ptr(), 0, None, seed, 700, d_costs.data_ptr(), None, ex.d_result.data_ptr(),
                          stream.cuda_stream)
        cost, index, first = ex.exchange(stream)
        assert (index, cost) == (want.best_index, want.best_cost), (model, seed, index, cost, want)
        assert np.array_equal(first[:6], want.first_action)
        # the host-staged exchange the controllers use (distributed.allgather_minloc): the record goes
        # through the pinned staging buffers, the 1-rank RCCL all-gather and the vectorised select unchanged
        sign = -1.0 if model == "reward" else 1.0
        c2, i2, f2 = bd.allgather_minloc(True, sign * want.best_cost, want.best_index, want.first_action, 6,
                                         device=0)
        assert (sign * c2, i2) == (want.best_cost, want.best_index) and np.array_equal(f2, want.first_action)
    eng.close()
    print(model, "ok")
dist.destroy_process_group()
print("RECORD_EXCHANGE_OK")
'''


def test_record_exchange_over_a_one_rank_rccl_group():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1")
    p = subprocess.run([sys.executable, "-c", f"REPO = {REPO!r}\n" + CHILD], capture_output=True, text=True,
                       timeout=180, cwd=REPO, env=env)
    print(p.stdout[-2000:])
    assert p.returncode == 0 and "RECORD_EXCHANGE_OK" in p.stdout, p.stderr[-3000:]
