"""The per-engine timing switch (bcmpc_engine_set_timing): off by default, so the synchronous
get_action carries no HIP event markers; on, last_kernel_ms reads the rollout's events.  The
switch changes no result bit (team kernel at small K, split kernel at larger K)."""
import numpy as np
import pytest

from oracle import mpc_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("K,H,hidden,act,ln,kernel", [(400, 7, 256, "relu", True, None),
                                                      (8192, 5, 500, "tanh", False, "split4")])
def test_timing_switch(K, H, hidden, act, ln, kernel):
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    norm = orc.synthetic_normalization(seed=3)
    w = orc.synthetic_weights(20, 6, hidden, 2, act, ln, seed_base=77)
    eng = RolloutEngine(20, 6, hidden, 2, act, ln, H, K, kernel=kernel)
    eng.set_weights(MLPSpec(w.kernels, w.biases, act, w.ln_gamma, w.ln_beta), norm, 1)
    state = orc.synthetic_state(norm, seed=4)
    plain = eng.get_action(state, None, seed=21, return_costs=True)
    with pytest.raises(Exception, match="not timed"):
        eng.last_kernel_ms()
    eng.set_timing(True)
    timed = eng.get_action(state, None, seed=21, return_costs=True)
    rollout_ms, argmin_ms = eng.last_kernel_ms()
    assert rollout_ms > 0.0 and argmin_ms >= 0.0
    assert np.array_equal(plain.costs, timed.costs) and plain.best_index == timed.best_index
    assert np.array_equal(plain.first_action, timed.first_action)
    eng.set_timing(False)
    again = eng.get_action(state, None, seed=21)
    assert again.best_index == plain.best_index
    with pytest.raises(Exception, match="not timed"):
        eng.last_kernel_ms()
    eng.close()
