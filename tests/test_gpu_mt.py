"""NumPy's legacy MT19937 draw made on the GPU (csrc/mt_device.hip) against NumPy itself.

MPCcontroller.sample_random_actions (controllers.py:53) draws np.random.uniform(low, high,
[H, K, A]) from the global RandomState.  The library draws this engine's shard of that array on
the device -- chunks of the stream reached by MT19937 jump-ahead polynomials, generated and scaled
by one workgroup each -- and hands back the state NumPy would hold afterwards.  Bit-exact: every
double and the final (key, pos) equal NumPy's, for any start position (pos 0..624, odd word
offsets that split a double across two blocks), any shard, and chunk sizes small enough to force
hundreds of jumped chunks.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

# (K_global, K, offset, H, A, pos, chunk words (None: library default), coefficient slices)
CASES = [
    (1000, 1000, 0, 15, 6, 624, None, None),          # cfg1 draw, default plan (round 4: 2^12-word chunks, jumps)
    (1000, 1000, 0, 15, 6, 623, 2000, 4),              # 90 chunks: jumps, pos 623 (first double straddles)
    (4096, 4096, 0, 20, 6, 1, 5000, None),             # cfg2, pos 1
    (8192, 3000, 2500, 7, 5, 0, 3000, 3),              # a shard: runs per step, A = 5
    (8192, 2692, 5500, 7, 5, 311, 3000, 1),            # the last shard (its chunk ends the draw), S = 1
    (20, 7, 13, 3, 1, 17, 4, 2),                       # tiny, A = 1, ragged
    (65536, 65536, 0, 6, 6, 624, None, None),          # 4.7M words, default plan
    (262144, 32768, 98304, 20, 6, 400, None, None),    # one rank of cfg4 (draws 1/8 of 63M words)
]


@pytest.mark.parametrize("case", CASES, ids=[f"kg{c[0]}_k{c[1]}_off{c[2]}_h{c[3]}_a{c[4]}_pos{c[5]}_w{c[6]}"
                                             for c in CASES])
def test_device_draw_equals_numpy(case, monkeypatch):
    from bc_mpc_amd.engine import RolloutEngine
    KG, K, off, H, A, pos, chunk, splits = case
    if chunk is not None:
        monkeypatch.setenv("BCMPC_MT_CHUNK_WORDS", str(chunk))
    if splits is not None:
        monkeypatch.setenv("BCMPC_MT_SPLITS", str(splits))
    rs = np.random.RandomState(7)
    low = -1.0 - rs.rand(A)                                # distinct bounds per action column
    high = 1.0 + rs.rand(A)
    np.random.seed(1234 + KG + pos)
    st = np.random.get_state()
    st0 = (st[0], st[1], pos, 0, 0.0)                      # any position in the key block
    np.random.set_state(st0)
    want = np.random.uniform(low, high, [H, KG, A])[:, off:off + K]
    st_want = np.random.get_state()
    eng = RolloutEngine(20, A, 64, 2, "tanh", False, H, K, device=0, cost="none")
    np.random.set_state(st0)
    got = eng.numpy_stream_draw(low, high, KG, off)
    st_got = np.random.get_state()
    eng.close()
    bad = np.argwhere(got != want)
    assert bad.size == 0, f"{len(bad)} doubles differ, first at {bad[:3].tolist()}"
    assert np.array_equal(st_got[1], st_want[1]) and st_got[2] == st_want[2]


def test_device_draw_consecutive_calls_continue_the_stream():
    """Three draws in a row (the plan is reused, the key changes): each equals NumPy's next draw."""
    from bc_mpc_amd.engine import RolloutEngine
    H, K, A = 9, 777, 6
    low, high = -np.ones(A), np.ones(A)
    eng = RolloutEngine(20, A, 64, 2, "tanh", False, H, K, device=0, cost="none")
    np.random.seed(5)
    st = np.random.get_state()
    for _ in range(3):
        np.random.set_state(st)
        want = np.random.uniform(low, high, [H, K, A])
        st_next = np.random.get_state()
        np.random.set_state(st)
        got = eng.numpy_stream_draw(low, high, K, 0)
        assert np.array_equal(got, want)
        st = np.random.get_state()
        assert np.array_equal(st[1], st_next[1]) and st[2] == st_next[2]
    eng.close()


@pytest.mark.parametrize("path,K,H", [("device", 3000, 8), ("host", 3000, 8), ("zero_copy", 3000, 8),
                                      ("device", 400, 7), ("zero_copy", 400, 7)])
def test_get_action_numpy_stream_paths_agree(path, K, H, monkeypatch):
    """bcmpc_get_action_mt19937 on every draw path (the device chain, the host split + upload, the host
    draw read in place by the kernel for small draws): the same costs and argmin as the engine fed
    NumPy's own array, and NumPy's stream left where its one draw leaves it."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    monkeypatch.setenv("BCMPC_MT_PATH", "host" if path == "host" else "device")
    monkeypatch.setenv("BCMPC_MT_ZC_WORDS", str(1 << 30) if path == "zero_copy" else "0")
    S, A = 20, 6
    w = orc.synthetic_weights(S, A, 128, 2, "tanh", False)
    norm = orc.synthetic_normalization(S, A)
    state = orc.synthetic_state(norm)
    low, high = -np.ones(A), np.ones(A)
    eng = RolloutEngine(S, A, 128, 2, "tanh", False, H, K, device=0)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, 1)
    np.random.seed(31)
    st0 = np.random.get_state()
    actions = np.random.uniform(low, high, [H, K, A])
    st_want = np.random.get_state()
    ref = eng.get_action(state, actions, return_costs=True)
    np.random.set_state(st0)
    res = eng.get_action_numpy_stream(state, low, high, K, return_costs=True)
    st = np.random.get_state()
    eng.close()
    assert np.array_equal(res.costs, ref.costs) and res.best_index == ref.best_index
    assert np.array_equal(res.first_action, actions[0, ref.best_index])
    assert np.array_equal(st[1], st_want[1]) and st[2] == st_want[2]


def test_failed_call_leaves_the_stream_untouched():
    """An engine without weights fails (BCMPC_ERR_STATE) before anything is drawn for the caller:
    NumPy's global state is unchanged (the reference would not have been called either)."""
    from bc_mpc_amd.engine import RolloutEngine
    eng = RolloutEngine(20, 6, 64, 2, "tanh", False, 4, 100, device=0)
    np.random.seed(8)
    st0 = np.random.get_state()
    with pytest.raises(Exception):
        eng.get_action_numpy_stream(np.zeros(20), -np.ones(6), np.ones(6), 100)
    st = np.random.get_state()
    eng.close()
    assert np.array_equal(st[1], st0[1]) and st[2] == st0[2]


def test_zero_copy_shard_continues_the_stream(monkeypatch):
    """A rank's shard of a small draw on the zero-copy path (k_global > K, offset > 0): its costs are
    the engine's on NumPy's own rows, and the stream ends where the WHOLE draw leaves it."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    monkeypatch.setenv("BCMPC_MT_ZC_WORDS", str(1 << 30))
    S, A, H, KG, K, off = 20, 6, 5, 1000, 333, 500
    w = orc.synthetic_weights(S, A, 128, 2, "tanh", False)
    norm = orc.synthetic_normalization(S, A)
    state = orc.synthetic_state(norm)
    low, high = -np.ones(A), np.ones(A)
    eng = RolloutEngine(S, A, 128, 2, "tanh", False, H, K, device=0)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation), norm, 1)
    np.random.seed(77)
    for _ in range(4):           # consecutive control steps: new rows in the same pinned buffer every call
        st0 = np.random.get_state()
        actions = np.random.uniform(low, high, [H, KG, A])[:, off:off + K]
        st_want = np.random.get_state()
        ref = eng.get_action(state, np.ascontiguousarray(actions), cand_offset=off, return_costs=True)
        np.random.set_state(st0)
        res = eng.get_action_numpy_stream(state, low, high, KG, cand_offset=off, return_costs=True)
        st = np.random.get_state()
        assert np.array_equal(res.costs, ref.costs) and res.best_index == ref.best_index
        assert np.array_equal(res.first_action, ref.first_action)
        assert np.array_equal(st[1], st_want[1]) and st[2] == st_want[2]
    eng.close()


@pytest.mark.parametrize("predraw", ["1", "0"])
def test_predraw_sequence_bitexact_with_interleaved_draws(predraw, monkeypatch):
    """The drop-in at train_mpc_ppo.py's K = 400, H = 7 (the zero-copy draw, with the pre-draw worker
    on or off): a sequence of MPCcontroller.get_action calls, some separated by foreign draws from the
    global stream (the worker's rows must then be discarded), each returning the reference's action for
    the array np.random.uniform would return at that point, and leaving NumPy's state exactly where the
    reference leaves it (controllers.py:53, :82-85)."""
    monkeypatch.setenv("BCMPC_MT_PREDRAW", predraw)
    from bc_mpc_amd import MPCcontroller, cheetah_cost_fn
    from oracle import mpc_oracle as orc
    S, A, K, H = 20, 6, 400, 7
    w = orc.synthetic_weights(S, A, 256, 2, "relu", True, seed_base=5)
    norm = orc.synthetic_normalization(S, A)
    dyn = orc.NumpyDynamics(w, norm)

    class Box:
        low, high = -np.ones(A, np.float32), np.ones(A, np.float32)
        shape = (A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (S,)

    ctrl = MPCcontroller(Env(), dyn, horizon=H, cost_fn=cheetah_cost_fn, num_simulated_paths=K)
    np.random.seed(123)
    state = orc.synthetic_state(norm)
    for i in range(8):
        if i in (3, 4, 6):
            np.random.random(1 + i)                     # another consumer of the global stream
        ref = np.random.RandomState()
        ref.set_state(np.random.get_state())
        paths = ref.uniform(Box.low, Box.high, [H, K, A])
        costs, _ = orc.rollout(dyn, state, paths)
        a = ctrl.get_action(state)
        st_got, st_ref = np.random.get_state(), ref.get_state()
        assert st_got[2] == st_ref[2] and np.array_equal(st_got[1], st_ref[1]), f"call {i}: stream position"
        best = int(np.argmin(costs))
        srt = np.sort(costs)
        if srt[1] - srt[0] > 2e-4:
            assert np.array_equal(a, paths[0, best]), f"call {i}"
        state = state + 0.01 * np.sin(np.arange(S) + i)   # the next control step's state


@pytest.mark.parametrize("K,H", [(400, 30), (3000, 8)])
def test_stochastic_policy_dropin_advances_the_stream_only(K, H, monkeypatch):
    """MPCcontrollerPolicyNetReward with self_exp=True (run.sh's recipe) draws the exploration array
    (controllers.py:310-316) but rolls out the policy's own samples (:322-324): the library only advances
    NumPy's state (no rows; pre-computed by the worker).  Same action and same stream position as the
    host path that draws every row (BCMPC_MT_PATH=host), and as np.random.uniform itself."""
    from bc_mpc_amd import MPCcontrollerPolicyNetReward
    from bc_mpc_amd.dynamics import NNDynamicsRewardModel
    from oracle import mpc_oracle as orc
    S, A = 20, 6
    norm = orc.synthetic_normalization(S, A, reward=True)
    w = orc.synthetic_reward_weights(S, A, 500, True, seed_base=9)
    pol = orc.NumpyPolicy(orc.synthetic_policy(S, A, 128, 2))

    class Box:
        low, high = -np.ones(A, np.float32), np.ones(A, np.float32)
        shape = (A,)

    class Env:
        action_space = Box()

        class observation_space:
            shape = (S,)

    state = orc.synthetic_state(norm)
    out = {}
    for path in ("default", "host"):
        if path == "host":
            monkeypatch.setenv("BCMPC_MT_PATH", "host")
        dyn = NNDynamicsRewardModel(Env(), norm, 512, 1, 1e-3, layer_norm=True, size=500, device=0)
        dyn.load_weights(w.kernels, w.biases, w.ln_gamma, w.ln_beta)
        ctrl = MPCcontrollerPolicyNetReward(Env(), dyn, pol, explore=0.5, self_exp=True, horizon=H,
                                            num_simulated_paths=K, seed=5)
        np.random.seed(7)
        acts, states = [], []
        for i in range(3):
            ref = np.random.RandomState()
            ref.set_state(np.random.get_state())
            ref.uniform(Box.low, Box.high, [H, K, A])
            acts.append(ctrl.get_action(state))
            st, want = np.random.get_state(), ref.get_state()
            assert st[2] == want[2] and np.array_equal(st[1], want[1]), f"{path} call {i}: stream position"
            states.append((st[1].copy(), st[2]))
        out[path] = acts
        ctrl._engine.close()
    for a, b in zip(out["default"], out["host"]):
        assert np.array_equal(a, b)


# (2 ms: since round 4 the next job starts when a call launches, so a 300-us hold could finish during the
#  reference call the test makes between two calls and turn a late hit into a plain hit)
@pytest.mark.parametrize("delay_us,expect", [(2000, "late"), (400000, "rerun")])
def test_late_predraw_hit_waits_for_the_rows(delay_us, expect, monkeypatch):
    """Back-to-back NumPy-stream calls on a team-kernel engine (K = 400, H = 7, 2x256 relu + LN) while the
    pre-draw worker is held back (BCMPC_MT_PREDRAW_DELAY_US): each call finds its rows still being drawn
    and launches at once, the kernel waiting for the rows' sequence word (a late hit).  2 ms: every late
    call returns exactly the costs of the same engine on NumPy's own array; 0.4 s (past the kernel's 0.2-s
    wait): the team gives up and the call is rerun on the fallback engine with a fresh draw.  NumPy's
    stream ends where np.random.uniform leaves it either way (controllers.py:53)."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    monkeypatch.setenv("BCMPC_MT_PREDRAW", "1")
    monkeypatch.setenv("BCMPC_MT_PREDRAW_DELAY_US", str(delay_us))
    S, A, H, K = 20, 6, 7, 400
    w = orc.synthetic_weights(S, A, 256, 2, "relu", True)
    norm = orc.synthetic_normalization(S, A)
    state = orc.synthetic_state(norm)
    low, high = -np.ones(A), np.ones(A)
    eng = RolloutEngine(S, A, 256, 2, "relu", True, H, K, device=0)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), norm, 1)
    if eng.info()["kernel"] != "team":
        eng.close()
        pytest.skip("not a team-kernel engine")
    np.random.seed(31)
    calls = 6 if expect == "late" else 2
    for i in range(calls):
        st0 = np.random.get_state()
        actions = np.random.uniform(low, high, [H, K, A])
        st_want = np.random.get_state()
        np.random.set_state(st0)
        res = eng.get_action_numpy_stream(state, low, high, K)          # back to back: the job is in flight
        st = np.random.get_state()
        assert np.array_equal(st[1], st_want[1]) and st[2] == st_want[2], f"call {i}: stream position"
        if expect == "late":
            np.random.set_state(st0)
            ref = eng.get_action(state, np.ascontiguousarray(actions), return_costs=True)
            np.random.set_state(st_want)
            assert res.best_index == ref.best_index and np.array_equal(res.first_action, ref.first_action), f"call {i}"
        else:
            costs, _ = orc.rollout(orc.NumpyDynamics(w, norm), state, actions)
            srt = np.sort(costs)
            assert costs[res.best_index] <= srt[0] + 2e-4, f"call {i}: not a near-optimal row"
            assert np.array_equal(res.first_action, actions[0, res.best_index])
        state = state + 0.01
    stats = eng.predraw_stats()
    print(f"[late predraw] delay {delay_us} us: {stats}, team reruns {eng.team_reruns}")
    if expect == "late":
        assert stats["late"] >= calls - 2
    else:
        assert stats["late"] >= 1 and eng.team_reruns >= 1
    eng.close()


@pytest.mark.parametrize("hidden,L,act,ln,K,H", [(500, 2, "tanh", False, 1000, 15),     # cfg1: team kernel
                                                 (500, 2, "tanh", False, 8192, 10),     # split slab kernel
                                                 (256, 2, "relu", True, 2000, 12)])
def test_speculative_device_draw(hidden, L, act, ln, K, H, monkeypatch):
    """Device-path draws (> 2^16 words): each synchronous call enqueues the NEXT call's draw on the device
    from its own final state, right behind its argmin.  A call whose NumPy state is that start uses the rows
    (a hit); a foreign draw from the global stream in between makes it a miss (fresh draw).  Every call must
    pick exactly the candidate the same engine picks on np.random.uniform's own array and leave NumPy's stream
    where that call leaves it (controllers.py:53, :82-85); two misses in a row pause the speculation."""
    from bc_mpc_amd.engine import MLPSpec, RolloutEngine
    from oracle import mpc_oracle as orc
    monkeypatch.setenv("BCMPC_MT_SPECULATE", "1")
    S, A = 20, 6
    w = orc.synthetic_weights(S, A, hidden, L, act, ln)
    norm = orc.synthetic_normalization(S, A)
    state = orc.synthetic_state(norm)
    low, high = -np.ones(A), np.ones(A)
    eng = RolloutEngine(S, A, hidden, L, act, ln, H, K, device=0)
    eng.set_weights(MLPSpec(w.kernels, w.biases, w.activation, w.ln_gamma, w.ln_beta), norm, 1)
    np.random.seed(11)
    foreign = {3, 6}
    for i in range(8):
        if i in foreign:
            np.random.random(5)                          # another consumer of the global stream
        st0 = np.random.get_state()
        actions = np.random.uniform(low, high, [H, K, A])
        st_want = np.random.get_state()
        ref = eng.get_action(state, np.ascontiguousarray(actions))
        np.random.set_state(st0)
        res = eng.get_action_numpy_stream(state, low, high, K)
        st = np.random.get_state()
        assert np.array_equal(st[1], st_want[1]) and st[2] == st_want[2], f"call {i}: stream position"
        assert res.best_index == ref.best_index and np.array_equal(res.first_action, ref.first_action), f"call {i}"
        assert np.array_equal(res.first_action, actions[0, res.best_index])
        state = state + 0.01
    s1 = eng.predraw_stats()
    # misses in a row: the speculation pauses (no further misses counted while paused)
    for i in range(6):
        np.random.random(3)
        st0 = np.random.get_state()
        actions = np.random.uniform(low, high, [H, K, A])
        st_want = np.random.get_state()
        ref = eng.get_action(state, np.ascontiguousarray(actions))
        np.random.set_state(st0)
        res = eng.get_action_numpy_stream(state, low, high, K)
        st = np.random.get_state()
        assert np.array_equal(st[1], st_want[1]) and st[2] == st_want[2], f"foreign call {i}: stream position"
        assert res.best_index == ref.best_index, f"foreign call {i}"
    s2 = eng.predraw_stats()
    print(f"[speculative draw] {eng.info()['kernel']} K={K} H={H}: after the mixed run {s1}, after the "
          f"foreign run {s2}")
    assert s1["spec_hits"] == 5 and s1["spec_misses"] == 2
    assert s2["spec_misses"] - s1["spec_misses"] == 2 and s2["spec_hits"] == s1["spec_hits"]
    eng.close()
