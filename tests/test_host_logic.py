"""Host-side logic that needs no GPU: sharding, min-loc selection, cost
recognition, weight extraction."""
import numpy as np
import pytest

from bc_mpc_amd import cost_functions as cf
from bc_mpc_amd import distributed as dd
from bc_mpc_amd import weights as ww


@pytest.mark.parametrize("K,world", [(1, 1), (7, 2), (65536, 8), (3, 8), (262144, 8), (1000, 3)])
def test_shard_ranges_partition_k(K, world):
    rngs = [dd.shard_range(K, r, world) for r in range(world)]
    assert rngs[0][0] == 0 and rngs[-1][1] == K
    for (a, b), (c, d) in zip(rngs, rngs[1:]):
        assert b == c and b >= a
    sizes = [b - a for a, b in rngs]
    assert max(sizes) - min(sizes) <= 1


@pytest.mark.parametrize("seed", range(20))
def test_sharded_minloc_equals_np_argmin(seed):
    rs = np.random.RandomState(seed)
    K = int(rs.randint(1, 200))
    costs = np.round(rs.standard_normal(K), 1)          # many exact ties
    if seed % 3 == 0:
        costs[rs.randint(0, K, size=2)] = np.nan
    if seed % 5 == 0:
        costs[:] = 7.0
    world = int(rs.randint(1, 9))
    recs = []
    for r in range(world):
        lo, hi = dd.shard_range(K, r, world)
        if hi == lo:
            recs.append([0.0, np.inf, -1.0])
            continue
        i = int(np.argmin(costs[lo:hi]))
        recs.append([1.0, costs[lo + i], float(lo + i)])
    best = dd.select(np.asarray(recs))
    assert int(best[2]) == int(np.argmin(costs))


def test_cheetah_cost_recognition():
    assert cf.is_cheetah_cost(cf.cheetah_cost_fn)

    def cheetah_cost_fn(state, action, next_state):     # same name, different maths
        return cf.cheetah_cost_fn(state, action, next_state) + 1e-12
    assert not cf.is_cheetah_cost(cheetah_cost_fn)

    def my_cost(state, action, next_state):
        return cf.cheetah_cost_fn(state, action, next_state)
    assert not cf.is_cheetah_cost(my_cost)               # unknown name -> trajectory mode
    assert not cf.is_cheetah_cost(None)


def test_cheetah_cost_recognises_a_faithful_copy():
    # a verbatim-semantics implementation under the reference's function name
    def cheetah_cost_fn(state, action, next_state):
        scores = np.zeros((state.shape[0],))
        scores[state[:, 5] >= 0.2] += 10
        scores[state[:, 6] >= 0] += 10
        scores[state[:, 7] >= 0] += 10
        scores -= (next_state[:, 17] - state[:, 17]) / 0.01
        return scores
    assert cf.is_cheetah_cost(cheetah_cost_fn)


def test_weight_extraction_from_numpy_standin():
    from oracle import mpc_oracle as orc
    w = orc.synthetic_weights(20, 6, 64, 2, "relu", True)
    dyn = orc.NumpyDynamics(w, orc.synthetic_normalization())
    spec, norm, v1 = ww.extract(dyn)
    assert spec.activation == "relu" and spec.layer_norm and spec.n_layers == 2 and spec.hidden == 64
    assert len(norm) == 10 and norm[0].dtype == np.float64
    _, _, v2 = ww.extract(dyn)
    assert v1 == v2
    dyn.weights.kernels[1] = dyn.weights.kernels[1] * 2
    _, _, v3 = ww.extract(dyn)
    assert v3 != v1


def test_tf_fit_hook_bumps_version():
    class Fake:
        def fit(self, data):
            return 1.0, 0
    f = Fake()
    ww._install_fit_hook(f)
    v0 = f._bcmpc_version
    f.fit(None)
    f.fit(None)
    assert f._bcmpc_version == v0 + 2


class _RecordingEngine:
    """RolloutEngine stand-in recording which action source get_action took."""
    calls = []

    def __init__(self, *a, **k):
        self.device = k.get("device", 0)

    def set_action_bounds(self, low, high):
        pass

    def set_weights(self, spec, norm, version):
        pass

    def set_policy(self, spec, explore, version):
        pass

    def set_discount(self, gamma):
        pass

    def numpy_stream_available(self, low, high):
        return True

    def get_action_numpy_stream(self, state, low, high, k_global, cand_offset=0, return_costs=False, seed=0):
        from bc_mpc_amd.engine import StepResult
        _RecordingEngine.calls.append("numpy_stream")
        return StepResult(0, 1.0, np.zeros(6))

    def get_action(self, state, actions, seed=0, cand_offset=0, return_costs=False):
        from bc_mpc_amd.engine import StepResult
        _RecordingEngine.calls.append("host_array")
        return StepResult(0, 1.0, np.zeros(6))

    def close(self):
        pass


class _Box:
    def __init__(self, n, lo, hi):
        self.low, self.high, self.shape = np.full(n, lo, np.float32), np.full(n, hi, np.float32), (n,)


class _Env:
    action_space = _Box(6, -1, 1)
    observation_space = _Box(20, -np.inf, np.inf)


@pytest.mark.parametrize("cls", ["MPCcontroller", "MPCcontrollerPolicyNet", "MPCcontrollerPolicyNetReward"])
def test_stock_samplers_take_the_library_draw(monkeypatch, cls):
    """Every controller whose sample_random_actions is the reference's np.random.uniform body
    (controllers.py:43-55, 181-186, 310-316) -- including the reward subclass, which restates its
    own copy -- draws through the library (get_action_numpy_stream); an instance or subclass
    override of the sampler falls back to the host array."""
    from bc_mpc_amd import controllers as C
    from bc_mpc_amd.cost_functions import cheetah_cost_fn
    from oracle import mpc_oracle as orc
    monkeypatch.setattr(C, "RolloutEngine", _RecordingEngine)
    norm = orc.synthetic_normalization(reward=cls.endswith("Reward"))
    if cls.endswith("Reward"):
        dyn = orc.NumpyRewardDynamics(orc.synthetic_reward_weights(20, 6, 64), norm)
    else:
        dyn = orc.NumpyDynamics(orc.synthetic_weights(20, 6, 64, 2, "tanh", False), norm)
    pol = orc.NumpyPolicy(orc.synthetic_policy())
    make = {"MPCcontroller": lambda: C.MPCcontroller(_Env(), dyn, 3, cheetah_cost_fn, 8),
            "MPCcontrollerPolicyNet": lambda: C.MPCcontrollerPolicyNet(_Env(), dyn, pol, 0.5, False, 3,
                                                                       cheetah_cost_fn, 8),
            "MPCcontrollerPolicyNetReward": lambda: C.MPCcontrollerPolicyNetReward(_Env(), dyn, pol, 0.5, False, 3,
                                                                                   cheetah_cost_fn, 8)}[cls]
    _RecordingEngine.calls = []
    make().get_action(orc.synthetic_state(norm))
    assert _RecordingEngine.calls == ["numpy_stream"]
    # an override is the caller's own sampler: its array is used as is
    ctrl = make()
    ctrl.sample_random_actions = lambda: np.zeros((3, 8, 6))
    _RecordingEngine.calls = []
    ctrl.get_action(orc.synthetic_state(norm))
    assert _RecordingEngine.calls == ["host_array"]


def test_legacy_mt_state_pointers_are_numpys_own_state():
    """bcmpc_get_action_mt19937 advances NumPy's MT19937 state in place through these pointers
    (engine._legacy_mt_state): they must address exactly what get_state() / set_state() see."""
    import ctypes
    from bc_mpc_amd import engine
    np.random.seed(99)
    np.random.random(17)
    mt = engine._legacy_mt_state()
    assert mt is not None
    bg, key_p, pos_p = mt
    st = np.random.get_state()
    key = np.ctypeslib.as_array(key_p, shape=(624,))
    assert np.array_equal(key, st[1]) and pos_p[0] == st[2] == 34      # two words per double
    # an in-place write is NumPy's next state (what the library does after a successful draw)
    want = np.random.RandomState(5).get_state()
    ctypes.memmove(key_p, want[1].ctypes.data, 624 * 4)
    pos_p[0] = want[2]
    assert np.array_equal(np.random.random(4), np.random.RandomState(5).random_sample(4))
    assert engine._legacy_mt_state() is mt                      # cached per generator object


def test_replaced_normalisation_changes_the_engine_version():
    """A normalisation attribute replaced on the model (same weights) gives a new engine version, so the
    engine re-uploads it; the same objects keep the version (weights.extract / weight_token)."""
    from oracle import mpc_oracle as orc
    w = orc.synthetic_weights(20, 6, 64, 2, "relu", True)
    dyn = orc.NumpyDynamics(w, orc.synthetic_normalization())
    _, norm1, v1 = ww.extract(dyn)
    assert ww.extract(dyn)[2] == v1
    dyn.std_obs = np.asarray(dyn.std_obs) * 2.0
    _, norm2, v2 = ww.extract(dyn)
    assert v2 != v1 and np.array_equal(norm2[1], norm1[1] * 2.0)
    assert ww.extract(dyn)[2] == v2

    class Stamped:                                      # a model with its own version stamp (ours / TF hook)
        version = 3

        def mlp_spec(self):
            return None
    m = Stamped()
    for n, a in zip(ww._NORM_ATTRS, orc.synthetic_normalization()):
        setattr(m, n, a)
    t1 = ww.weight_token(m)
    assert ww.same_token(m, t1)
    m.mean_obs = np.array(m.mean_obs)
    assert not ww.same_token(m, t1)
    t2 = ww.weight_token(m)
    m.version = 4
    assert not ww.same_token(m, t2) and ww.same_token(m, ww.weight_token(m))


def test_seed_stream_is_the_one_at_a_time_sequence():
    """The policy controllers' per-call Philox seeds (_SeedStream, drawn 64 at a time) are exactly
    RandomState(seed).randint(0, 2**62) called once per get_action; unread() puts a seed back, and
    get_state / set_state carry the unread seeds."""
    from bc_mpc_amd.controllers import _SeedStream
    ref = np.random.RandomState(0x5EEDF00D)
    want = [int(ref.randint(0, 2**62, dtype=np.int64)) for _ in range(150)]
    s = _SeedStream(0x5EEDF00D)
    got = []
    for i in range(150):
        v = s.next()
        if i % 7 == 3:                      # a call that drew nothing: the host path takes the same seed
            s.unread(v)
            v = s.next()
        got.append(v)
        if i == 70:
            st = s.get_state()
    assert got == want
    t = _SeedStream(1)
    t.set_state(st)
    assert [t.next() for _ in range(79)] == want[71:]


@pytest.mark.parametrize("seed", range(40))
def test_vectorised_select_matches_the_pairwise_order(seed):
    """distributed.select (vectorised) == a left fold of distributed.better over the same records: invalid
    records lose, the first NaN (by index) wins, else the smallest cost, ties to the lower index."""
    rs = np.random.RandomState(seed)
    n = int(rs.randint(1, 12))
    recs = np.zeros((n, 9))
    recs[:, 0] = rs.rand(n) < 0.8
    recs[:, 1] = np.round(rs.standard_normal(n), 0)            # many ties
    recs[:, 2] = rs.permutation(1000)[:n]
    recs[:, 3:] = rs.standard_normal((n, 6))
    if seed % 4 == 0:
        recs[rs.randint(0, n, size=2), 1] = np.nan
    if seed % 7 == 0:
        recs[:, 1] = np.inf
    want = recs[0]
    for r in recs[1:]:
        if dd.better(r, want):
            want = r
    got = dd.select(recs)
    assert np.array_equal(got, want, equal_nan=True)
