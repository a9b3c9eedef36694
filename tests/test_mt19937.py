"""The library's MT19937 restatement (csrc/mt19937.cpp, bcmpc_mt19937_uniform) against NumPy's
legacy global generator: np.random.uniform(low, high, [H, K, A]) (controllers.py:53) bit for bit,
and the global stream left exactly where that call leaves it.  Host-only: runs without a GPU."""
import ctypes

import numpy as np
import pytest


def _draw(lib, low, high, n_rows):
    st = np.random.get_state()
    key = np.array(st[1], dtype=np.uint32)
    pos = ctypes.c_int32(int(st[2]))
    out = np.empty((n_rows, len(low)))
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
    assert lib.bcmpc_mt19937_uniform(key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos),
                                     dp(low), dp(high), len(low), n_rows, dp(out)) == 0
    np.random.set_state((st[0], key, pos.value, st[3], st[4]))
    return out


@pytest.mark.parametrize("seed", [0, 7, 2**31 - 1])
@pytest.mark.parametrize("pre_words", [0, 1, 2, 311, 623, 624, 625, 1249])
def test_uniform_matches_numpy_stream(seed, pre_words):
    from bc_mpc_amd import _lib
    lib = _lib.load()
    low = np.array([-1, -0.5, 0, -2, -3, 0.1], np.float32)         # gym Box bounds are float32
    high = np.array([1, 0.5, 2, 2, 3, 0.2], np.float32)
    H, K = 5, 131
    np.random.seed(seed)
    np.random.randint(0, 2**31 - 1, size=pre_words, dtype=np.int64)   # leaves the position anywhere (odd too)
    st = np.random.get_state()
    want = np.random.uniform(low=low, high=high, size=[H, K, 6])
    after = np.random.random(3)
    np.random.set_state(st)
    got = _draw(lib, low.astype(np.float64), high.astype(np.float64), H * K).reshape(H, K, 6)
    assert np.array_equal(got, want)
    assert np.array_equal(np.random.random(3), after)


@pytest.mark.parametrize("A", [1, 3, 5, 8, 11, 16])
@pytest.mark.parametrize("pre_words", [0, 1, 623, 1249])
def test_uniform_any_action_dim(A, pre_words):
    """The one-pass draw (every row kept) for action dims whose bound pattern spans 8..128 doubles."""
    from bc_mpc_amd import _lib
    lib = _lib.load()
    rs = np.random.RandomState(A)
    low = rs.uniform(-3, 0, A).astype(np.float32)
    high = (low + rs.uniform(0.1, 4, A)).astype(np.float32)
    np.random.seed(11)
    np.random.randint(0, 2**31 - 1, size=pre_words, dtype=np.int64)
    st = np.random.get_state()
    want = np.random.uniform(low=low, high=high, size=[7, 97, A])
    after = np.random.random(3)
    np.random.set_state(st)
    got = _draw(lib, low.astype(np.float64), high.astype(np.float64), 7 * 97).reshape(7, 97, A)
    assert np.array_equal(got, want)
    assert np.array_equal(np.random.random(3), after)


def _draw_par(lib, low, high, n_rows, period, keep_lo, keep_hi, threads, min_words):
    st = np.random.get_state()
    key = np.array(st[1], dtype=np.uint32)
    pos = ctypes.c_int32(int(st[2]))
    out = np.empty((n_rows // period * (keep_hi - keep_lo), len(low)))
    used = ctypes.c_int32(0)
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
    assert lib.bcmpc_mt19937_uniform_par(key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos),
                                         dp(low), dp(high), len(low), n_rows, period, keep_lo, keep_hi, dp(out),
                                         threads, min_words, ctypes.byref(used)) == 0
    return out, key, pos.value, used.value


@pytest.mark.parametrize("pre_words", [0, 1, 2, 311, 623, 624, 625, 1249, 5000])
@pytest.mark.parametrize("threads", [2, 3, 8])
@pytest.mark.parametrize("shard", [None, (17, 251), (0, 1), (299, 300)])
def test_threaded_jump_ahead_matches_numpy(pre_words, threads, shard):
    """Jump-ahead split of the draw (csrc/mt_jump.cpp): every thread's slice, the shard selection
    and the final (key, pos) -- the representation np.random.get_state() holds, not only the
    stream -- equal NumPy's one np.random.uniform call."""
    from bc_mpc_amd import _lib
    lib = _lib.load()
    low = np.array([-1, -0.5, 0, -2, -3, 0.1])
    high = np.array([1, 0.5, 2, 2, 3, 0.2])
    H, K = 9, 300
    lo, hi = shard or (0, K)
    np.random.seed(11)
    np.random.randint(0, 2**31 - 1, size=pre_words, dtype=np.int64)
    st = np.random.get_state()
    want = np.random.uniform(low=low, high=high, size=[H, K, 6])
    st_after = np.random.get_state()
    np.random.set_state(st)
    got, key, pos, used = _draw_par(lib, low, high, H * K, K, lo, hi, threads, 1)
    assert used == threads                      # forced split (1 word per thread minimum)
    assert np.array_equal(got.reshape(H, hi - lo, 6), want[:, lo:hi])
    assert np.array_equal(key, st_after[1]) and pos == st_after[2]


def test_threaded_default_threshold_large_draw():
    """A draw of several million words splits under the library's default threshold and still equals
    NumPy's; a small one stays serial."""
    from bc_mpc_amd import _lib
    lib = _lib.load()
    low, high = -np.ones(6), np.ones(6)
    H, K = 6, 65536
    np.random.seed(1234)
    np.random.random(777)
    st = np.random.get_state()
    want = np.random.uniform(low=low, high=high, size=[H, K, 6])
    st_after = np.random.get_state()
    np.random.set_state(st)
    got, key, pos, used = _draw_par(lib, low, high, H * K, K, 0, K, 4, -1)
    assert used == 4
    assert np.array_equal(got.reshape(H, K, 6), want)
    assert np.array_equal(key, st_after[1]) and pos == st_after[2]
    np.random.set_state(st)
    small = np.random.uniform(low=low, high=high, size=[3, 100, 6])
    st_small = np.random.get_state()
    np.random.set_state(st)
    got, key, pos, used = _draw_par(lib, low, high, 3 * 100, 100, 0, 100, 4, -1)
    assert used == 1
    assert np.array_equal(got.reshape(3, 100, 6), small)
    assert np.array_equal(key, st_small[1]) and pos == st_small[2]


def test_shard_draw_jumps_over_other_ranks_rows():
    """A rank's slice of every step at multi-GPU sizes (rank 1 of 4, K_global = 32768, H = 20): the
    threads jump over the other ranks' rows (one jump per run of kept rows) and still land on NumPy's
    values and NumPy's final state."""
    from bc_mpc_amd import _lib
    lib = _lib.load()
    low, high = -np.ones(6), np.ones(6)
    H, Kg, N, r = 20, 32768, 4, 1
    lo, hi = r * Kg // N, (r + 1) * Kg // N
    np.random.seed(4242)
    np.random.random(5)
    st = np.random.get_state()
    want = np.random.uniform(low=low, high=high, size=[H, Kg, 6])[:, lo:hi]
    st_after = np.random.get_state()
    np.random.set_state(st)
    got, key, pos, used = _draw_par(lib, low, high, H * Kg, Kg, lo, hi, 8, 1 << 16)
    assert used == 8
    assert np.array_equal(got.reshape(H, hi - lo, 6), want)
    assert np.array_equal(key, st_after[1]) and pos == st_after[2]
