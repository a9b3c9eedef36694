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
