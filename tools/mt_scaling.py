"""Host-only: scaling of the library's NumPy-stream draw (bcmpc_mt19937_uniform_par) over host threads
at cfg3 size (H=20, K=65536, A=6), plus the CPUs this process may use."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from bc_mpc_amd import _lib
    lib = _lib.load()
    H, K, A = 20, 65536, 6
    buf = np.ones((H * K, A))
    lo, hi = -np.ones(A), np.ones(A)
    dp = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))   # noqa: E731
    np.random.seed(0)
    st = np.random.get_state()
    out = {"affinity_cpus": len(os.sched_getaffinity(0)), "cpu_count": os.cpu_count()}
    for thr in (1, 2, 4, 8, 12, 16):
        key = np.array(st[1], dtype=np.uint32)
        used = ctypes.c_int32(0)
        ts = []
        for _ in range(7):
            pos = ctypes.c_int32(int(st[2]))
            k2 = key.copy()
            t0 = time.perf_counter()
            lib.bcmpc_mt19937_uniform_par(k2.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos),
                                          dp(lo), dp(hi), A, H * K, K, 0, K, dp(buf), thr, 1, ctypes.byref(used))
            ts.append(time.perf_counter() - t0)
        out[f"t{thr}_ms"] = round(float(np.median(ts)) * 1e3, 3)
        out[f"t{thr}_first_ms"] = round(ts[0] * 1e3, 3)
    # one rank's shard at cfg4 (rank 3 of 8: K_global = 262144, 32768 kept per step): the serial path
    # draws every row of every step; the split path jumps over the other ranks' rows
    Kg, Ks, r = 262144, 32768, 3
    sbuf = np.ones((H * Ks, A))
    for name, thr in (("cfg4_rank3_serial_ms", 1), ("cfg4_rank3_split_ms", 0)):
        key = np.array(st[1], dtype=np.uint32)
        used = ctypes.c_int32(0)
        ts = []
        for _ in range(5):
            pos = ctypes.c_int32(int(st[2]))
            k2 = key.copy()
            t0 = time.perf_counter()
            lib.bcmpc_mt19937_uniform_par(k2.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), ctypes.byref(pos),
                                          dp(lo), dp(hi), A, H * Kg, Kg, r * Ks, (r + 1) * Ks, dp(sbuf), thr, -1,
                                          ctypes.byref(used))
            ts.append(time.perf_counter() - t0)
        out[name] = round(float(np.median(ts)) * 1e3, 3)
        out[name.replace("_ms", "_threads")] = used.value
    print(json.dumps(out))


if __name__ == "__main__":
    main()
