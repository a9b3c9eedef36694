timeout -k 10 120 python tools/mt_scaling.py && BCMPC_MT_DEBUG=1 timeout -k 10 60 python - <<'PY'
import sys, os; sys.path.insert(0, os.getcwd())
import ctypes, numpy as np, time
from bc_mpc_amd import _lib
lib=_lib.load()
H,K,A=20,65536,6
buf=np.ones((H*K,A)); lo,hi=-np.ones(A),np.ones(A)
dp=lambda a:a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))
np.random.seed(0); st=np.random.get_state()
for thr in (2,2,8,8):
    key=np.array(st[1],dtype=np.uint32); pos=ctypes.c_int32(int(st[2])); used=ctypes.c_int32()
    t0=time.perf_counter()
    lib.bcmpc_mt19937_uniform_par(key.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),ctypes.byref(pos),dp(lo),dp(hi),A,H*K,K,0,K,dp(buf),thr,1,ctypes.byref(used))
    print(thr, (time.perf_counter()-t0)*1e3, flush=True)
PY
