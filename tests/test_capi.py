"""C ABI checks that need no GPU: the library loads, exports every symbol the
header declares, and ctypes struct layouts equal the C compiler's."""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from conftest import REPO

HEADER = os.path.join(REPO, "include", "bcmpc.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(bcmpc_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    from bc_mpc_amd import _lib
    lib = _lib.load()
    names = declared_functions()
    assert len(names) >= 12
    for n in names:
        assert hasattr(lib, n), n
    bound = {s[0] for s in _lib.SIGNATURES}
    assert bound == set(names), "ctypes signature table out of sync with include/bcmpc.h"
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for n in names:
        assert re.search(rf"\bT {n}\b", out), n


def test_abi_version_and_error_channel_without_gpu():
    from bc_mpc_amd import _lib
    lib = _lib.load()
    assert lib.bcmpc_abi_version() == _lib.ABI_VERSION
    # argument validation runs before any HIP call
    cfg = _lib.Config(state_dim=20, action_dim=6, hidden=500, n_layers=2, horizon=0, num_paths=16)
    h = ctypes.c_void_p()
    assert lib.bcmpc_create(ctypes.byref(cfg), ctypes.byref(h)) == _lib.ERR_ARG
    assert b"horizon" in lib.bcmpc_last_error()
    cfg.horizon, cfg.hidden = 5, 4096
    assert lib.bcmpc_create(ctypes.byref(cfg), ctypes.byref(h)) == _lib.ERR_UNSUPPORTED
    with pytest.raises(ValueError):
        _lib.check(_lib.ERR_EMPTY)


def test_struct_layouts_match_c():
    from bc_mpc_amd import _lib
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "bcmpc.h"
#define P(T, f) printf(#T "." #f " %zu\n", offsetof(T, f));
int main(void) {
  printf("bcmpc_config %zu\nbcmpc_weights %zu\nbcmpc_result %zu\n",
         sizeof(bcmpc_config), sizeof(bcmpc_weights), sizeof(bcmpc_result));
  P(bcmpc_config, num_paths) P(bcmpc_config, precision) P(bcmpc_config, device) P(bcmpc_config, reserved)
  P(bcmpc_weights, mean_obs) P(bcmpc_weights, std_deltas)
  P(bcmpc_result, best_cost) P(bcmpc_result, first_action)
  return 0; }
'''
    with tempfile.TemporaryDirectory() as d:
        c = os.path.join(d, "t.c")
        exe = os.path.join(d, "t")
        open(c, "w").write(src)
        subprocess.run(["gcc", "-std=c99", "-I", os.path.join(REPO, "include"), c, "-o", exe], check=True)
        lines = subprocess.run([exe], capture_output=True, text=True, check=True).stdout.split("\n")
    got = dict(l.rsplit(" ", 1) for l in lines if l)
    assert int(got["bcmpc_config"]) == ctypes.sizeof(_lib.Config)
    assert int(got["bcmpc_weights"]) == ctypes.sizeof(_lib.Weights)
    assert int(got["bcmpc_result"]) == ctypes.sizeof(_lib.Result)
    for key, v in got.items():
        if "." in key:
            t, f = key.split(".")
            cls = {"bcmpc_config": _lib.Config, "bcmpc_weights": _lib.Weights, "bcmpc_result": _lib.Result}[t]
            assert getattr(cls, f).offset == int(v), key


def _record(index, cost, a0=0.0):
    from bc_mpc_amd import _lib
    r = _lib.Result()
    r.best_index, r.best_cost = index, cost
    r.first_action[0] = a0
    return r


@pytest.mark.parametrize("costs,indices,maximize,want", [
    ([3.5, 1.25, 1.25], [7, 107, 207], False, 107),                  # tie across ranks: lower global index
    ([3.5, 1.25, 1.25], [7, 207, 107], False, 107),                  # (order of the records does not matter)
    ([2.0, float("nan"), float("nan")], [1, 900, 400], False, 400),  # a NaN wins, the first NaN (lowest index)
    ([3.5, 1.25, 9.0], [7, 107, 5], True, 5),                        # np.argmax for the learned reward
    ([-1.0], [42], False, 42),
])
def test_select_results_is_np_argmin_over_ranks(costs, indices, maximize, want):
    """bcmpc_select_results (the host twin of the device selection after the RCCL all-gather,
    csrc/comm.hip): the global np.argmin / np.argmax of the ranks' shard results."""
    import numpy as np
    from bc_mpc_amd import distributed as bd
    recs = [_record(i, c, float(i)) for c, i in zip(costs, indices)]
    cost, index, first = bd.select_results_host(recs, maximize=maximize)
    assert index == want and first[0] == float(want)
    # the same as np.argmin / np.argmax of the concatenated global cost vector
    full = np.full(max(indices) + 1, np.inf if not maximize else -np.inf)
    full[indices] = costs
    assert index == int(np.argmax(full) if maximize else np.argmin(full))


def test_comm_arguments_validated_without_gpu():
    from bc_mpc_amd import _lib
    lib = _lib.load()
    buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
    h = ctypes.c_void_p()
    assert lib.bcmpc_comm_init(buf, 0, 0, 0, ctypes.byref(h)) == _lib.ERR_ARG
    assert lib.bcmpc_comm_init(buf, 2, 2, 0, ctypes.byref(h)) == _lib.ERR_ARG
    assert b"rank" in lib.bcmpc_last_error()
    assert lib.bcmpc_engine_set_comm(None, None) == _lib.ERR_ARG
    assert lib.bcmpc_select_results(None, 0, 0, None) == _lib.ERR_ARG


def test_timing_switch_arguments_validated_without_gpu():
    from bc_mpc_amd import _lib
    lib = _lib.load()
    assert lib.bcmpc_engine_set_timing(None, 1) == _lib.ERR_ARG
    r, m = ctypes.c_float(), ctypes.c_float()
    assert lib.bcmpc_last_kernel_ms(None, ctypes.byref(r), ctypes.byref(m)) == _lib.ERR_ARG


def test_integration_stub_structs_match_the_library():
    """The ctypes stub INTEGRATION.md shows a maintainer (no package import) declares the same struct
    layouts as include/bcmpc.h."""
    from bc_mpc_amd import _lib
    text = open(os.path.join(REPO, "INTEGRATION.md")).read()
    blocks = re.findall(r"```python\n(.*?)```", text, flags=re.S)
    stub = next(b for b in blocks if "class Cfg(ctypes.Structure)" in b)
    defs = stub[stub.index("class Cfg"):stub.index("def make_controller")]
    ns = {"ctypes": ctypes}
    exec(defs, ns)
    assert ctypes.sizeof(ns["Cfg"]) == ctypes.sizeof(_lib.Config)
    assert ctypes.sizeof(ns["W"]) == ctypes.sizeof(_lib.Weights)
    assert ctypes.sizeof(ns["Res"]) == ctypes.sizeof(_lib.Result)
    assert [f[0] for f in ns["W"]._fields_] == [f[0] for f in _lib.Weights._fields_]
    assert [f[0] for f in ns["Cfg"]._fields_] == [f[0] for f in _lib.Config._fields_]
