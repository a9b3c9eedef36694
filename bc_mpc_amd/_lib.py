"""ctypes binding of libbcmpc.so (include/bcmpc.h).

The library is built in-tree (``make`` / ``__graft_entry__.build()``) and is
the only compute path: if it is missing this module raises ImportError --
there is no CPU fallback.

PyTorch-ROCm ships its own ``libamdhip64.so.7`` (same SONAME as
/opt/rocm's).  Importing torch first makes the dynamic linker reuse torch's
HIP runtime for libbcmpc, so device pointers from torch tensors and from the
engine live in ONE runtime.
"""
from __future__ import annotations

import ctypes
import os

try:  # single HIP runtime per process (see module docstring)
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is part of the image
    torch = None

LIB_PATH = os.environ.get("BCMPC_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "libbcmpc.so")

MAX_LAYERS = 8
MAX_STATE = 32
MAX_ACTION = 16
COMM_ID_BYTES = 128
ABI_VERSION = 4

OK, ERR_ARG, ERR_UNSUPPORTED, ERR_HIP, ERR_STATE, ERR_EMPTY = range(6)
ACT_TANH, ACT_RELU = 0, 1
COST_CHEETAH, COST_NONE, COST_REWARD = 0, 1, 2
MODEL_DELTA, MODEL_REWARD = 0, 1
PREC_FP32, PREC_SPLIT_F16, PREC_F16 = 0, 1, 2
# "f16": single-pass f16 MFMA (BASELINE cfg3's bf16-class GEMM), not the fp32 tolerance
PRECISIONS = {"fp32": PREC_FP32, "split": PREC_SPLIT_F16, "f16": PREC_F16}
KERNELS = {"auto": 0, "solo": 1, "group2": 2, "group4": 3, "group8": 4, "split1": 5, "split2": 6, "split4": 7, "splitr": 8, "team": 9}
# ("splitr" and "group2" stay in the enum for the ABI; bcmpc_create refuses them since round 6)


class Config(ctypes.Structure):
    _fields_ = [
        ("state_dim", ctypes.c_int32),
        ("action_dim", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("activation", ctypes.c_int32),
        ("layer_norm", ctypes.c_int32),
        ("horizon", ctypes.c_int32),
        ("cost", ctypes.c_int32),
        ("num_paths", ctypes.c_int64),
        ("precision", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("kernel", ctypes.c_int32),
        ("policy_hidden", ctypes.c_int32),
        ("policy_layers", ctypes.c_int32),
        ("policy_mode", ctypes.c_int32),
        ("model", ctypes.c_int32),
        ("reserved", ctypes.c_int32 * 3),
    ]


_FP = ctypes.POINTER(ctypes.c_float)
_DP = ctypes.POINTER(ctypes.c_double)


class Weights(ctypes.Structure):
    _fields_ = [
        ("kernels", ctypes.POINTER(_FP)),
        ("biases", ctypes.POINTER(_FP)),
        ("ln_gamma", ctypes.POINTER(_FP)),
        ("ln_beta", ctypes.POINTER(_FP)),
        ("mean_obs", _DP),
        ("std_obs", _DP),
        ("mean_action", _DP),
        ("std_action", _DP),
        ("mean_deltas", _DP),
        ("std_deltas", _DP),
        ("mean_reward", _DP),
        ("std_reward", _DP),
    ]


class Policy(ctypes.Structure):
    _fields_ = [
        ("kernels", ctypes.POINTER(_FP)),
        ("biases", ctypes.POINTER(_FP)),
        ("ob_mean", _FP),
        ("ob_std", _FP),
        ("logstd", _FP),
        ("explore", ctypes.c_double),
    ]


POLICY_MODES = {"explore": 0, "stochastic": 1}


class Cem(ctypes.Structure):
    _fields_ = [
        ("iterations", ctypes.c_int32),
        ("n_elite", ctypes.c_int32),
        ("alpha", ctypes.c_double),
        ("k_global", ctypes.c_int64),
    ]


class Elite(ctypes.Structure):
    _fields_ = [("cost", ctypes.c_double), ("index", ctypes.c_int64)]


class Result(ctypes.Structure):
    _fields_ = [
        ("best_index", ctypes.c_int64),
        ("best_cost", ctypes.c_double),
        ("first_action", ctypes.c_double * MAX_ACTION),
    ]


# (name, restype, argtypes) -- every symbol include/bcmpc.h declares
class FitConfig(ctypes.Structure):
    _fields_ = [
        ("state_dim", ctypes.c_int32),
        ("action_dim", ctypes.c_int32),
        ("hidden", ctypes.c_int32),
        ("n_layers", ctypes.c_int32),
        ("activation", ctypes.c_int32),
        ("layer_norm", ctypes.c_int32),
        ("batch_size", ctypes.c_int32),
        ("device", ctypes.c_int32),
        ("learning_rate", ctypes.c_float),
        ("beta1", ctypes.c_float),
        ("beta2", ctypes.c_float),
        ("epsilon", ctypes.c_float),
        ("model", ctypes.c_int32),
    ]


SIGNATURES = [
    ("bcmpc_abi_version", ctypes.c_int, []),
    ("bcmpc_last_error", ctypes.c_char_p, []),
    ("bcmpc_create", ctypes.c_int, [ctypes.POINTER(Config), ctypes.POINTER(ctypes.c_void_p)]),
    ("bcmpc_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("bcmpc_set_weights", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Weights), ctypes.c_uint64]),
    ("bcmpc_weights_version", ctypes.c_uint64, [ctypes.c_void_p]),
    ("bcmpc_predraw_stats", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    ("bcmpc_set_policy", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Policy), ctypes.c_uint64]),
    ("bcmpc_first_actions", ctypes.c_int, [ctypes.c_void_p, _DP]),
    ("bcmpc_set_discount", ctypes.c_int, [ctypes.c_void_p, ctypes.c_double]),
    ("bcmpc_set_action_bounds", ctypes.c_int, [ctypes.c_void_p, _DP, _DP]),
    ("bcmpc_get_action", ctypes.c_int,
     [ctypes.c_void_p, _DP, _DP, ctypes.c_uint64, ctypes.c_int64, ctypes.POINTER(Result), _DP]),
    ("bcmpc_get_action_mt19937", ctypes.c_int,
     [ctypes.c_void_p, _DP, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32), _DP, _DP,
      ctypes.c_int64, ctypes.c_int64, ctypes.c_uint64, ctypes.POINTER(Result), _DP]),
    ("bcmpc_mt19937_uniform", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32), _DP, _DP, ctypes.c_int32, ctypes.c_int64,
      _DP]),
    ("bcmpc_mt19937_uniform_par", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32), _DP, _DP, ctypes.c_int32, ctypes.c_int64,
      ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, _DP, ctypes.c_int32, ctypes.c_int64,
      ctypes.POINTER(ctypes.c_int32)]),
    ("bcmpc_rollout_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("bcmpc_rollout_policy_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int64, ctypes.c_void_p,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("bcmpc_cem_get_action", ctypes.c_int,
     [ctypes.c_void_p, _DP, ctypes.POINTER(Cem), ctypes.c_uint64, _DP, _DP, ctypes.POINTER(Result)]),
    ("bcmpc_cem_rollout_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32,
      ctypes.c_int64, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p]),
    ("bcmpc_select_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("bcmpc_cem_refit_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int32, ctypes.c_double,
      ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]),
    ("bcmpc_stream", ctypes.c_void_p, [ctypes.c_void_p]),
    ("bcmpc_engine_status", ctypes.c_int, [ctypes.c_void_p]),
    ("bcmpc_engine_team_reruns", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint64)]),
    ("bcmpc_select_results_async", ctypes.c_int,
     [ctypes.c_void_p, ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p]),
    ("bcmpc_engine_set_timing", ctypes.c_int, [ctypes.c_void_p, ctypes.c_int32]),
    ("bcmpc_last_kernel_ms", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_float)]),
    ("bcmpc_fit_create", ctypes.c_int, [ctypes.POINTER(FitConfig), ctypes.POINTER(ctypes.c_void_p)]),
    ("bcmpc_fit_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("bcmpc_fit_set_params", ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(Weights)]),
    ("bcmpc_fit_get_params", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(_FP), ctypes.POINTER(_FP), ctypes.POINTER(_FP), ctypes.POINTER(_FP)]),
    ("bcmpc_fit_set_data", ctypes.c_int, [ctypes.c_void_p, _DP, _DP, _DP, ctypes.c_int64]),
    ("bcmpc_fit_run", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int32), ctypes.c_int32, _FP]),
    ("bcmpc_fit_last_error", ctypes.c_char_p, []),
    ("bcmpc_fit_set_rewards", ctypes.c_int, [ctypes.c_void_p, _DP, ctypes.c_int64]),
    ("bcmpc_fit_reward_losses", ctypes.c_int, [ctypes.c_void_p, _FP]),
    ("bcmpc_comm_unique_id", ctypes.c_int, [ctypes.POINTER(ctypes.c_uint8)]),
    ("bcmpc_comm_init", ctypes.c_int,
     [ctypes.POINTER(ctypes.c_uint8), ctypes.c_int32, ctypes.c_int32, ctypes.c_int32, ctypes.POINTER(ctypes.c_void_p)]),
    ("bcmpc_comm_destroy", ctypes.c_int, [ctypes.c_void_p]),
    ("bcmpc_engine_set_comm", ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    ("bcmpc_select_results", ctypes.c_int, [ctypes.POINTER(Result), ctypes.c_int32, ctypes.c_int32,
                                            ctypes.POINTER(Result)]),
    ("bcmpc_mt19937_uniform_device", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_int32), _DP, _DP, ctypes.c_int64,
      ctypes.c_int64, _DP]),
    ("bcmpc_engine_layout", ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.c_int32]),
    ("bcmpc_engine_info", ctypes.c_int,
     [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int64),
      ctypes.POINTER(ctypes.c_int32), ctypes.POINTER(ctypes.c_int32)]),
]

_lib = None


def load() -> ctypes.CDLL:
    """Load libbcmpc.so once; raise ImportError (loudly) when it is absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"libbcmpc.so not found at {LIB_PATH}: build it with `make` or "
            "`python -c 'import __graft_entry__ as g; g.build()'` (no CPU fallback exists)")
    lib = ctypes.CDLL(LIB_PATH)
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.bcmpc_abi_version() != ABI_VERSION:
        raise ImportError(f"libbcmpc ABI {lib.bcmpc_abi_version()} != expected {ABI_VERSION}")
    _lib = lib
    return lib


class BcmpcError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"[bcmpc status {code}] {msg}")
        self.code = code


def check(code: int, fit: bool = False) -> None:
    if code == OK:
        return
    lib = load()
    msg = (lib.bcmpc_fit_last_error() if fit else lib.bcmpc_last_error()).decode(errors="replace")
    if code == ERR_EMPTY:
        raise ValueError(msg)                  # np.argmin on an empty sequence
    if code in (ERR_ARG, ERR_UNSUPPORTED):
        raise ValueError(f"[bcmpc status {code}] {msg}")
    raise BcmpcError(code, msg)
