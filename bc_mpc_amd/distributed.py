"""Candidate sharding across ranks + the one per-step min-loc exchange.

The K candidates of one control step are independent rollouts of the same
initial state (controllers.py:63-71); the only cross-candidate operation is
``np.argmin`` (controllers.py:82).  With one process per GPU
(torch.distributed, backend "nccl" = RCCL over xGMI), rank r owns the
contiguous global range ``shard_range(K, r, world)`` and after its local
rollout contributes one record ``[valid, cost, index, first_action...]``.

Exchange, RCCL (backend "nccl"): ``LibraryComm`` -- libbcmpc's own communicator
(bcmpc_comm_*, csrc/comm.hip), bootstrapped by broadcasting its 128-byte RCCL id
through torch.distributed once; attached to the engine, every get_action
all-gathers the 144-byte result records on the device right after the argmin
launch and reduces them with np.argmin's rule there (no host round trip, no
torch collective on the control step).  Other backends (gloo, the CPU tests):
a single ``all_gather_into_tensor`` of (3 + A) doubles per rank.
An exact min-loc needs the f64 cost AND the index (np.argmin tie-break:
lowest index; NaN wins) -- 128 bits that do not fit a 64-bit
``all_reduce(MIN)`` key without rounding the cost, so the exchange is an
all-gather of the tiny records (latency-bound, one collective per step) and
every rank applies the same deterministic selection.
"""
from __future__ import annotations

import math
from typing import Optional, Sequence, Tuple

import numpy as np


def world(group=None) -> Tuple[int, int]:
    try:
        import torch.distributed as dist
    except Exception:  # pragma: no cover
        return 0, 1
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(group), dist.get_world_size(group)
    return 0, 1


class LibraryComm:
    """libbcmpc's communicator (bcmpc_comm_init: one RCCL communicator over the group's ranks, on
    this rank's GPU).  Collective: every rank of ``group`` constructs it together; rank 0's RCCL
    unique id travels by ``torch.distributed.broadcast_object_list`` (bootstrap only)."""

    def __init__(self, device: int, group=None):
        import ctypes
        import torch
        import torch.distributed as dist
        from . import _lib
        self._lib = _lib.load()
        self.rank, self.size = world(group)
        self.device = int(device)
        buf = (ctypes.c_uint8 * _lib.COMM_ID_BYTES)()
        if self.rank == 0:
            _lib.check(self._lib.bcmpc_comm_unique_id(buf))
        obj = [bytes(buf)]
        src = 0 if group is None else dist.get_global_rank(group, 0)
        # (the group's own backend carries the id: CUDA tensors under nccl, host tensors under gloo)
        dev = torch.device("cuda", self.device) if dist.get_backend(group) == "nccl" else torch.device("cpu")
        dist.broadcast_object_list(obj, src=src, group=group, device=dev)
        ctypes.memmove(buf, obj[0], _lib.COMM_ID_BYTES)
        h = ctypes.c_void_p()
        _lib.check(self._lib.bcmpc_comm_init(buf, self.size, self.rank, self.device, ctypes.byref(h)))
        self.handle = h

    def close(self) -> None:
        if getattr(self, "handle", None):
            self._lib.bcmpc_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass


def use_library_comm(group=None) -> bool:
    """BCMPC_LIBRARY_COMM=1 (opt-in until a multi-GPU run has exercised it): the library exchanges the
    records itself under RCCL (backend "nccl", csrc/comm.hip); by default the torch all-gather of the
    records (allgather_minloc) carries the one exchange of a control step."""
    import os
    rank, ws = world(group)
    if ws == 1 or os.environ.get("BCMPC_LIBRARY_COMM", "0") != "1":
        return False
    import torch.distributed as dist
    return dist.get_backend(group) == "nccl"


def select_results_host(records, maximize: bool = False) -> Tuple[float, int, np.ndarray]:
    """np.argmin (np.argmax) over bcmpc_result records through the library's own rule
    (bcmpc_select_results, the host twin of the device selection)."""
    import ctypes
    from . import _lib
    lib = _lib.load()
    n = len(records)
    arr = (_lib.Result * n)(*records)
    out = _lib.Result()
    _lib.check(lib.bcmpc_select_results(arr, n, int(bool(maximize)), ctypes.byref(out)))
    return float(out.best_cost), int(out.best_index), np.array(out.first_action[:], dtype=np.float64)


def shard_range(K: int, rank: int, world_size: int) -> Tuple[int, int]:
    """Contiguous global candidate range of ``rank``; the first K % world ranks get one more."""
    base, rem = divmod(int(K), int(world_size))
    lo = rank * base + min(rank, rem)
    return lo, lo + base + (1 if rank < rem else 0)


def better(a: Sequence[float], b: Sequence[float]) -> bool:
    """np.argmin order on records (valid, cost, index): invalid records lose;
    a NaN cost beats every number; smaller cost wins; ties -> lower index."""
    av, bv = a[0] > 0.5, b[0] > 0.5
    if av != bv:
        return av
    if not av:
        return False
    an, bn = math.isnan(a[1]), math.isnan(b[1])
    if an != bn:
        return an
    if not an and a[1] != b[1]:
        return a[1] < b[1]
    return a[2] < b[2]


def select(records: np.ndarray) -> np.ndarray:
    """The winning record under ``better``'s order, vectorised: the first NaN cost by index if any valid record
    has one, else the smallest cost, ties to the lower index; records[0] when none is valid."""
    r = np.asarray(records, dtype=np.float64)
    valid = r[:, 0] > 0.5
    if not valid.any():
        return r[0]
    cost = r[:, 1]
    nan = valid & np.isnan(cost)
    cand = nan if nan.any() else valid & (cost == np.min(cost[valid & ~np.isnan(cost)]))
    rows = np.flatnonzero(cand)
    return r[rows[np.argmin(r[rows, 2])]]


_STAGING = {}


def _staging(backend, dev, n, ws, group):
    """Per (group, device, record size) buffers of the host-staged exchange, kept across control steps:
    under nccl a pinned host record, its device copy, the gathered device records and their pinned host
    copy (so both copies are asynchronous on the device's current stream and one synchronisation ends
    the step); under gloo the host record and the gathered host records."""
    import torch
    key = (id(group), backend, str(dev), n, ws)
    b = _STAGING.get(key)
    if b is None:
        f64 = torch.float64
        if backend == "nccl":
            b = (torch.zeros(n, dtype=f64).pin_memory(), torch.zeros(n, dtype=f64, device=dev),
                 torch.zeros(ws * n, dtype=f64, device=dev), torch.zeros(ws * n, dtype=f64).pin_memory())
        else:
            b = (torch.zeros(n, dtype=f64), None, torch.zeros(ws * n, dtype=f64), None)
        _STAGING[key] = b
    return b


def allgather_minloc(valid: bool, cost: float, index: int, first_action: Optional[np.ndarray],
                     action_dim: int, group=None, device: Optional[int] = None) -> Tuple[float, int, np.ndarray]:
    """One collective per control step; returns the global (cost, index, first_action).
    ``device``: the GPU this rank's engine runs on -- under nccl (RCCL) the record goes through
    that device, so each rank's collective uses its own GPU even when the caller never called
    torch.cuda.set_device (default: torch's current device).  The record's copies go through pinned
    buffers kept per group and device (``_staging``): H2D, the all-gather and the D2H are enqueued
    back to back on that device's current stream, one synchronisation, the selection vectorised on the
    host (the host-staged tail's cost per step)."""
    import torch
    import torch.distributed as dist
    rank, ws = world(group)
    n = 3 + action_dim
    if not (dist.is_available() and dist.is_initialized()):      # (a 1-rank group still gathers: tests)
        fa = np.zeros(action_dim) if first_action is None else np.asarray(first_action, dtype=np.float64).copy()
        return float(cost), int(index), fa
    backend = dist.get_backend(group)
    dev = (torch.device("cuda", torch.cuda.current_device() if device is None else int(device))
           if backend == "nccl" else torch.device("cpu"))
    h_rec, d_rec, out, h_out = _staging(backend, dev, n, ws, group)
    rec = h_rec.numpy()
    rec[0] = 1.0 if valid else 0.0
    rec[1] = cost
    rec[2] = float(index)
    rec[3:] = 0.0 if first_action is None else first_action
    if backend == "nccl":
        with torch.cuda.device(dev):
            stream = torch.cuda.current_stream(dev)
            d_rec.copy_(h_rec, non_blocking=True)
            dist.all_gather_into_tensor(out, d_rec, group=group)
            h_out.copy_(out, non_blocking=True)
            stream.synchronize()
        recs = h_out.numpy().reshape(ws, n)
    else:
        dist.all_gather_into_tensor(out, h_rec, group=group)
        recs = out.numpy().reshape(ws, n)
    best = select(recs)
    if best[0] < 0.5:
        raise ValueError("attempt to get argmin of an empty sequence")
    return float(best[1]), int(best[2]), best[3:].copy()


class RecordExchange:
    """The torch-carried exchange with the selection on the device (the bench's N > 1 default; the
    per-step cost against the host-staged forms: DESIGN.md §7).  Per control step:

    1. this rank's ``bcmpc_result`` (144 bytes) is written into ``d_result`` by the argmin launch;
    2. ONE ``all_gather_into_tensor`` of the records (RCCL over xGMI under nccl; under gloo through
       host memory), stream-ordered after that launch on torch's current stream;
    3. ``bcmpc_select_results_async`` (the library's np.argmin / np.argmax rule, comm.hip) reduces
       the ``world`` records on the same stream;
    4. one D2H of the 144-byte winner into pinned memory, one stream synchronisation.

    No host round trip sits between the argmin and the collective, and the host never walks the
    records.  Every rank must hold >= 1 candidate."""

    def __init__(self, device: int, maximize: bool = False, group=None):
        import torch
        import torch.distributed as dist
        from . import _lib
        self._lib = _lib.load()
        self.rank, self.size = world(group)
        self.group = group
        self.maximize = int(bool(maximize))
        self.device = torch.device("cuda", int(device))
        self.collective = dist.is_available() and dist.is_initialized()   # (a 1-rank group gathers too)
        self.backend = dist.get_backend(group) if self.collective else "none"
        nb = ctypes_sizeof_result()
        self.d_result = torch.zeros(nb, dtype=torch.uint8, device=self.device)
        self.d_all = torch.zeros(max(1, self.size) * nb, dtype=torch.uint8, device=self.device)
        self.d_best = torch.zeros(nb, dtype=torch.uint8, device=self.device)
        self.h_best = torch.zeros(nb, dtype=torch.uint8).pin_memory()
        self._nb = nb

    def exchange(self, stream) -> Tuple[float, int, np.ndarray]:
        """Steps 2-4 on ``stream`` (a torch.cuda.Stream: the one the argmin was launched on)."""
        import ctypes
        import torch
        import torch.distributed as dist
        from . import _lib
        with torch.cuda.stream(stream):
            if self.collective:
                if self.backend == "nccl":
                    dist.all_gather_into_tensor(self.d_all, self.d_result, group=self.group)
                else:                                  # gloo: host tensors
                    out = torch.empty(self.size * self._nb, dtype=torch.uint8)
                    dist.all_gather_into_tensor(out, self.d_result.cpu(), group=self.group)
                    self.d_all.copy_(out)
            else:
                self.d_all.copy_(self.d_result)
            _lib.check(self._lib.bcmpc_select_results_async(
                ctypes.c_void_p(self.d_all.data_ptr()), max(1, self.size), self.maximize,
                ctypes.c_void_p(self.d_best.data_ptr()), ctypes.c_void_p(stream.cuda_stream)))
            self.h_best.copy_(self.d_best, non_blocking=True)
        stream.synchronize()
        raw = self.h_best.numpy()
        index = int(raw[:8].view(np.int64)[0])
        cost = float(raw[8:16].view(np.float64)[0])
        return cost, index, raw[16:].view(np.float64).copy()


def ctypes_sizeof_result() -> int:
    import ctypes
    from . import _lib
    return ctypes.sizeof(_lib.Result)


def allgather_result(d_result, action_dim: int, maximize: bool = False, group=None) -> Tuple[float, int, np.ndarray]:
    """The torch-side form of the exchange (gloo rehearsals; nccl without the library communicator):
    ``d_result`` is this rank's ``bcmpc_result``
    (144 bytes: int64 index, f64 cost, f64 first_action[16]) as a uint8 CUDA tensor, written by
    the argmin launch; the all-gather is stream-ordered after it, so there is no host round trip
    before the collective and one device-to-host copy after it.  Every rank must hold >= 1
    candidate (K > 0).  ``maximize``: learned reward (np.argmax, controllers.py:152).  The records
    are reduced by bcmpc_select_results, the host twin of the library's device selection."""
    import torch
    import torch.distributed as dist
    rank, ws = world(group)
    nb = d_result.numel()
    if ws == 1:
        raw = d_result.cpu().numpy()
    else:
        src = d_result if dist.get_backend(group) == "nccl" else d_result.cpu()   # gloo: host tensors
        out = torch.empty(ws * nb, dtype=torch.uint8, device=src.device)
        dist.all_gather_into_tensor(out, src, group=group)
        raw = out.cpu().numpy()
    raw = raw.reshape(max(ws, 1), nb)
    from . import _lib
    recs = [_lib.Result.from_buffer_copy(raw[r].tobytes()) for r in range(raw.shape[0])]
    cost, index, first = select_results_host(recs, maximize=maximize)   # the library's own rule
    return cost, index, first[:action_dim].copy()
