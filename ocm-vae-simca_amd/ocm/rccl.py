"""A raw RCCL communicator for collectives captured into HIP graphs.

Why not ``torch.distributed`` for the captured gradient all-reduce
(ocm/vae_train.py, C5): every eager collective that ProcessGroupNCCL issues
becomes a ``WorkNCCL`` on its watchdog thread's list, and the watchdog polls
each one's end event with ``hipEventQuery`` until it has seen it complete.
While ANY stream of the process is capturing, the HIP runtime refuses that
query from the watchdog thread (``hipErrorStreamCaptureUnsupported`` — the
watchdog runs in the default global capture-interaction mode, and a
thread-local capture elsewhere does not change that), and the watchdog
aborts the process (round 4, ``gpurun_out/r04p/tests.log:28-40``: the end
event of a warm-up all-reduce still listed when the step was captured).

So the trainer's collectives — the one-time broadcast of rank 0's state and
the per-step gradient all-reduce — run on a communicator of their own,
created here with ``ncclCommInitRank`` over the ranks of the given process
group (the unique id travels through the group's store, so no collective is
needed to set it up).  Nothing issued on it is tracked by any watchdog, so a
capture can never race a poll of the trainer's own work: by construction, not
by timing.  ``ncclAvg`` does DDP's division by the world size inside the
all-reduce (one kernel fewer per step).

The library is the librccl.so torch itself loaded (torch/lib), so device
pointers, streams and the RCCL version are torch's.
"""
from __future__ import annotations

import ctypes
import os
import pickle
import time

import torch
import torch.distributed as dist

__all__ = ["Communicator", "pending_pg_collectives", "wait_pg_collectives_retired"]

NCCL_UNIQUE_ID_BYTES = 128  # rccl.h:40
_DTYPES = {torch.float32: 7, torch.float64: 8, torch.uint8: 1, torch.int64: 4, torch.bfloat16: 9,
           torch.float16: 6, torch.int32: 2}  # ncclDataType_t, rccl.h:456-470
NCCL_SUM, NCCL_AVG = 0, 4  # ncclRedOp_t, rccl.h:447-452


class _UniqueId(ctypes.Structure):
    _fields_ = [("internal", ctypes.c_char * NCCL_UNIQUE_ID_BYTES)]


_lib = None
_seq: dict = {}


def _load():
    global _lib
    if _lib is None:
        path = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
        if not os.path.exists(path):
            path = "librccl.so"
        lib = ctypes.CDLL(path)
        vp = ctypes.c_void_p
        lib.ncclGetUniqueId.argtypes = [ctypes.POINTER(_UniqueId)]
        lib.ncclCommInitRank.argtypes = [ctypes.POINTER(vp), ctypes.c_int, _UniqueId, ctypes.c_int]
        lib.ncclAllReduce.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp, vp]
        lib.ncclBroadcast.argtypes = [vp, vp, ctypes.c_size_t, ctypes.c_int, ctypes.c_int, vp, vp]
        lib.ncclCommDestroy.argtypes = [vp]
        lib.ncclGetErrorString.argtypes = [ctypes.c_int]
        lib.ncclGetErrorString.restype = ctypes.c_char_p
        for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclAllReduce", "ncclBroadcast", "ncclCommDestroy"):
            getattr(lib, f).restype = ctypes.c_int
        _lib = lib
    return _lib


def _check(rc: int, what: str):
    if rc != 0:
        raise RuntimeError(f"{what}: RCCL error {rc} ({_load().ncclGetErrorString(rc).decode(errors='replace')})")


def _store_of(group):
    """The store the process group rendezvoused through (keys are namespaced
    by the group's global ranks and a per-process sequence number)."""
    from torch.distributed import distributed_c10d as c10d

    return c10d._get_default_store()


class Communicator:
    """An RCCL communicator over the ranks of ``group`` (None: WORLD) on
    ``device``.  Collective calls are stream-ordered on the current stream of
    that device and may be captured into a HIP graph."""

    def __init__(self, group=None, device=None):
        lib = _load()
        self.device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(self.world))
        n = _seq.get(ranks, 0)
        _seq[ranks] = n + 1
        key = "ocm_rccl/" + "_".join(map(str, ranks)) + f"/{n}"
        store = _store_of(group)
        uid = _UniqueId()
        if self.rank == 0:
            _check(lib.ncclGetUniqueId(ctypes.byref(uid)), "ncclGetUniqueId")
            store.set(key, bytes(uid.internal))
        else:
            raw = store.get(key)
            ctypes.memmove(ctypes.addressof(uid), raw, NCCL_UNIQUE_ID_BYTES)
        self._comm = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            _check(lib.ncclCommInitRank(ctypes.byref(self._comm), self.world, uid, self.rank), "ncclCommInitRank")

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @staticmethod
    def _args(t: torch.Tensor):
        if not (t.is_cuda and t.is_contiguous()):
            raise ValueError("RCCL collectives take contiguous device tensors")
        if t.dtype not in _DTYPES:
            raise ValueError(f"unsupported dtype {t.dtype}")
        return ctypes.c_void_p(t.data_ptr()), t.numel(), _DTYPES[t.dtype]

    def all_reduce(self, t: torch.Tensor, average: bool = False):
        """In place: Σ over ranks (or the mean, ``average=True``: ncclAvg)."""
        p, n, dt = self._args(t)
        _check(_load().ncclAllReduce(p, p, n, dt, NCCL_AVG if average else NCCL_SUM, self._comm, self._stream()),
               "ncclAllReduce")

    def broadcast(self, t: torch.Tensor, root: int = 0):
        """In place from group rank ``root``."""
        p, n, dt = self._args(t)
        _check(_load().ncclBroadcast(p, p, n, dt, root, self._comm, self._stream()), "ncclBroadcast")

    def close(self):
        """Destroy the communicator (no graph that captured it may replay after)."""
        if self._comm:
            _check(_load().ncclCommDestroy(self._comm), "ncclCommDestroy")
            self._comm = ctypes.c_void_p()


RECORDER_ENV = ("TORCH_FR_BUFFER_SIZE", "TORCH_NCCL_TRACE_BUFFER_SIZE")  # torch reads the first one set


def recorder_enabled() -> bool:
    """Whether ProcessGroupNCCL keeps a flight recorder (a non-zero buffer
    size, read by torch when the process group starts; ``ocm`` sets one on
    import unless the caller chose a value)."""
    for name in RECORDER_ENV:
        v = os.environ.get(name)
        if v is not None:
            try:
                return int(v) > 0
            except ValueError:
                return False
    return False


def pending_pg_collectives() -> int | None:
    """Eager ProcessGroupNCCL collectives their watchdogs still track (the
    flight recorder's entries the watchdog has not retired yet), or None when
    the recorder is unavailable (disabled, or not in this torch build).  The
    dump is this process's own data."""
    if not recorder_enabled():
        return None
    try:
        from torch._C._distributed_c10d import _dump_nccl_trace
    except ImportError:
        return None
    try:
        raw = _dump_nccl_trace(includeCollectives=True, includeStackTraces=False, onlyActive=True)
    except Exception:  # noqa: BLE001 — no NCCL process group in this process
        return None
    return len(pickle.loads(raw).get("entries", []))


def _nccl_group_exists(group=None) -> bool:
    return (dist.is_available() and dist.is_initialized()
            and "nccl" in str(dist.get_backend(group)).lower())


def wait_pg_collectives_retired(group=None, timeout: float = 30.0) -> int:
    """Block until every eager ProcessGroupNCCL collective issued before has
    been retired by its watchdog (so no watchdog will query an event while a
    graph is being captured); raises after ``timeout`` seconds.  The wait is a
    condition on the watchdogs' own records, not a guess at their poll period.
    Returns the number that was pending.  When an NCCL process group exists but
    its flight recorder is off, nothing tells when the watchdog is done, so
    this raises instead of proceeding."""
    first = pending_pg_collectives()
    if first is None:
        if not _nccl_group_exists(group):
            return 0
        raise RuntimeError("a HIP-graph capture beside a ProcessGroupNCCL needs its flight recorder to know when the "
                           "watchdog has retired the eager collectives (a poll during the capture aborts the process, "
                           "ocm/rccl.py); set TORCH_FR_BUFFER_SIZE (e.g. 2000) before init_process_group — importing "
                           "ocm first does — or pass graph=False")
    if not first:
        return 0
    torch.cuda.synchronize()
    t0 = time.monotonic()
    while True:
        n = pending_pg_collectives()
        if not n:
            return first
        if time.monotonic() - t0 > timeout:
            raise RuntimeError(f"{n} ProcessGroupNCCL collective(s) still tracked by the watchdog after {timeout} s; "
                               "a HIP-graph capture now would abort the process (ocm/rccl.py)")
        time.sleep(0.005)
