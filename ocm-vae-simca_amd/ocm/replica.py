"""When the reference entry points may run collectively.

An unchanged driver under ``torchrun`` (``simca_nuts.py:186-189``,
``utils/CVSIMCA.py:103-269``) calls ``SIMCA.fit`` / ``predict`` /
``cross_validate_simca_grid`` on every rank with the SAME full X and y: the
rows can then be split over the ranks (each rank fits / scores its contiguous
block, one all-reduce) and every rank still returns the single-process
result.  A DDP driver whose ranks hold DIFFERENT data (per-rank latents,
per-rank folds) calling the same entry points must get the reference's
per-process behaviour instead.  Which of the two is the case is not visible
from an initialised process group alone, so the drop-ins exchange a cheap
fingerprint of their arguments first (``replicated_group``): the row count,
the width, the element type, a hash of the labels and a hash of a fixed
sample of rows.  Every rank receives every rank's fingerprint, so every rank
takes the same decision and no collective that follows can mismatch.

The exchange is itself a collective: under a process group of more than one
rank every rank must call the drop-in, as an unchanged driver does.  Code
that calls a drop-in on a subset of the ranks (rank-0 evaluation) wraps the
call in ``with ocm.replica.per_process():`` — no collective, the reference's
single-process behaviour.
"""
from __future__ import annotations

import contextlib
import threading

import numpy as np
import torch
import torch.distributed as dist

__all__ = ["replicated_group", "per_process", "fingerprint", "gather_rows"]

SAMPLE_ROWS = 256  # rows hashed per call (≤ 2 MiB at p = 2048)
_FIELDS = 7

_state = threading.local()


@contextlib.contextmanager
def per_process():
    """Within this block the drop-ins never run collectively (no fingerprint
    exchange, no sharding): for calls made on a subset of the ranks."""
    prev = getattr(_state, "off", False)
    _state.off = True
    try:
        yield
    finally:
        _state.off = prev


def _world() -> int:
    if getattr(_state, "off", False) or not (dist.is_available() and dist.is_initialized()):
        return 1
    return dist.get_world_size()


def _hash(b: bytes) -> int:
    try:
        import xxhash

        h = xxhash.xxh3_64_intdigest(b)
    except ImportError:  # pragma: no cover - the image ships xxhash
        import hashlib

        h = int.from_bytes(hashlib.blake2b(b, digest_size=8).digest(), "little")
    return h & 0x7FFFFFFFFFFFFFFF


def _array_hash(a: np.ndarray) -> int:
    if a.dtype == object:
        a = a.astype(str)
    a = np.ascontiguousarray(a)
    return _hash(f"{a.dtype.str}{a.shape}".encode() + a.tobytes())


def _labels_hash(y) -> int:
    if y is None:
        return 0
    if isinstance(y, torch.Tensor):
        y = y.detach().cpu().numpy()
    return _array_hash(np.asarray(y))


def _rows_hash(X, n: int) -> tuple[int, int]:
    """(type code, hash of SAMPLE_ROWS evenly spaced rows).  A lazy
    preprocessing view hashes its raw rows and its transform parameters."""
    from .prepview import PrepView

    extra = b""
    if isinstance(X, PrepView):
        extra = repr((X.window, X.polyorder, X.deriv, X.delta, X.snv, X.through)).encode()
        src = X.written() if X.written() is not None else X.X
        code = 3
    else:
        src = X
        code = None
    idx = np.unique(np.linspace(0, max(n - 1, 0), min(n, SAMPLE_ROWS)).astype(np.int64)) if n > 0 else \
        np.zeros(0, np.int64)
    if isinstance(src, torch.Tensor):
        sample = src.index_select(0, torch.from_numpy(idx).to(src.device)).detach().cpu().numpy()
        dt = src.dtype
        if code is None:
            code = 2 if dt == torch.float64 else 1
    else:
        a = np.asarray(src)
        sample = a[idx]
        if code is None:
            code = 2 if a.dtype == np.float64 else 1
    return code, _hash(extra + np.ascontiguousarray(sample).tobytes() + idx.tobytes())


def fingerprint(X, y=None, eligible: bool = True) -> np.ndarray:
    """[eligible, n, p, type code, hash of y, hash of sampled rows, y length]
    as int64 (the vector every rank all-gathers)."""
    n = int(X.shape[0])
    p = int(X.shape[1]) if len(X.shape) > 1 else 1
    code, xh = _rows_hash(X, n)
    ylen = -1 if y is None else int(len(y))
    return np.array([1 if eligible else 0, n, p, code, _labels_hash(y), xh, ylen], dtype=np.int64)


def _exchange(fp: np.ndarray, group=None) -> np.ndarray:
    """(world, _FIELDS) matrix of every rank's fingerprint."""
    W = dist.get_world_size(group)
    on_dev = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_dev else torch.device("cpu")
    mine = torch.from_numpy(fp).to(dev)
    parts = [torch.empty_like(mine) for _ in range(W)]
    dist.all_gather(parts, mine, group=group)
    return torch.stack(parts).cpu().numpy()


def replicated_group(X, y=None, eligible: bool = True):
    """``dist.group.WORLD`` when a process group of more than one rank is
    initialised, collectives are not switched off (``per_process``), and every
    rank passed the same (X, y) and is ``eligible``; otherwise None.  Under a
    group of > 1 ranks every rank must call it (it all-gathers the
    fingerprints), whatever its arguments."""
    if _world() < 2:
        return None
    fps = _exchange(fingerprint(X, y, eligible))
    if not fps[:, 0].all() or not (fps == fps[0]).all():
        return None
    return dist.group.WORLD


def gather_rows(t: torch.Tensor, counts, group=None) -> torch.Tensor:
    """Concatenate every rank's row block (rank r holds ``counts[r]`` rows of
    ``t``'s trailing shape) in rank order, on every rank: one all-gather of
    blocks padded to the largest."""
    W = dist.get_world_size(group)
    width = max(int(c) for c in counts)
    pad = torch.zeros((width,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
    if t.shape[0]:
        pad[: t.shape[0]] = t
    parts = [torch.empty_like(pad) for _ in range(W)]
    dist.all_gather(parts, pad, group=group)
    return torch.cat([part[: int(c)] for part, c in zip(parts, counts)])
