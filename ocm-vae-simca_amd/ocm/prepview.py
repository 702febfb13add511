"""Lazy preprocessed view of a spectra matrix.

The drivers preprocess right before SIMCA — SNV then Savitzky–Golay
(simca_nuts.py:47-52, utils/data_utils.py:57-61) or Savitzky–Golay alone
(simca_new_cheese.py:37-38).  ``PrepView`` stands for the preprocessed matrix
without computing it: it holds the raw float32 rows in HBM, the filter taps and
(for SNV) the per-row statistics, and every libocm kernel that reads it applies
the transform in its load path (``include/ocm.h`` ``ocm_prep``): the i8×3
quantiser of the Gram, the single-pass scoring kernel, the shift / threshold
samples and the exact outlier fix-up.  The preprocessed matrix is never
written to HBM on those paths.  ``materialize()`` writes it (the same float32
values the fused kernels use).

Write-through views (``through=True``, ``snv_savgol(..., lazy="write")``,
round 5): the Gram of all the view's rows (a fit) runs the stencil in its
quantiser as above and also writes X′ from there
(``ocm_gram_f32_prep_write``); from then on the view IS that tensor to every
consumer (the fit-set and predict scoring read it with the plain single-pass
kernel).  The stencil runs once and the eager pass's separate read of X and
the quantiser's read of X′ become one read: it costs X′'s memory, which the
no-copy view does not.

The view quacks like the (m, p) float32 device tensor it stands for where the
engine looks (``shape``, ``dtype``, ``device``, ``ndim``, ``len``); anything
else (slicing, arithmetic) is done on ``materialize()``.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import Context, check, ptr, stream_handle


class OcmPrep(ctypes.Structure):
    """include/ocm.h ``ocm_prep``."""
    _fields_ = [("window", ctypes.c_int32), ("deriv", ctypes.c_int32), ("snv", ctypes.c_int32),
                ("pad_", ctypes.c_int32), ("taps", ctypes.c_void_p), ("rowstat", ctypes.c_void_p)]


def materialised_count(device: int | None = None) -> int:
    """How many times libocm wrote a lazy view out on a fallback path
    (``ocm_prep_materialised``); the fused paths never do."""
    out = ctypes.c_int64(0)
    check(_lib.load().ocm_prep_materialised(Context.get(device).handle, ctypes.byref(out)), "ocm_prep_materialised")
    return int(out.value)


class PrepView:
    """SNV (optional) then Savitzky–Golay (optional) of the rows of ``X``,
    evaluated lazily inside the kernels that consume it."""

    def __init__(self, X: torch.Tensor, window_length: int | None, polyorder: int, deriv: int, delta: float,
                 snv: bool, taps64=None, through: bool = False):
        if not (isinstance(X, torch.Tensor) and X.is_cuda and X.dtype == torch.float32 and X.dim() == 2):
            raise TypeError("PrepView wraps a 2-D float32 CUDA tensor")
        if X.stride(1) != 1:
            X = X.contiguous()
        self.X = X
        self.window = int(window_length) if window_length is not None else 0
        self.polyorder = int(polyorder)
        self.deriv = int(deriv) if self.window else 0
        self.delta = float(delta)
        self.snv = bool(snv)
        if not self.window and not self.snv:
            raise ValueError("PrepView: nothing to apply (no SNV and no filter)")
        self._taps = (torch.from_numpy(taps64).to(torch.float32).to(X.device)
                      if self.window else None)
        self._rowstat = None
        self.through = bool(through)
        self._xp = None  # X′ once a write-through Gram has formed it

    def written(self) -> torch.Tensor | None:
        """X′ when a write-through Gram has written it (else None)."""
        return self._xp

    def _set_written(self, xp: torch.Tensor):
        self._xp = xp

    # ---- tensor-like surface the engine reads ----
    @property
    def shape(self):
        return self.X.shape

    @property
    def dtype(self):
        return torch.float32

    @property
    def device(self):
        return self.X.device

    @property
    def ndim(self):
        return 2

    @property
    def is_cuda(self):
        return True

    def dim(self):
        return 2

    def size(self, d=None):
        return self.X.shape if d is None else self.X.shape[d]

    def __len__(self):
        return self.X.shape[0]

    def stride(self, d=None):
        return self.X.stride() if d is None else self.X.stride(d)

    def __repr__(self):
        return (f"PrepView(shape={tuple(self.shape)}, snv={self.snv}, window={self.window or None}, "
                f"polyorder={self.polyorder}, deriv={self.deriv}, through={self.through}, "
                f"written={self._xp is not None})")

    # ---- the transform ----
    def rowstat(self) -> torch.Tensor | None:
        """(m_r, s_r) per row (SNV only): one read-only pass over X, computed
        once per view (ocm_prep_rowstats_f32)."""
        if not self.snv:
            return None
        if self._rowstat is None:
            m, p = self.X.shape
            rs = torch.empty((m, 2), dtype=torch.float32, device=self.X.device)
            check(_lib.load().ocm_prep_rowstats_f32(Context.get(self.X.device.index).handle, ptr(self.X),
                                                    self.X.stride(0), m, p, ptr(rs),
                                                    stream_handle(self.X.device)), "ocm_prep_rowstats_f32")
            self._rowstat = rs
        return self._rowstat

    def struct(self) -> OcmPrep:
        rs = self.rowstat()
        return OcmPrep(self.window, self.deriv, 1 if self.snv else 0, 0,
                       self._taps.data_ptr() if self._taps is not None else None,
                       rs.data_ptr() if rs is not None else None)

    def materialize(self, rows: torch.Tensor | None = None) -> torch.Tensor:
        """The preprocessed rows (all, or X[rows]) as a float32 tensor."""
        if self._xp is not None:
            return self._xp if rows is None else self._xp.index_select(0, rows)
        m = self.X.shape[0] if rows is None else int(rows.numel())
        p = self.X.shape[1]
        out = torch.empty((m, p), dtype=torch.float32, device=self.X.device)
        st = self.struct()
        check(_lib.load().ocm_prep_apply_f32(Context.get(self.X.device.index).handle, ptr(self.X), self.X.stride(0),
                                             ptr(rows), m, p, ctypes.byref(st), ptr(out), p,
                                             stream_handle(self.X.device)), "ocm_prep_apply_f32")
        return out

    def __getitem__(self, idx):
        """Row selection (``X[rows]``, ``X[rows, :]``, as the CV refit loop
        does): a view of the selected raw rows (the reference's X[rows] is a
        copy too); anything else indexes the materialised matrix.  A written
        write-through view indexes X′."""
        if self._xp is not None:
            return self._xp[idx]
        if isinstance(idx, tuple):
            if len(idx) == 2 and isinstance(idx[1], slice) and idx[1] == slice(None):
                idx = idx[0]
            else:
                return self.materialize()[idx]
        if isinstance(idx, slice):
            sel = idx
        else:
            sel = torch.as_tensor(idx, device=self.X.device)
            if sel.dtype == torch.bool:
                sel = torch.nonzero(sel).flatten()
            sel = sel.to(torch.int64)
        sub = PrepView.__new__(PrepView)
        sub.__dict__.update(self.__dict__)
        sub.X = self.X[sel]
        if sub.X.dim() != 2:
            raise IndexError("PrepView: select rows (a 2-D view)")
        sub.X = sub.X.contiguous()
        sub._rowstat = self._rowstat[sel].contiguous() if self._rowstat is not None else None
        sub._xp = None
        return sub

    def __array__(self, dtype=None, copy=None):
        a = self.numpy()
        return a if dtype is None else a.astype(dtype)

    def cpu(self):
        return self.materialize().cpu()

    def numpy(self):
        return self.materialize().cpu().numpy()
