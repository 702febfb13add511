"""Spectral preprocessing on the GPU.

``snv_savgol(X, window_length, polyorder, deriv, delta, snv=True)`` applies
the drivers' preprocessing as ONE HBM pass per row (``ocm_snv_savgol_f32``):

    SNV (simca_nuts.py:47-49, utils/data_utils.py:57):
        x ← (x − mean_row) / (std_row + 1e-8)      np.std ddof 0, float32 result
    Savitzky–Golay (simca_nuts.py:51, simca_new_cheese.py:37-38):
        scipy.signal.savgol_filter(x, window_length, polyorder, deriv, delta,
                                   axis=1, mode='interp')

``mode='interp'`` is linear in the samples, so it is a set of taps: the
interior correlation coefficients (``savgol_coeffs(..., use='dot')``) and,
for the first / last ``window_length // 2`` outputs, the rows of the map
"least-squares polynomial fit of the first / last window, differentiated
``deriv`` times, evaluated there" (scipy's ``_fit_edge``), built here by
fitting the identity.
"""
from __future__ import annotations

import functools

import numpy as np
import torch
from scipy.signal import savgol_coeffs

from . import _lib, engine
from ._lib import Context, check, ptr
from .prepview import PrepView

__all__ = ["savgol_taps", "snv_savgol", "snv", "savgol_filter", "mahalanobis_outlier_mask", "PrepView"]


@functools.lru_cache(maxsize=64)
def savgol_taps(window_length: int, polyorder: int, deriv: int = 0, delta: float = 1.0) -> np.ndarray:
    """[interior (w)] ++ [left edge (half × w)] ++ [right edge (half × w)] fp64 taps."""
    w = int(window_length)
    if w % 2 != 1 or w < 1:
        raise ValueError("window_length must be a positive odd integer")
    if polyorder >= w:
        raise ValueError("polyorder must be less than window_length.")
    half = w // 2
    interior = savgol_coeffs(w, polyorder, deriv=deriv, delta=delta, use="dot")
    t = np.arange(w, dtype=np.float64)
    # polynomial fit of each unit vector (columns of I), differentiated, evaluated at the edge points
    coeffs = np.polyfit(t, np.eye(w), polyorder)  # (polyorder+1, w)
    for _ in range(deriv):
        coeffs = (coeffs[:-1] * np.arange(coeffs.shape[0] - 1, 0, -1)[:, None]) if coeffs.shape[0] > 1 \
            else np.zeros((1, w))
    ev_left = np.arange(0, half, dtype=np.float64)
    ev_right = np.arange(w - half, w, dtype=np.float64)
    left = np.stack([np.polyval(coeffs, x) for x in ev_left]) / delta ** deriv if half else np.zeros((0, w))
    right = np.stack([np.polyval(coeffs, x) for x in ev_right]) / delta ** deriv if half else np.zeros((0, w))
    return np.ascontiguousarray(np.concatenate([interior, left.ravel(), right.ravel()]), dtype=np.float64)


def snv_savgol(X, window_length: int | None = None, polyorder: int = 2, deriv: int = 0, delta: float = 1.0,
               snv: bool = True, out: torch.Tensor | None = None, lazy: bool = False):
    """SNV (optional) then Savitzky–Golay (optional: ``window_length=None``)
    along the wavelength axis of a (m, p) float32 matrix in HBM.

    ``lazy=True`` returns a ``PrepView``: nothing is computed here (SNV row
    statistics on first use), and ``utils.SIMCA`` fit / predict / transform,
    the CV engine and the engine entry points apply the transform in their
    load paths, so the preprocessed matrix is never written to HBM.

    ``lazy="write"`` returns a write-through ``PrepView``: the first Gram over
    all its rows (a fit) forms X′ in its quantiser and writes it as a side
    output, and every later consumer reads that X′ (the stencil runs once; X′
    costs its memory, as the eager pass does)."""
    Xd = engine.as_device_f32(X)
    if isinstance(Xd, PrepView):
        Xd = Xd.materialize()
    m, p = Xd.shape
    if window_length is not None and int(window_length) > p:
        raise ValueError("If mode is 'interp', window_length must be less than or equal to the size of x.")
    if lazy not in (False, True, "write"):
        raise ValueError('snv_savgol: lazy must be False, True or "write"')
    if lazy:
        if out is not None:
            raise ValueError("snv_savgol: `out` and a lazy view exclude each other")
        tp = savgol_taps(int(window_length), int(polyorder), int(deriv), float(delta)) if window_length else None
        return PrepView(Xd, window_length, polyorder, deriv, delta, snv, tp, through=(lazy == "write"))
    if out is None:
        out = torch.empty((m, p), dtype=torch.float32, device=Xd.device)
    w = 0
    taps = None
    if window_length is not None:
        w = int(window_length)
        tp = savgol_taps(w, int(polyorder), int(deriv), float(delta))
        taps = tp.ctypes.data_as(_lib.ctypes.POINTER(_lib.c_f64))
    check(_lib.load().ocm_snv_savgol_f32(Context.get(Xd.device.index).handle, ptr(Xd), Xd.stride(0), m, p,
                                         1 if snv else 0, w, taps, ptr(out), out.stride(0),
                                         engine._stream(Xd.device)), "ocm_snv_savgol_f32")
    return out


def snv(X, out=None) -> torch.Tensor:
    """(x − mean_row) / (std_row + 1e-8)."""
    return snv_savgol(X, None, snv=True, out=out)


def savgol_filter(X, window_length, polyorder, deriv=0, delta=1.0, out=None) -> torch.Tensor:
    """scipy.signal.savgol_filter(X, ..., axis=1, mode='interp') on the GPU."""
    return snv_savgol(X, window_length, polyorder, deriv, delta, snv=False, out=out)


def mahalanobis_outlier_mask(X, n_components: int, percentile: float = 95.0, rows=None):
    """PCA-score Mahalanobis outlier screen of the drivers (simca_nuts.py:126-147,
    utils/data_utils.py:64-80): scores T of a PCA(n_components) fit, md_i =
    √((t_i − t̄)ᵀ pinv(cov T) (t_i − t̄)), keep md ≤ percentile(md, 95).

    On the engine: the Gram / eigensolver / scoring kernels give T² with
    pinv(cov T) = diag(1/λ) (exact PCA scores are centred and uncorrelated),
    md = √T², and the percentile is the device radix select on md (NumPy's
    linear interpolation in md).  Returns (keep mask bool (n,), threshold)."""
    import torch

    Xd = engine.as_device_f32(X)
    n = Xd.shape[0] if rows is None else int(rows.numel())
    fit = engine.fit_class(Xd, rows, n, int(n_components), theta_mode=0, want_T=False)
    md = torch.sqrt(fit.T2)
    thr = engine.percentile(md, float(percentile))
    return md <= thr, thr
