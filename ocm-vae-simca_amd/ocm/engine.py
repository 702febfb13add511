"""Device-side SIMCA engine: the hot path of SURVEY.md §8(a) on libocm.

``fit_class`` = utils/SIMCA.py:62-99 (``_fit_one_class``) and
``score_class`` = :120-145 (``predict`` for one class), re-planned for one
MI355X:

    shift  = mean of ≤4096 sample rows        ocm_colmean_f32   (tiny)
    G, s   = Σ (x-shift)(x-shift)ᵀ, Σ (x-shift) ocm_gram_f32      (FP32 MFMA, 1 HBM pass)
    C, μ   = (G - n d dᵀ)/(n-1), shift + d      ocm_cov_from_gram
    λ, P, θ = top-k eigenpairs, tail moments   ocm_eig_topk      (fp64, HBM-resident C)
    T, T², Q (+ moments, fused decision)        ocm_score_f32     (FP32 MFMA projection, 2 register-streamed sweeps)
    limits                                      host fp64 scalars (ocm/limits.py)

All arrays stay in HBM; only scalars cross to the host.  The second,
randomized ``PCA(k)`` the reference fits for predict (utils/SIMCA.py:75) is
not repeated: it estimates the same leading subspace the eigensolver already
returns exactly (SURVEY.md §8c caveat 1).
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field

import numpy as np
import torch

from . import _lib
from ._lib import Context, OcmDecision, TYPE_CODES, check, ptr, stream_handle
from .prepview import PrepView

SHIFT_SAMPLE = 4096
EIG_TOL = 1e-10
EIG_MAX_ITER = 3000


def require_device():
    if not torch.cuda.is_available():
        raise _lib.OcmError("no HIP device visible: the SIMCA engine runs on MI355X (gfx950) only")


def as_device_f32(X, device=None) -> torch.Tensor:
    """Host NumPy / torch input -> contiguous float32 tensor in HBM (a lazy
    ``PrepView`` passes through: the kernels read it in place)."""
    require_device()
    if isinstance(X, PrepView):
        return X
    if isinstance(X, torch.Tensor):
        t = X
        if device is None and t.is_cuda:
            device = t.device
    else:
        t = torch.from_numpy(np.ascontiguousarray(X))
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    t = t.to(device=device, dtype=torch.float32, non_blocking=False)
    if not t.is_contiguous():
        t = t.contiguous()
    return t


def as_device_x(X, device=None) -> torch.Tensor:
    """Spectra in HBM in the arithmetic the reference would use: float64 input
    stays float64 (sklearn's PCA follows the input dtype, utils/SIMCA.py:64-66),
    anything else becomes float32."""
    if isinstance(X, PrepView):
        return X
    f64 = (X.dtype == torch.float64) if isinstance(X, torch.Tensor) else (np.asarray(X).dtype == np.float64)
    if not f64:
        return as_device_f32(X, device)
    require_device()
    t = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X))
    if device is None:
        device = t.device if t.is_cuda else torch.device("cuda", torch.cuda.current_device())
    t = t.to(device=device, dtype=torch.float64)
    return t if t.is_contiguous() else t.contiguous()


@dataclass
class ClassFit:
    """Per-class model state (device tensors + host scalars)."""
    k: int
    n: int
    p: int
    mean64: torch.Tensor
    evals: torch.Tensor          # (k,) f64
    P64: torch.Tensor            # (k, p) f64, svd_flip sign convention (scoring operand)
    invcov: torch.Tensor | None = None  # (k, k) f64 = pinv(cov(T)) = diag(1/λ); built on first use (invcov_mat)
    inv_diag: torch.Tensor = None  # (k,) f64: its diagonal (the scoring kernels' operand)
    thetas: tuple = (0.0, 0.0, 0.0)
    evals_host: np.ndarray = None
    T: torch.Tensor | None = None
    T2: torch.Tensor | None = None
    Q: torch.Tensor | None = None
    stats_dev: torch.Tensor | None = None  # (4,) f64 on the device: ΣT², Σ(T²)², ΣQ, ΣQ² (all ranks)
    eig_iters: int = 0
    C: torch.Tensor | None = None
    extra: dict = field(default_factory=dict)

    def invcov_mat(self) -> torch.Tensor:
        if self.invcov is None:
            self.invcov = torch.diag(self.inv_diag)
        return self.invcov

    def _stats(self) -> np.ndarray:
        # read on first use only: nothing on the Fdist / jm path waits for the
        # fit-set scoring kernel (its launch returns at once)
        if "stats_host" not in self.extra:
            self.extra["stats_host"] = (self.stats_dev.cpu().numpy() if self.stats_dev is not None
                                        else np.zeros(4))
        return self.extra["stats_host"]

    @property
    def T2_stats(self) -> tuple:
        s = self._stats()
        return (float(s[0]), float(s[1]))

    @property
    def Q_stats(self) -> tuple:
        s = self._stats()
        return (float(s[2]), float(s[3]))


def _stream(dev):
    return stream_handle(dev)


def _plain(X):
    """A write-through view that has been written is its X′ tensor."""
    if isinstance(X, PrepView) and X.written() is not None:
        return X.written()
    return X


def colmean(X: torch.Tensor, rows: torch.Tensor | None, n: int) -> torch.Tensor:
    X = _plain(X)
    ctx = Context.get(X.device.index)
    out = torch.empty(X.shape[1], dtype=torch.float64, device=X.device)
    if isinstance(X, PrepView):
        st = X.struct()
        check(_lib.load().ocm_colmean_f32_prep(ctx.handle, ptr(X.X), X.X.stride(0), ptr(rows), n, X.shape[1],
                                               ctypes.byref(st), ptr(out), _stream(X.device)), "ocm_colmean_f32_prep")
        return out
    fn = "ocm_colmean_f64" if X.dtype == torch.float64 else "ocm_colmean_f32"
    check(getattr(_lib.load(), fn)(ctx.handle, ptr(X), X.stride(0), ptr(rows), n, X.shape[1], ptr(out),
                                   _stream(X.device)), fn)
    return out


def cast_f32(a: torch.Tensor) -> torch.Tensor:
    ctx = Context.get(a.device.index)
    out = torch.empty(a.shape, dtype=torch.float32, device=a.device)
    check(_lib.load().ocm_cast_f64_f32(ctx.handle, ptr(a), a.numel(), ptr(out), _stream(a.device)),
          "ocm_cast_f64_f32")
    return out


GRAM_MODES = {"i8x3": 0, "f32": 1, "bf16x3": 2, "i8x3k32": 3}  # include/ocm.h OCM_GRAM_*
_gram_mode = "i8x3"


def set_gram_mode(name: str) -> str:
    """Process-wide Gram arithmetic for fits ("i8x3" default, "f32", "bf16x3");
    returns the previous mode.  An explicit API choice (ocm_gram_f32_ex), not
    an environment switch inside the library."""
    global _gram_mode
    if name not in GRAM_MODES:
        raise ValueError(f"gram mode must be one of {sorted(GRAM_MODES)}")
    prev, _gram_mode = _gram_mode, name
    return prev


def gram(X: torch.Tensor, rows: torch.Tensor | None, seg_offsets, shift32: torch.Tensor, mode: str | None = None,
         chunk_rows: int = 0):
    """Per-segment shifted Gram (nseg, p, p) f64 and column sums (nseg, p).
    float64 X takes the fp64-MFMA Gram (``mode`` does not apply)."""
    X = _plain(X)
    p = X.shape[1]
    seg = [int(s) for s in seg_offsets]
    nseg = len(seg) - 1
    n = seg[-1]
    G = torch.empty((nseg, p, p), dtype=torch.float64, device=X.device)
    cs = torch.empty((nseg, p), dtype=torch.float64, device=X.device)
    arr = (ctypes.c_int64 * len(seg))(*seg)
    ctx = Context.get(X.device.index)
    if (isinstance(X, PrepView) and X.through and rows is None and n == X.shape[0]
            and (mode or _gram_mode) == "i8x3"):
        # write-through: the quantiser also writes X′, which later consumers read
        st = X.struct()
        xp = torch.empty(X.shape, dtype=torch.float32, device=X.device)
        check(_lib.load().ocm_gram_f32_prep_write(ctx.handle, ptr(X.X), X.X.stride(0), n, p, ptr(shift32), arr, nseg,
                                                  int(chunk_rows), ctypes.byref(st), ptr(G), ptr(cs), ptr(xp),
                                                  xp.stride(0), _stream(X.device)), "ocm_gram_f32_prep_write")
        X._set_written(xp)
        return G, cs
    if isinstance(X, PrepView):  # the preprocessing runs in the quantiser's load path
        st = X.struct()
        check(_lib.load().ocm_gram_f32_prep(ctx.handle, ptr(X.X), X.X.stride(0), ptr(rows), n, p, ptr(shift32), arr,
                                            nseg, GRAM_MODES[mode or _gram_mode], int(chunk_rows), ctypes.byref(st),
                                            ptr(G), ptr(cs), _stream(X.device)), "ocm_gram_f32_prep")
        return G, cs
    if X.dtype == torch.float64:
        check(_lib.load().ocm_gram_f64(ctx.handle, ptr(X), X.stride(0), ptr(rows), n, p, ptr(shift32), arr, nseg,
                                       ptr(G), ptr(cs), _stream(X.device)), "ocm_gram_f64")
        return G, cs
    code = GRAM_MODES[mode or _gram_mode]
    check(_lib.load().ocm_gram_f32_ex(ctx.handle, ptr(X), X.stride(0), ptr(rows), n, p, ptr(shift32), arr, nseg,
                                      code, int(chunk_rows), ptr(G), ptr(cs), _stream(X.device)), "ocm_gram_f32_ex")
    return G, cs


def last_gram_marks(device_index: int) -> int:
    """(row, column-group) values the i8×3 outlier guard screened out in the
    last Gram on this device (0 on clean data)."""
    out = ctypes.c_int64(0)
    check(_lib.load().ocm_gram_last_marks(Context.get(device_index).handle, ctypes.byref(out)), "ocm_gram_last_marks")
    return int(out.value)


def cov_from_gram(terms, shift32: torch.Tensor, n: int):
    """terms: list of (coef, G (p,p), colsum (p,)) -> (C (p,p) f64, mean (p,) f64)."""
    p = shift32.shape[0]
    dev = shift32.device
    C = torch.empty((p, p), dtype=torch.float64, device=dev)
    mean = torch.empty(p, dtype=torch.float64, device=dev)
    nt = len(terms)
    Gp = (ctypes.c_void_p * nt)(*[t[1].data_ptr() for t in terms])
    Sp = (ctypes.c_void_p * nt)(*[t[2].data_ptr() for t in terms])
    cf = (ctypes.c_double * nt)(*[float(t[0]) for t in terms])
    ctx = Context.get(dev.index)
    check(_lib.load().ocm_cov_from_gram(ctx.handle, Gp, Sp, cf, nt, ptr(shift32), n, p, ptr(C), ptr(mean),
                                        _stream(dev)), "ocm_cov_from_gram")
    return C, mean


def eigh_dense(C: torch.Tensor, k: int = 0):
    """Every eigenvalue of the symmetric fp64 C (descending) and, for k > 0,
    the leading k eigenvectors as rows with the svd_flip sign
    (ocm_eigh_f64: Householder tridiagonalisation on the GPU)."""
    p = C.shape[0]
    dev = C.device
    evals = torch.empty(p, dtype=torch.float64, device=dev)
    evecs = torch.empty((k, p), dtype=torch.float64, device=dev) if k > 0 else None
    check(_lib.load().ocm_eigh_f64(Context.get(dev.index).handle, ptr(C.contiguous()), p, ptr(evals), int(k),
                                   ptr(evecs), _stream(dev)), "ocm_eigh_f64")
    return evals, evecs


def eig_topk(C: torch.Tensor, k: int, theta_mode: int, tol=EIG_TOL, max_iter=EIG_MAX_ITER, theta3_slice=(0, 1),
             dense_fallback=True, inv_out: torch.Tensor | None = None, rcond=1e-15):
    """Top-k eigenpairs + tail moments of C (ocm_eig_topk_ex).  When the Ritz
    residuals miss ``tol`` within ``max_iter`` iterations (no usable spectral
    gap after component k: a flat noise floor), the loadings of the
    unconverged subspace are never handed on: the dense solver
    (``eigh_dense``) gives the exact top-k and θ_m = Σ_{i>k} λ_iᵐ, as the
    reference's full SVD would (utils/SIMCA.py:64-66, 189-191), with a
    warning; ``dense_fallback=False`` raises ``OcmNotConverged`` instead.
    ``theta3_slice = (s, S)``: this call's share of the θ3 trace work (the
    ranks of a sharded fit sum the partials).  ``inv_out`` (k,): also 1/λ
    with pinv's cutoff (``inv_evals``), queued inside the call
    (ocm_eig_topk_ex2)."""
    p = C.shape[0]
    dev = C.device
    evals = torch.empty(k, dtype=torch.float64, device=dev)
    evecs = torch.empty((k, p), dtype=torch.float64, device=dev)
    theta = torch.zeros(3, dtype=torch.float64, device=dev)
    iters = ctypes.c_int32(0)
    ctx = Context.get(dev.index)
    if inv_out is not None:
        rc = _lib.load().ocm_eig_topk_ex2(ctx.handle, ptr(C), p, k, tol, max_iter, theta_mode, int(theta3_slice[0]),
                                          int(theta3_slice[1]), ptr(evals), ptr(evecs), ptr(theta),
                                          ctypes.byref(iters), float(rcond), ptr(inv_out), _stream(dev))
    else:
        rc = _lib.load().ocm_eig_topk_ex(ctx.handle, ptr(C), p, k, tol, max_iter, theta_mode, int(theta3_slice[0]),
                                         int(theta3_slice[1]), ptr(evals), ptr(evecs), ptr(theta),
                                         ctypes.byref(iters), _stream(dev))
    if rc == _lib.OCM_ERR_NOCONV:
        msg = (f"ocm_eig_topk: the leading {k} eigenpairs of the {p}x{p} covariance did not converge to tol={tol} "
               f"in {max_iter} iterations (no usable spectral gap after component {k})")
        if not dense_fallback:
            raise _lib.OcmNotConverged(msg + "; pick n_components at a gap in the spectrum")
        import warnings

        warnings.warn(msg + "; using the dense eigensolver (ocm_eigh_f64)", RuntimeWarning, stacklevel=2)
        lam, vec = eigh_dense(C, k)
        tail = lam[k:]
        th = torch.zeros(3, dtype=torch.float64, device=dev)
        if theta_mode >= 1:
            th[0] = tail.sum()
            th[1] = (tail * tail).sum()
        if theta_mode >= 2 and theta3_slice[0] == 0:  # the whole θ3 on slice 0 (the ranks sum the slices)
            th[2] = (tail * tail * tail).sum()
        top = lam[:k].clone()
        if inv_out is not None:
            inv_evals(top, rcond, out=inv_out)
        return top, vec, th, int(max_iter)
    check(rc, "ocm_eig_topk_ex")
    return evals, evecs, theta, int(iters.value)


def sym_pinv(A: torch.Tensor, rcond=1e-15) -> torch.Tensor:
    d = A.shape[0]
    out = torch.empty_like(A)
    ctx = Context.get(A.device.index)
    check(_lib.load().ocm_sym_pinv_f64(ctx.handle, ptr(A.contiguous()), d, rcond, ptr(out), _stream(A.device)),
          "ocm_sym_pinv_f64")
    return out


def make_decision(type_name: str, t2_scale: float, q_scale: float, dlim: float) -> OcmDecision:
    return OcmDecision(TYPE_CODES[type_name], 0, float(t2_scale), float(q_scale), float(dlim))


def score_outputs(X, m: int, k: int, want_T=False, want_T2=True, want_Q=True, want_stats=False) -> dict:
    """The device tensors ``score`` writes (T and Q in the input dtype,
    utils/SIMCA.py:65-71); allocated ahead when the launch is latency-critical."""
    dev = X.device
    vdt = torch.float64 if X.dtype == torch.float64 else torch.float32
    return {"T": torch.empty((m, k), dtype=vdt, device=dev) if want_T else None,
            "T2": torch.empty(m, dtype=torch.float64, device=dev) if want_T2 else None,
            "Q": torch.empty(m, dtype=vdt, device=dev) if want_Q else None,
            "stats": torch.empty(4, dtype=torch.float64, device=dev) if want_stats else None}


def score(X: torch.Tensor, rows: torch.Tensor | None, m: int, P64: torch.Tensor, mean64: torch.Tensor,
          A: torch.Tensor, want_T=False, want_T2=True, want_Q=True, decision: OcmDecision | None = None,
          accept_out: torch.Tensor | None = None, accept_stride: int = 1, want_stats=False, outs=None):
    """Fused scoring: P64 (k, p) f64 orthonormal rows, mean64 (p,) f64, A the
    (k, k) quadratic form (ocm_score_f32) or its diagonal (k,) (ocm_score_f32_diag,
    the single-HBM-pass kernel for the SIMCA shapes).  Returns dict of device tensors.
    ``outs``: the outputs allocated beforehand (``score_outputs``)."""
    X = _plain(X)
    k, p = P64.shape
    dev = X.device
    out = {}
    if isinstance(X, PrepView) and A.dim() != 1:  # a general quadratic form: score the materialised rows
        X, rows = X.materialize(rows), None
    f64 = X.dtype == torch.float64
    if f64 and A.dim() != 1:
        raise ValueError("float64 spectra are scored with a diagonal quadratic form (ocm_score_f64_diag)")
    if outs is None:
        outs = score_outputs(X, m, k, want_T, want_T2, want_Q, want_stats)
    T, T2, Q, st = outs["T"], outs["T2"], outs["Q"], outs["stats"]
    ctx = Context.get(dev.index)
    dec_p = ctypes.byref(decision) if decision is not None else None
    if isinstance(X, PrepView):  # the preprocessing runs on each row tile in registers
        prep = X.struct()
        check(_lib.load().ocm_score_f32_diag_prep(ctx.handle, ptr(X.X), X.X.stride(0), ptr(rows), m, p,
                                                  ctypes.byref(prep), ptr(P64), ptr(mean64), ptr(A), k, ptr(T),
                                                  ptr(T2), ptr(Q), dec_p, ptr(accept_out), accept_stride, ptr(st),
                                                  _stream(dev)), "ocm_score_f32_diag_prep")
        out["T"], out["T2"], out["Q"], out["stats"] = T, T2, Q, st
        return out
    fn = "ocm_score_f64_diag" if f64 else ("ocm_score_f32_diag" if A.dim() == 1 else "ocm_score_f32")
    check(getattr(_lib.load(), fn)(ctx.handle, ptr(X), X.stride(0), ptr(rows), m, p, ptr(P64), ptr(mean64),
                                   ptr(A), k, ptr(T), ptr(T2), ptr(Q), dec_p, ptr(accept_out), accept_stride,
                                   ptr(st), _stream(dev)), fn)
    out["T"], out["T2"], out["Q"], out["stats"] = T, T2, Q, st
    return out


def decide(T2: torch.Tensor, Q: torch.Tensor, decision: OcmDecision, want_red=True, want_dred=False,
           accept_out=None, accept_stride=1):
    m = T2.shape[0]
    dev = T2.device
    t2r = torch.empty(m, dtype=torch.float64, device=dev) if want_red else None
    qr = torch.empty(m, dtype=torch.float64, device=dev) if want_red else None
    dr = torch.empty(m, dtype=torch.float64, device=dev) if want_dred else None
    ctx = Context.get(dev.index)
    fn = "ocm_decide_f64" if Q.dtype == torch.float64 else "ocm_decide"
    check(getattr(_lib.load(), fn)(ctx.handle, ptr(T2), ptr(Q), m, ctypes.byref(decision), ptr(t2r), ptr(qr),
                                   ptr(dr), ptr(accept_out), accept_stride, _stream(dev)), fn)
    return t2r, qr, dr


def confusion_counts(accept: torch.Tensor, positive: torch.Tensor, stride: int = 1) -> torch.Tensor:
    """{TP, TN, FP, FN} (int64, device) of a 0/1 prediction column ``accept``
    (float64, read at ``stride``) against the uint8 mask ``positive``."""
    m = positive.numel()
    out = torch.empty(4, dtype=torch.int64, device=positive.device)
    check(_lib.load().ocm_confusion_counts(Context.get(positive.device.index).handle, ptr(accept), m, int(stride),
                                           ptr(positive), ptr(out), _stream(positive.device)),
          "ocm_confusion_counts")
    return out


def percentile(v: torch.Tensor, pct: float) -> float:
    dtype = 0 if v.dtype == torch.float64 else 1
    if v.dtype not in (torch.float64, torch.float32):
        raise TypeError("percentile: float32/float64 only")
    out = ctypes.c_double(0.0)
    ctx = Context.get(v.device.index)
    check(_lib.load().ocm_percentile(ctx.handle, ptr(v), dtype, v.numel(), float(pct), ctypes.byref(out),
                                     _stream(v.device)), "ocm_percentile")
    return out.value


def gram_combine(terms, G_out: torch.Tensor | None, cs_out: torch.Tensor | None):
    """G_out = Σ coef·G, cs_out = Σ coef·colsum over terms [(coef, G, colsum)]."""
    nt = len(terms)
    dev = terms[0][1].device
    p = terms[0][1].shape[-1]
    Gp = (ctypes.c_void_p * nt)(*[t[1].data_ptr() for t in terms])
    with_cs = all(t[2] is not None for t in terms)
    if cs_out is not None and not with_cs:
        raise ValueError("gram_combine: cs_out needs every term's column sums")
    Sp = (ctypes.c_void_p * nt)(*[t[2].data_ptr() for t in terms]) if with_cs else None
    cf = (ctypes.c_double * nt)(*[float(t[0]) for t in terms])
    check(_lib.load().ocm_gram_combine(Context.get(dev.index).handle, Gp, Sp, cf, nt, p, ptr(G_out), ptr(cs_out),
                                       _stream(dev)), "ocm_gram_combine")


def cv_prefix(T: torch.Tensor, Q: torch.Tensor, inv_evals: torch.Tensor, lvs, want_T2=False, want_Q=False,
              want_stats=True):
    """Per-LV T² / Q of rows scored at LV_max (+ moments {ΣT², ΣT²², ΣQ, ΣQ²} per LV)."""
    m, k = T.shape
    dev = T.device
    nlv = len(lvs)
    T2o = torch.empty((nlv, m), dtype=torch.float64, device=dev) if want_T2 else None
    Qo = torch.empty((nlv, m), dtype=torch.float32, device=dev) if want_Q else None
    st = torch.empty((nlv, 4), dtype=torch.float64, device=dev) if want_stats else None
    arr = (ctypes.c_int32 * nlv)(*[int(v) for v in lvs])
    check(_lib.load().ocm_cv_prefix(Context.get(dev.index).handle, ptr(T), m, k, ptr(Q), ptr(inv_evals), arr, nlv,
                                    ptr(T2o), ptr(Qo), ptr(st), _stream(dev)), "ocm_cv_prefix")
    return T2o, Qo, st


def cv_counts(T: torch.Tensor, Q: torch.Tensor, inv_evals: torch.Tensor, positive: torch.Tensor, m_split: int,
              configs, want_accept=False):
    """Confusion counts (ncfg, 2, 4) uint64-as-int64 {TP, TN, FP, FN} for rows [0, m_split) and
    [m_split, m); configs = [(lv, type_name, t2_scale, q_scale, dlim)]."""
    m, k = T.shape
    dev = T.device
    nc = len(configs)
    counts = torch.empty((nc, 2, 4), dtype=torch.int64, device=dev)
    acc = torch.empty((nc, m), dtype=torch.float64, device=dev) if want_accept else None
    # ≤ OCM_CV_MAXCFG configurations per launch (the kernel's LDS counters)
    for c0 in range(0, nc, _lib.OCM_CV_MAXCFG):
        part = configs[c0:c0 + _lib.OCM_CV_MAXCFG]
        n = len(part)
        arr = (_lib.OcmCvConfig * n)(*[_lib.OcmCvConfig(int(lv), TYPE_CODES[ty], float(a), float(b), float(d))
                                       for (lv, ty, a, b, d) in part])
        check(_lib.load().ocm_cv_counts(Context.get(dev.index).handle, ptr(T), m, k, ptr(Q), ptr(inv_evals),
                                        ptr(positive), int(m_split), arr, n, ptr(counts[c0:]),
                                        ptr(acc[c0:] if acc is not None else None), _stream(dev)), "ocm_cv_counts")
    return counts, acc


def radix_hist(v: torch.Tensor, prefix: int, shift: int, hist: torch.Tensor | None = None) -> torch.Tensor:
    """One radix-select pass (ocm_radix_hist): 256-bin counts of the order keys
    of ``v`` that match ``prefix`` above bit ``shift + 8``, binned by the 8 bits
    at ``shift``.  int64 tensor on the device."""
    if v.dtype not in (torch.float64, torch.float32):
        raise TypeError("radix_hist: float32/float64 only")
    if hist is None:
        hist = torch.empty(256, dtype=torch.int64, device=v.device)
    if v.numel() == 0:  # a rank without values takes part in the all-reduce with zeros
        return hist.zero_()
    check(_lib.load().ocm_radix_hist(Context.get(v.device.index).handle, ptr(v), 0 if v.dtype == torch.float64 else 1,
                                     v.numel(), ctypes.c_uint64(prefix), shift, ptr(hist), _stream(v.device)),
          "ocm_radix_hist")
    return hist


def rowsq_residual(x: torch.Tensor, xhat: torch.Tensor) -> torch.Tensor:
    """q_i = Σ_j (x_ij − xhat_ij)² (float32 out, fp64 accumulation).  ``xhat``
    may be one row (shape (p,) or (1, p)): it is broadcast to every row."""
    m, p = x.shape
    if m == 0:
        return torch.empty(0, dtype=torch.float32, device=x.device)
    if x.stride(1) != 1:
        x = x.contiguous()
    bcast = xhat.dim() == 1 or xhat.shape[0] == 1
    xh = xhat.reshape(1, p) if bcast else xhat
    if xh.stride(-1) != 1:
        xh = xh.contiguous()
    q = torch.empty(m, dtype=torch.float32, device=x.device)
    ctx = Context.get(x.device.index)
    check(_lib.load().ocm_rowsq_residual_f32(ctx.handle, ptr(x), x.stride(0), ptr(xh), 0 if bcast else xh.stride(0),
                                             m, p, ptr(q), _stream(x.device)), "ocm_rowsq_residual_f32")
    return q


def rowsq_minmax(x: torch.Tensor, xhat: torch.Tensor, eps: float = 1e-8) -> torch.Tensor:
    """Per-sample min–max scaled residual Σ_j (s(x) − s(x̂))² (float32 out):
    utils/final_vaesimca.py:417-423, 484-490 (ocm_rowsq_minmax_f32)."""
    m, p = x.shape
    if m == 0:
        return torch.empty(0, dtype=torch.float32, device=x.device)
    x = x if x.stride(1) == 1 else x.contiguous()
    xhat = xhat if xhat.stride(1) == 1 else xhat.contiguous()
    q = torch.empty(m, dtype=torch.float32, device=x.device)
    check(_lib.load().ocm_rowsq_minmax_f32(Context.get(x.device.index).handle, ptr(x), x.stride(0), ptr(xhat),
                                           xhat.stride(0), m, p, float(eps), ptr(q), _stream(x.device)),
          "ocm_rowsq_minmax_f32")
    return q


_SIDE: dict = {}


def _side_stream(dev: torch.device) -> torch.cuda.Stream:
    """One auxiliary stream per device for small D2H reads that must not wait
    for work queued after them on the launch stream."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=key)
    return _SIDE[key]


_PINNED: dict = {}


def _pinned(dev: torch.device, n: int) -> torch.Tensor:
    """A per-device pinned float64 staging buffer of ≥ n values (fit_class
    reads it back before it returns, so consecutive fits can share it; a fresh
    pinned allocation per fit cost host time on the GPU's critical path)."""
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    buf = _PINNED.get(key)
    if buf is None or buf.numel() < n:
        buf = _PINNED[key] = torch.empty(max(n, 64), dtype=torch.float64, pin_memory=True)
    return buf[:n]


def inv_evals(evals: torch.Tensor, rcond=1e-15, out: torch.Tensor | None = None) -> torch.Tensor:
    """Diagonal of pinv(cov(T)) for T = centred scores on the eigenbasis:
    cov(T) = diag(λ) (utils/SIMCA.py:69 with np.linalg.pinv's rcond=1e-15 cutoff)."""
    lam = evals.to(torch.float64).contiguous()
    if out is None:
        out = torch.empty_like(lam)
    check(_lib.load().ocm_inv_evals_f64(Context.get(lam.device.index).handle, ptr(lam), lam.numel(), float(rcond),
                                        ptr(out), _stream(lam.device)), "ocm_inv_evals_f64")
    return out


def invcov_from_evals(evals: torch.Tensor, rcond=1e-15) -> torch.Tensor:
    """pinv(cov(T)) as the (k, k) matrix the reference stores (``invcovT``)."""
    return torch.diag(inv_evals(evals, rcond))


def gram_pack(G: torch.Tensor, cs: torch.Tensor, shift32: torch.Tensor, n: int, out: torch.Tensor | None = None):
    """This rank's moments about zero in the packed all-reduce layout
    (ocm_gram_pack): p(p+1)/2 + p + 1 doubles."""
    p = shift32.shape[0]
    if out is None:
        out = torch.empty(p * (p + 1) // 2 + p + 1, dtype=torch.float64, device=G.device)
    check(_lib.load().ocm_gram_pack(Context.get(G.device.index).handle, ptr(G), ptr(cs), ptr(shift32), int(n), p,
                                    ptr(out), _stream(G.device)), "ocm_gram_pack")
    return out


def cov_from_packed(packed: torch.Tensor, p: int):
    """(C, mean) from summed packed moments (ocm_cov_from_packed; n read on the device)."""
    dev = packed.device
    C = torch.empty((p, p), dtype=torch.float64, device=dev)
    mean = torch.empty(p, dtype=torch.float64, device=dev)
    check(_lib.load().ocm_cov_from_packed(Context.get(dev.index).handle, ptr(packed), p, ptr(C), ptr(mean),
                                          _stream(dev)), "ocm_cov_from_packed")
    return C, mean


# ---- optional per-phase timing (bench.py): HIP events on the launch stream ----
_phase_timer = None


def set_phase_timer(timer):
    """Install (or clear with None) a recorder with ``mark(name)``; the fit
    and scoring paths then mark their phase boundaries on the launch stream."""
    global _phase_timer
    prev, _phase_timer = _phase_timer, timer
    return prev


def _mark(name: str):
    if _phase_timer is not None:
        _phase_timer.mark(name)


def common_shift(X: torch.Tensor, rows: torch.Tensor | None, n: int, allreduce) -> torch.Tensor:
    """The Gram shift every rank of a sharded fit uses (f32): the mean of the
    ranks' sample means (ranks without rows do not count), one all-reduce of
    p + 1 doubles.  One shift for all ranks means the summed moments stay
    centred to O(σ) and C is formed as (G − c cᵀ/n)/(n − 1) about it, never
    as (M − n μμᵀ)/(n − 1) about zero (which would cancel |μ|²/λ_tail)."""
    p = X.shape[1]
    buf = torch.zeros(p + 1, dtype=torch.float64, device=X.device)
    if n > 0:
        buf[:p] = colmean(X, rows, max(1, min(n, SHIFT_SAMPLE)))
        buf[p] = 1.0
    allreduce([buf])
    return cast_f32(buf[:p] / buf[p].clamp_min(1.0))


def fit_class(X: torch.Tensor, rows: torch.Tensor | None, n: int, k: int, theta_mode: int,
              want_T=True, keep_C=False, shift32: torch.Tensor | None = None, allreduce=None,
              need_stats=True) -> ClassFit:
    """Gram → covariance → top-k eigenpairs → fit-set scores for one class.

    ``allreduce`` (optional callable on a list of device tensors, with the
    rank / world size as attributes) marks a class whose rows are sharded
    over GPUs: every rank's Gram is taken about one common
    shift (``common_shift``), packed as its upper triangle (``ocm_gram_pack``
    about a zero shift) and summed in ONE all-reduce; the θ3 trace work is
    split over the ranks and its partials summed; the fit-set moments are
    all-reduced only when ``need_stats``."""
    p = X.shape[1]
    if k > p or k < 1:
        raise ValueError(f"n_components={k} must be in [1, {p}]")
    _mark("start")
    if shift32 is None and allreduce is not None:
        shift32 = common_shift(X, rows, n, allreduce)
    elif shift32 is None:
        shift64 = colmean(X, rows, max(1, min(n, SHIFT_SAMPLE))) if n > 0 else torch.zeros(p, dtype=torch.float64,
                                                                                          device=X.device)
        shift32 = cast_f32(shift64)
    _mark("shift")
    slice_ = (0, 1)
    if allreduce is None:
        G, cs = gram(X, rows, [0, n], shift32)
        _mark("gram")
        n_total = n
        if n_total < 2:
            raise ValueError("SIMCA needs at least 2 samples in a class")
        C, mean64 = cov_from_gram([(1.0, G[0], cs[0])], shift32, n_total)
        del G
        _mark("cov")
    else:
        zero32 = torch.zeros(p, dtype=torch.float32, device=X.device)
        if n > 0:
            G, cs = gram(X, rows, [0, n], shift32)
            packed = gram_pack(G[0], cs[0], zero32, n)  # moments of y = x − shift
            del G, cs
        else:  # a rank without rows contributes zeros
            packed = torch.zeros(p * (p + 1) // 2 + p + 1, dtype=torch.float64, device=X.device)
        _mark("gram")
        allreduce([packed])
        _mark("allreduce")
        C, d = cov_from_packed(packed, p)
        mean64 = d + shift32.to(torch.float64)
        _mark("cov")
        slice_ = (allreduce.rank, allreduce.world)
        n_total = None
    # the fit-set outputs are allocated while the GPU still runs the Gram and the
    # eigensolve: once the eigensolver has read its convergence test back, the
    # launch queue is nearly empty and every host µs before the scoring launch
    # is GPU idle time
    pre = score_outputs(_plain(X), n, k, want_T, True, True, True) if n > 0 else None
    inv = torch.empty(k, dtype=torch.float64, device=X.device)
    eig_done = torch.cuda.Event()
    evals, evecs, theta, iters = eig_topk(C, k, theta_mode, theta3_slice=slice_, inv_out=inv)
    if n_total is None:
        n_total = int(round(float(packed[-1].item())))  # complete: the eigensolver synchronised
        if n_total < 2:
            raise ValueError("SIMCA needs at least 2 samples in a class")
        if theta_mode >= 2 and slice_[1] > 1:
            allreduce([theta[2:]])  # θ3 partials of the ranks' trace slices
    _mark("eig")
    # The host needs λ and θ for the limits (SciPy), the device needs 1/λ for
    # the fit-set scoring.  The eigensolver has just synchronised on its
    # convergence test, so the launch queue is nearly empty: 1/λ and the
    # scoring are launched first (every host µs before that launch is GPU idle
    # time), then λ and θ go to pinned memory on a side stream that waits only
    # for the eigensolve, and the limits overlap the scoring.
    eig_done.record(torch.cuda.current_stream(X.device))  # (1/λ was queued inside the eigensolve)
    if n > 0:
        sc = score(X, rows, n, evecs, mean64, inv, want_T=want_T, want_stats=True, outs=pre)
    else:  # T and Q in the dtype the other ranks' scoring produces (utils/SIMCA.py:65-71)
        vdt = torch.float64 if X.dtype == torch.float64 else torch.float32
        sc = {"T": torch.empty((0, k), dtype=vdt, device=X.device) if want_T else None,
              "T2": torch.empty(0, dtype=torch.float64, device=X.device),
              "Q": torch.empty(0, dtype=vdt, device=X.device),
              "stats": torch.zeros(4, dtype=torch.float64, device=X.device)}
    host_buf = _pinned(X.device, k + 3)
    side = _side_stream(X.device)
    with torch.cuda.stream(side):
        side.wait_event(eig_done)
        host_buf[:k].copy_(evals, non_blocking=True)
        host_buf[k:].copy_(theta, non_blocking=True)
        copied = torch.cuda.Event()
        copied.record(side)
    _mark("fit_score")
    copied.synchronize()
    host = host_buf.numpy().copy()
    ev_h = host[:k]
    th = tuple(float(v) for v in host[k:k + 3])
    stats = sc["stats"]
    if allreduce is not None and need_stats:
        allreduce([stats])  # stream-ordered: no host wait
    fit = ClassFit(k=k, n=n_total, p=p, mean64=mean64, evals=evals, P64=evecs, inv_diag=inv, thetas=th,
                   evals_host=ev_h, T=sc["T"], T2=sc["T2"], Q=sc["Q"], stats_dev=stats, eig_iters=iters,
                   C=C if keep_C else None)
    fit.extra["shift32"] = shift32
    return fit
