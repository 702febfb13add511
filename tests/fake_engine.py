"""Test-only CPU stand-in for ``ocm.engine`` (NumPy / torch-CPU arithmetic).

Used ONLY by the CPU test suite to exercise the host and multi-rank logic of
the fold engine (ocm/cv.py) and the row-sharded SIMCA (ocm/dist.py) under
torch.distributed ``gloo`` without a GPU.
It implements the same contracts as the libocm entry points it stands in for
(include/ocm.h) with exact fp64 NumPy arithmetic: it is never imported by the
package, and the GPU tests call the real HIP kernels.
"""
from __future__ import annotations

import numpy as np
import torch

SHIFT_SAMPLE = 4096


def as_device_f32(X, device=None):
    t = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X))
    return t.to(torch.float32).contiguous()


def as_device_x(X, device=None):
    """ocm.engine.as_device_x: float64 stays float64, anything else float32."""
    t = X if isinstance(X, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(X))
    return (t.to(torch.float64) if t.dtype == torch.float64 else t.to(torch.float32)).contiguous()


def _rows(X, rows, n):
    Xn = X.numpy()
    if rows is None:
        return Xn[:n]
    return Xn[rows.numpy()[:n]]


def colmean(X, rows, n):
    return torch.from_numpy(_rows(X, rows, n).astype(np.float64).mean(0))


def cast_f32(a):
    return a.to(torch.float32)


def gram(X, rows, seg_offsets, shift32):
    seg = [int(s) for s in seg_offsets]
    Y = _rows(X, rows, seg[-1]).astype(np.float64) - shift32.numpy().astype(np.float64)
    p = Y.shape[1]
    G = np.zeros((len(seg) - 1, p, p))
    cs = np.zeros((len(seg) - 1, p))
    for s in range(len(seg) - 1):
        B = Y[seg[s]:seg[s + 1]]
        G[s] = B.T @ B
        cs[s] = B.sum(0)
    return torch.from_numpy(G), torch.from_numpy(cs)


def gram_combine(terms, G_out, cs_out):
    if G_out is not None:
        G_out.copy_(sum(float(c) * G for c, G, _ in terms))
    if cs_out is not None:
        cs_out.copy_(sum(float(c) * s for c, _, s in terms))


def cov_from_gram(terms, shift32, n):
    Gc = sum(float(c) * G for c, G, _ in terms).numpy()
    sc = sum(float(c) * s for c, _, s in terms).numpy()
    d = sc / n
    C = (Gc - n * np.outer(d, d)) / (n - 1)
    return torch.from_numpy(C), torch.from_numpy(shift32.numpy().astype(np.float64) + d)


def gram_pack(G, cs, shift32, n, out=None):
    """ocm_gram_pack: moments about zero, upper triangle + Σx + n."""
    s = shift32.numpy().astype(np.float64)
    c = cs.numpy()
    M = G.numpy() + np.outer(s, c) + np.outer(c, s) + n * np.outer(s, s)
    iu = np.triu_indices(s.size)
    return torch.from_numpy(np.concatenate([M[iu], c + n * s, [float(n)]]))


def cov_from_packed(packed, p):
    a = packed.numpy()
    tri = p * (p + 1) // 2
    M = np.zeros((p, p))
    M[np.triu_indices(p)] = a[:tri]
    M = M + np.triu(M, 1).T
    n = a[-1]
    mu = a[tri:tri + p] / n
    return torch.from_numpy((M - n * np.outer(mu, mu)) / (n - 1)), torch.from_numpy(mu)


def _theta3_slice(D, slice_):
    """This slice's share of θ3 = trace(D³) as ocm_eig_topk_ex splits it: rows
    [p·s/S, p·(s+1)/S) of the Δ / O expansion (Δ the diagonal, O the rest),
    Σ_i Δ_i³ + 3 Σ_i Δ_i Σ_j O_ij² + Σ_ij O_ij (O_rowsᵀ O_rows)_ij."""
    p = D.shape[0]
    s, S = slice_
    r0, r1 = p * s // S, p * (s + 1) // S
    dg = np.diag(D)
    O = D - np.diag(dg)
    rows = slice(r0, r1)
    t = (dg[rows] ** 3).sum() + 3.0 * (dg[rows] * (O[rows] ** 2).sum(1)).sum()
    G = O[rows].T @ O[rows]
    return t + (O * G).sum()


def eig_topk(C, k, theta_mode, tol=None, max_iter=None, theta3_slice=(0, 1)):
    Cn = C.numpy()
    w, V = np.linalg.eigh(Cn)
    w, V = w[::-1], V[:, ::-1]
    P = V[:, :k].T.copy()
    idx = np.argmax(np.abs(P), axis=1)
    P *= np.sign(P[np.arange(k), idx])[:, None]
    tail = w[k:]
    th = np.array([tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()]) if theta_mode else np.zeros(3)
    if theta_mode >= 2 and Cn.shape[0] > 64:
        D = Cn - (V[:, :k] * w[:k]) @ V[:, :k].T
        th[2] = _theta3_slice(D, theta3_slice)
    elif theta_mode >= 2 and theta3_slice[0] != 0:
        th[2] = 0.0  # p ≤ 64: slice 0 carries the whole θ3
    return torch.from_numpy(w[:k].copy()), torch.from_numpy(P), torch.from_numpy(th), 1


def score(X, rows, m, P64, mean64, A, want_T=False, want_T2=True, want_Q=True, decision=None, accept_out=None,
          accept_stride=1, want_stats=False):
    Y = _rows(X, rows, m).astype(np.float64) - mean64.numpy()
    P = P64.numpy()
    T = Y @ P.T
    R = Y - T @ P
    Q = (R ** 2).sum(1).astype(np.float32)
    T32 = T.astype(np.float32)
    Am = np.diag(A.numpy()) if A.dim() == 1 else A.numpy()
    T2 = np.einsum("ij,jk,ik->i", T32.astype(np.float64), Am, T32.astype(np.float64))
    out = {"T": torch.from_numpy(T32) if want_T else None, "T2": torch.from_numpy(T2) if want_T2 else None,
           "Q": torch.from_numpy(Q) if want_Q else None, "stats": None}
    if want_stats:
        q = Q.astype(np.float64)
        out["stats"] = torch.tensor([T2.sum(), (T2 ** 2).sum(), q.sum(), (q ** 2).sum()], dtype=torch.float64)
    return out


def rowsq_residual(x, xhat):
    xn = x.numpy().astype(np.float64)
    xh = xhat.numpy().astype(np.float64).reshape(-1, xn.shape[1])
    return torch.from_numpy(((xn - xh) ** 2).sum(1).astype(np.float32))


def sym_pinv(A, rcond=1e-15):
    w, V = np.linalg.eigh(A.numpy())
    cut = rcond * np.abs(w).max()
    inv = np.where(np.abs(w) > cut, 1.0 / np.where(w == 0, 1, w), 0.0)
    return torch.from_numpy((V * inv) @ V.T)


def _prefix(T, Q, inv, lv):
    t2sq = T.numpy().astype(np.float64) ** 2
    t2 = (t2sq[:, :lv] * inv.numpy()[:lv]).sum(1)
    q = (Q.numpy().astype(np.float64) + t2sq[:, lv:].sum(1)).astype(np.float32)
    return t2, q


def cv_prefix(T, Q, inv_evals, lvs, want_T2=False, want_Q=False, want_stats=True):
    T2s, Qs, st = [], [], []
    for lv in lvs:
        t2, q = _prefix(T, Q, inv_evals, lv)
        T2s.append(t2)
        Qs.append(q)
        qd = q.astype(np.float64)
        st.append([t2.sum(), (t2 ** 2).sum(), qd.sum(), (qd ** 2).sum()])
    return (torch.from_numpy(np.stack(T2s)) if want_T2 else None,
            torch.from_numpy(np.stack(Qs)) if want_Q else None,
            torch.tensor(st, dtype=torch.float64) if want_stats else None)


def cv_counts(T, Q, inv_evals, positive, m_split, configs, want_accept=False):
    pos = positive.numpy().astype(bool)
    m = pos.shape[0]
    counts = np.zeros((len(configs), 2, 4), dtype=np.int64)
    acc_all = np.zeros((len(configs), m))
    for c, (lv, ty, a, b, dl) in enumerate(configs):
        t2, q = _prefix(T, Q, inv_evals, lv)
        t, qq = t2 * a, q.astype(np.float64) * b
        d = {"sim": np.maximum(t, qq), "alt": np.sqrt(t * t + qq * qq)}.get(ty, t + qq)
        acc = d < dl
        acc_all[c] = acc
        for part, sl in ((0, slice(0, m_split)), (1, slice(m_split, m))):
            A, P = acc[sl], pos[sl]
            counts[c, part] = [np.sum(A & P), np.sum(~A & ~P), np.sum(A & ~P), np.sum(~A & P)]
    return torch.from_numpy(counts), (torch.from_numpy(acc_all) if want_accept else None)


def percentile(v, pct):
    return float(np.percentile(v.numpy(), pct))


def _okey(v: np.ndarray) -> np.ndarray:
    """Order-preserving unsigned keys (the IEEE sign trick of ocm_select.hip)."""
    if v.dtype == np.float64:
        u = v.view(np.uint64)
        return np.where(u >> np.uint64(63), ~u, u | np.uint64(1 << 63))
    u = v.view(np.uint32).astype(np.uint64)
    return np.where(u >> np.uint64(31), (~u) & np.uint64(0xFFFFFFFF), u | np.uint64(0x80000000))


def radix_hist(v, prefix, shift, hist=None):
    a = v.numpy()
    nbits = 64 if a.dtype == np.float64 else 32
    keys = _okey(a)
    if shift + 8 >= nbits:
        sel = keys
    else:
        hi = np.uint64(((~0) << (shift + 8)) & ((1 << nbits) - 1))
        sel = keys[((keys ^ np.uint64(prefix)) & hi) == 0]
    digits = ((sel >> np.uint64(shift)) & np.uint64(255)).astype(np.int64)
    return torch.from_numpy(np.bincount(digits, minlength=256).astype(np.int64))


def make_decision(type_name, t2_scale, q_scale, dlim):
    from ocm._lib import OcmDecision, TYPE_CODES

    return OcmDecision(TYPE_CODES[type_name], 0, float(t2_scale), float(q_scale), float(dlim))


def _dred(code, t, q):
    return {0: np.maximum(t, q), 1: np.sqrt(t * t + q * q)}.get(code, t + q)


_score_plain = score


def score(X, rows, m, P64, mean64, A, want_T=False, want_T2=True, want_Q=True, decision=None, accept_out=None,
          accept_stride=1, want_stats=False):
    out = _score_plain(X, rows, m, P64, mean64, A, want_T=True, want_T2=True, want_Q=True, want_stats=want_stats)
    if decision is not None:
        d = _dred(decision.type, out["T2"].numpy() * decision.t2_scale,
                  out["Q"].numpy().astype(np.float64) * decision.q_scale)
        acc = torch.from_numpy((d < decision.dlim).astype(np.float64))
        if accept_out.dim() == 2:  # a column of the (m, C) prediction matrix
            accept_out[:m, 0].copy_(acc)
        else:
            accept_out[::accept_stride][:m].copy_(acc)
    if not want_T:
        out["T"] = None
    return out


def decide(T2, Q, decision, want_red=True, want_dred=False, accept_out=None, accept_stride=1):
    t = T2.numpy() * decision.t2_scale
    q = Q.numpy().astype(np.float64) * decision.q_scale
    d = _dred(decision.type, t, q)
    return (torch.from_numpy(t) if want_red else None, torch.from_numpy(q) if want_red else None,
            torch.from_numpy(d) if want_dred else None)


def confusion_counts(accept, positive, stride=1):
    m = positive.numel()
    a = (accept[:m, 0] if accept.dim() == 2 else accept[::stride][:m]).numpy() == 1
    pos = positive.numpy().astype(bool)
    return torch.tensor([np.sum(a & pos), np.sum(~a & ~pos), np.sum(a & ~pos), np.sum(~a & pos)], dtype=torch.int64)


class _Fit:
    def __init__(self, **kw):
        self.__dict__.update(kw)
        self.extra = {}

    def invcov_mat(self):
        return self.invcov


def invcov_from_evals(evals, rcond=1e-15):
    lam = evals.to(torch.float64)
    cut = rcond * lam.abs().max()
    return torch.diag(torch.where(lam.abs() > cut, 1.0 / lam, torch.zeros_like(lam)))


def common_shift(X, rows, n, allreduce):
    """ocm.engine.common_shift: the mean of the ranks' sample means."""
    p = X.shape[1]
    buf = torch.zeros(p + 1, dtype=torch.float64)
    if n > 0:
        buf[:p] = colmean(X, rows, max(1, min(n, SHIFT_SAMPLE)))
        buf[p] = 1.0
    allreduce([buf])
    return cast_f32(buf[:p] / buf[p].clamp_min(1.0))


def fit_class(X, rows, n, k, theta_mode, want_T=True, keep_C=False, shift32=None, allreduce=None, need_stats=True):
    """Same control flow and collectives as ocm.engine.fit_class."""
    p = X.shape[1]
    if shift32 is None and allreduce is not None:
        shift32 = common_shift(X, rows, n, allreduce)
    elif shift32 is None:
        shift32 = cast_f32(colmean(X, rows, min(n, SHIFT_SAMPLE)))
    slice_ = (0, 1)
    if allreduce is None:
        G, cs = gram(X, rows, [0, n], shift32)
        n_total = n
        C, mean64 = cov_from_gram([(1.0, G[0], cs[0])], shift32, n_total)
    else:
        G, cs = gram(X, rows, [0, n], shift32)
        packed = gram_pack(G[0], cs[0], torch.zeros_like(shift32), n)
        allreduce([packed])
        C, d = cov_from_packed(packed, p)
        mean64 = d + shift32.to(torch.float64)
        slice_ = (allreduce.rank, allreduce.world)
        n_total = int(round(float(packed[-1])))
    evals, evecs, theta, iters = eig_topk(C, k, theta_mode, theta3_slice=slice_)
    if allreduce is not None and theta_mode >= 2 and slice_[1] > 1:
        t3 = theta[2:].clone()
        allreduce([t3])
        theta[2:] = t3
    invcov = invcov_from_evals(evals)
    sc = score(X, rows, n, evecs, mean64, torch.diagonal(invcov).clone(), want_T=want_T, want_stats=True)
    stats = sc["stats"]
    if allreduce is not None and need_stats:
        allreduce([stats])
    st = stats.numpy()
    return _Fit(k=k, n=n_total, p=p, mean64=mean64, evals=evals, P64=evecs, invcov=invcov, inv_diag=torch.diagonal(invcov).clone(),
                thetas=tuple(float(v) for v in theta.numpy()), evals_host=evals.numpy(), T=sc["T"], T2=sc["T2"],
                Q=sc["Q"], T2_stats=(st[0], st[1]), Q_stats=(st[2], st[3]), eig_iters=iters, C=None)


def _mark(name):
    """Phase marks (ocm.engine.set_phase_timer): no timer in the CPU tests."""
