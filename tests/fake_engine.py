"""Test-only CPU stand-in for ``ocm.engine`` (NumPy / torch-CPU arithmetic).

Used ONLY by the CPU test suite to exercise the host and multi-rank logic of
the fold engine (ocm/cv.py) under torch.distributed ``gloo`` without a GPU.
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


def eig_topk(C, k, theta_mode, tol=None, max_iter=None):
    w, V = np.linalg.eigh(C.numpy())
    w, V = w[::-1], V[:, ::-1]
    P = V[:, :k].T.copy()
    idx = np.argmax(np.abs(P), axis=1)
    P *= np.sign(P[np.arange(k), idx])[:, None]
    tail = w[k:]
    th = np.array([tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()]) if theta_mode else np.zeros(3)
    return torch.from_numpy(w[:k].copy()), torch.from_numpy(P), torch.from_numpy(th), 1


def score(X, rows, m, P64, mean64, A, want_T=False, want_T2=True, want_Q=True, decision=None, accept_out=None,
          accept_stride=1, want_stats=False):
    Y = _rows(X, rows, m).astype(np.float64) - mean64.numpy()
    P = P64.numpy()
    T = Y @ P.T
    R = Y - T @ P
    Q = (R ** 2).sum(1).astype(np.float32)
    T32 = T.astype(np.float32)
    T2 = np.einsum("ij,jk,ik->i", T32.astype(np.float64), A.numpy(), T32.astype(np.float64))
    out = {"T": torch.from_numpy(T32) if want_T else None, "T2": torch.from_numpy(T2) if want_T2 else None,
           "Q": torch.from_numpy(Q) if want_Q else None, "stats": None}
    if want_stats:
        q = Q.astype(np.float64)
        out["stats"] = torch.tensor([T2.sum(), (T2 ** 2).sum(), q.sum(), (q ** 2).sum()], dtype=torch.float64)
    return out


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
