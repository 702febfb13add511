"""Row-sharded SIMCA over several GPUs (one process per GPU, RCCL).

SURVEY.md §8e: rows are independent and the covariance is a sum over rows,
so each rank accumulates the Gram / column sums of ITS rows
(``ocm_gram_f32``), one RCCL all-reduce over xGMI sums {G (p×p f64), Σy, n}
(the only exchange on the data path), every rank runs the same
deterministic fp64 eigensolver on the identical reduced C, and scores /
decides its own rows with no further traffic.  Moment-based limits
(chi2pom) all-reduce 4 scalars; percentile limits all-reduce the 256-bin
radix histograms of ``ocm_radix_hist`` per pass.

With world size 1 the same code runs with no collective.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import engine, limits


def make_allreduce(group=None):
    """Sum (or mean) a list of device tensors across the ranks of ``group``;
    the callable carries ``rank`` / ``world`` (the θ3 slice of this rank)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return None

    def allreduce(tensors, op="sum"):
        ws = dist.get_world_size(group)
        for t in tensors:
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
            if op == "mean":
                t.div_(ws)

    allreduce.rank = dist.get_rank(group)
    allreduce.world = dist.get_world_size(group)
    return allreduce


def percentile_sharded(v: torch.Tensor, pct: float, n_total: int, group=None) -> float:
    """np.percentile(linear) of the concatenation of every rank's ``v`` by a
    distributed radix select: each pass's 256-bin histogram (ocm_radix_hist)
    is all-reduced, so every rank walks the same digits.  The interpolation
    follows NumPy's dtype rules exactly as the single-GPU ocm_percentile does
    (float32 arithmetic for a float32 array)."""
    allreduce = make_allreduce(group)
    if allreduce is None:
        return engine.percentile(v, pct)
    f32 = v.dtype == torch.float32
    nbits = 32 if f32 else 64

    def kth(rank):
        prefix = 0
        for shift in range(nbits - 8, -1, -8):
            hist = engine.radix_hist(v, prefix, shift)
            allreduce([hist])
            c = np.cumsum(hist.cpu().numpy())
            dgt = int(np.searchsorted(c, rank, side="right"))
            rank -= int(c[dgt - 1]) if dgt > 0 else 0
            prefix |= dgt << shift
        return _key_to_value(prefix, 1 if f32 else 0)

    return _interp(kth, n_total, pct, f32)


def _interp(kth, n, pct, f32):
    """NumPy 2.2 method='linear' (numpy/lib/_function_base_impl.py): q, the
    virtual index and gamma in the array dtype; _lerp's b-side form for
    gamma >= 0.5; the top index takes the last order statistic."""
    ft = np.float32 if f32 else np.float64
    q = ft(pct) / ft(100)
    vi = ft(n - 1) * q
    lo_f = np.floor(vi)
    top = vi >= ft(n - 1)
    lo = n - 1 if top else int(lo_f)
    g = ft(vi - lo_f)
    a = ft(kth(lo))
    b = a if top else ft(kth(lo + 1))
    diff = ft(b - a)
    return float(ft(b - diff * (ft(1) - g)) if g >= ft(0.5) else ft(a + diff * g))


def _key_to_value(key: int, dtype: int) -> float:
    if dtype == 0:
        u = (key & 0x7FFFFFFFFFFFFFFF) if (key >> 63) else (~key & 0xFFFFFFFFFFFFFFFF)
        return float(np.array([u], dtype=np.uint64).view(np.float64)[0])
    k32 = key & 0xFFFFFFFF
    u = (k32 & 0x7FFFFFFF) if (k32 >> 31) else (~k32 & 0xFFFFFFFF)
    return float(np.array([u], dtype=np.uint32).view(np.float32)[0])


class ShardedSIMCA:
    """One-class SIMCA whose training / scoring rows are sharded over ranks.
    Configuration keywords as utils.SIMCA (type, t2lim, t2cl, qlim, qcl, dcl)."""

    def __init__(self, n_components=2, type="alt", t2lim="Fdist", t2cl=0.95, qlim="jm", qcl=0.95, dcl=0.95,
                 group=None, want_T=True):
        self.n_components = int(n_components)
        self.type, self.t2lim, self.t2cl, self.qlim, self.qcl, self.dcl = type, t2lim, t2cl, qlim, qcl, dcl
        if type == "dd":
            self.t2lim = self.qlim = "chi2pom"
        self.group = group
        self.want_T = want_T  # the reference's fit keeps the n×k scores T (utils/SIMCA.py:65, 89)

    def fit(self, X_local: torch.Tensor, rows=None, n_local=None):
        ar = make_allreduce(self.group)
        n_local = X_local.shape[0] if n_local is None else n_local
        k = self.n_components
        need_stats = "chi2pom" in (self.t2lim, self.qlim)  # moments feed only chi2pom limits
        self.fit_ = fit = engine.fit_class(X_local, rows, n_local, k, limits.theta_mode_for(self), want_T=self.want_T,
                                           allreduce=ar, need_stats=need_stats)
        n = fit.n
        T2m = limits.Moments(n, lambda: fit.T2_stats, None, lambda pct: percentile_sharded(fit.T2, pct, n, self.group))
        Qm = limits.Moments(n, lambda: fit.Q_stats, None, lambda pct: percentile_sharded(fit.Q, pct, n, self.group))
        self.T2_limit = limits.t2_limit(self, T2m, k)
        self.Q_limit = limits.q_limit(self, Qm, fit.thetas)
        self.D_limit = limits.critic_distance(self, self.T2_limit, self.Q_limit, fit.thetas, k)
        engine._mark("limits")
        if self.type == "dd":
            self.decision = engine.make_decision("dd", self._t2dof / self._t2scfact, self._qdof / self._qscfact,
                                                 self.D_limit)
        else:
            self.decision = engine.make_decision(self.type, 1.0 / self.T2_limit, 1.0 / self.Q_limit, self.D_limit)
        return self

    def predict(self, X_local: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        """Accept (1.0) / reject (0.0) per local row, float64 in HBM."""
        m = X_local.shape[0]
        if out is None:
            out = torch.empty(m, dtype=torch.float64, device=X_local.device)
        if m == 0:  # a rank without rows has nothing to score (its block is empty)
            return out
        fit = self.fit_
        engine.score(X_local, None, m, fit.P64, fit.mean64, fit.inv_diag, want_T2=False, want_Q=False,
                     decision=self.decision, accept_out=out, accept_stride=1)
        return out
