"""Host-side scalar limits of SIMCA (fp64 SciPy quantiles), computed from the
device-side moments / percentiles / tail traces.

Mirror of utils/SIMCA.py:156-236 (``_Tlim``, ``_Qlim``, ``_critic_distance``):
same formulas, same quirks (chi2pom state kept on the estimator and
overwritten per class; unknown limit names leave the result unbound).
"""
from __future__ import annotations

import functools
import math

import numpy as np
from scipy import stats
from scipy.special import erfinv


# The quantiles are pure functions of (level, degrees of freedom); SciPy's
# rv_continuous.ppf costs ≈ 140 µs of argument handling per call, the whole
# host side of a refit at 125k rows, so repeated fits with the same (n, k,
# level) look them up.  Results are SciPy's own, bit for bit.
@functools.lru_cache(maxsize=4096)
def _f_ppf(q: float, dfn: float, dfd: float) -> float:
    return stats.f.ppf(q, dfn, dfd)


@functools.lru_cache(maxsize=4096)
def _chi2_ppf(q: float, df: float) -> float:
    return stats.chi2.ppf(q, df)


class Moments:
    """n, Σx, Σx² of a device vector (from the scoring kernel's fused stats)
    plus a lazy percentile callback (device radix select).  ``s1`` may be a
    callable returning (Σx, Σx²): the sums are then read from the device only
    if a limit needs them (chi2pom / moments), so the Fdist / jm path never
    waits for the fit-set scoring kernel."""

    def __init__(self, n, s1, s2=None, percentile=None):
        self.n = int(n)
        if callable(s1):
            self._sums, self._s = s1, None
        else:
            self._sums, self._s = None, (float(s1), float(s2))
        self._pct = percentile

    def _get(self):
        if self._s is None:
            a, b = self._sums()
            self._s = (float(a), float(b))
        return self._s

    @property
    def s1(self) -> float:
        return self._get()[0]

    @property
    def s2(self) -> float:
        return self._get()[1]

    @property
    def mean(self) -> float:
        return self.s1 / self.n

    def var(self, ddof=1) -> float:
        if self.n - ddof <= 0:
            return float("nan")
        m = self.mean
        return max(self.s2 - self.n * m * m, 0.0) / (self.n - ddof)

    def percentile(self, pct: float) -> float:
        return self._pct(pct)


def t2_limit(est, T2: Moments, k: int) -> float:
    """utils/SIMCA.py:156-182."""
    n = T2.n
    if est.t2lim == "perc":
        return T2.percentile(est.t2cl * 100)
    if est.t2lim == "Fdistrig":
        F = _f_ppf(est.t2cl, k, n - k)
        return (k / n) * (n ** 2 - 1) / (n - k) * F
    if est.t2lim == "Fdist":
        F = _f_ppf(est.t2cl, k, n - k)
        return k * (n - 1) / (n - k) * F
    if est.t2lim == "chi2":
        return _chi2_ppf(est.t2cl, k)
    if est.t2lim == "chi2pom":
        h0 = float(T2.mean)
        v = float(T2.var(ddof=1)) if n > 1 else 0.0
        Nh = max(int(np.round(2 * (h0 ** 2) / v)) if v > 0 else 1, 1)
        est._t2dof = Nh
        est._t2scfact = h0
        return h0 * _chi2_ppf(est.t2cl, Nh) / Nh
    raise UnboundLocalError(f"local variable 'T2_limit' referenced before assignment (t2lim={est.t2lim!r})")


def q_limit(est, Q: Moments, thetas) -> float:
    """utils/SIMCA.py:184-217.  ``thetas`` = (θ1, θ2, θ3) of the discarded eigenvalues."""
    if est.qlim == "perc":
        return Q.percentile(est.qcl * 100)
    if est.qlim == "jm":
        th1, th2, th3 = thetas
        if th1 == 0:
            raise UnboundLocalError("local variable 'h0' referenced before assignment (jm limit with theta1 == 0)")
        h0 = 1 - (2 * th1 * th3) / (3 * th2 ** 2)
        h0 = max(h0, 0.001)
        ca = math.sqrt(2) * erfinv(2 * est.qcl - 1)
        h1 = ca * math.sqrt(2 * th2 * h0 ** 2) / th1
        h2 = th2 * h0 * (h0 - 1) / (th1 ** 2)
        return th1 * (h1 + 1 + h2) ** (1 / h0)
    if est.qlim == "chi2box":
        th1, th2, _ = thetas
        g = th2 / th1
        Ng = (th1 ** 2) / th2
        print("here we are")  # reference prints these (utils/SIMCA.py:207-208)
        print(th1, th2, g, Ng)
        return g * _chi2_ppf(est.qcl, Ng)
    if est.qlim == "chi2pom":
        v0 = np.float64(Q.mean)
        Nv = max(round(2 * (v0 ** 2) / np.float64(Q.var(ddof=1))), 1)
        est._qdof = Nv
        est._qscfact = float(v0)
        return float(v0 * _chi2_ppf(est.qcl, Nv) / Nv)
    raise UnboundLocalError(f"local variable 'Q_limit' referenced before assignment (qlim={est.qlim!r})")


def critic_distance(est, T2_limit, Q_limit, thetas, k: int):
    """utils/SIMCA.py:219-236."""
    if est.type == "sim":
        return 1
    if est.type == "alt":
        return np.sqrt(2)
    if est.type == "ci":
        th1, th2, _ = thetas
        tr1 = (k / T2_limit) + (th1 / Q_limit)
        tr2 = (k / T2_limit ** 2) + (th2 / Q_limit ** 2)
        gd = tr2 / tr1
        hd = tr1 ** 2 / tr2
        return gd * _chi2_ppf(est.dcl, hd)
    if est.type == "dd":
        return _chi2_ppf(est.dcl, est._t2dof + est._qdof)
    raise UnboundLocalError(f"local variable 'dlim' referenced before assignment (type={est.type!r})")


def theta_mode_for(est) -> int:
    """Which tail moments the configured limits need: jm → θ1..θ3,
    chi2box / ci → θ1..θ2, otherwise none."""
    if est.qlim == "jm":
        return 2
    if est.qlim == "chi2box" or est.type == "ci":
        return 1
    return 0
