"""SIMCA-on-latents for VAE-SIMCA on libocm's HIP kernels.

The latent statistics of the reference's VAE scripts run here on the same
kernels as SIMCA, at p = d (latent width):

* ``qhf_device``            — vae_model.compute_q_h_f (vae_model.py:162-182):
  q by ``ocm_rowsq_residual_f32``; the leverage h = diag(U Uᵀ) of the
  column-standardised latent equals (z−μ)ᵀ (Z_cᵀZ_c)⁺ (z−μ) (the column
  scaling cancels), i.e. the T² of ``ocm_score_f32`` with P = I and
  A = pinv(C)/(n−1) from ``ocm_gram_f32`` → ``ocm_cov_from_gram`` →
  ``ocm_sym_pinv_f64``.
* ``latent_stats``          — utils/final_vaesimca.py:428-442 (latent mean,
  (cov + 1e-6 I)⁻¹, 95th-percentile T² and Q thresholds; device radix select).
* ``full_distance_decision`` — utils/final_vaesimca.py:510-533 (Euclidean h
  about the stored mean, test-set moments with ddof 0, χ² decision).
* ``VAESIMCA``              — VAE_SIMCA.py:215-382 (latent T² with pinv(cov +
  1e-12 I), latent round-trip Q = ‖z − enc(dec(z))‖², the percentile-variant
  limits of that script, and its decision rule).

Moments of per-row vectors are taken in fp64 on the device; scalar limits
are host fp64 (SciPy) as in the reference.
"""
from __future__ import annotations

import math

import numpy as np
import torch
from scipy import special, stats

from . import engine

__all__ = ["qhf_device", "latent_stats", "full_distance_decision", "VAESIMCA", "latent_T2"]


def _moments(v: torch.Tensor, group=None):
    """(mean, unbiased std, ddof-0 std) in fp64 of a device vector — over the
    concatenation of every rank's vector when ``group`` spans several ranks
    (the reference takes these moments over the whole test
    set).  Each rank reduces (n, mean, Σ(d − mean)²) locally, one all-gather
    of those 3 doubles follows, and every rank combines them in rank order
    (Chan et al.'s pairwise update): the same numbers on every rank."""
    d = v.to(torch.float64)
    n = d.numel()
    m = d.mean() if n else torch.zeros((), dtype=torch.float64, device=d.device)
    ss = ((d - m) ** 2).sum()
    if _world(group) > 1:
        import torch.distributed as dist

        loc = torch.stack([torch.tensor(float(n), dtype=torch.float64, device=d.device), m, ss])
        parts = [torch.empty_like(loc) for _ in range(_world(group))]
        dist.all_gather(parts, loc, group=group)
        N, mean, s2 = 0.0, 0.0, 0.0
        for part in parts:
            nb, mb, sb = (float(x) for x in part.cpu().numpy())
            if nb == 0:
                continue
            delta = mb - mean
            tot = N + nb
            mean += delta * nb / tot
            s2 += sb + delta * delta * N * nb / tot
            N = tot
        n = int(N)
    else:
        out = torch.stack([m, ss]).cpu().numpy()
        mean, s2 = float(out[0]), float(out[1])
    return mean, math.sqrt(s2 / (n - 1)) if n > 1 else float("nan"), math.sqrt(s2 / n)


def _world(group) -> int:
    """Ranks a statistic spans: 1 unless a process group is passed EXPLICITLY.
    An initialised default group alone never makes a statistic cross-rank —
    the reference's statistics are per call (compute_q_h_f per batch,
    vae_model.py:162-182), so a DDP driver that calls them per rank must get
    per-rank numbers; pass ``group=dist.group.WORLD`` to pool every rank's rows."""
    if group is None:
        return 1
    import torch.distributed as dist

    return dist.get_world_size(group)


def _latent_cov(Z: torch.Tensor, group=None):
    """Column mean (f64) and covariance (f64, ddof 1) of latent rows on the GPU
    — of every rank's rows when ``group`` spans several ranks: every rank's
    Gram about one common shift (``engine.common_shift``), packed as its upper
    triangle (``ocm_gram_pack``) and summed in one all-reduce; a rank without
    rows contributes zeros (nothing of it enters the mean or the shift)."""
    n, d = Z.shape
    if _world(group) == 1:
        shift32 = engine.cast_f32(engine.colmean(Z, None, min(n, engine.SHIFT_SAMPLE)))
        G, cs = engine.gram(Z, None, [0, n], shift32)
        C, mean = engine.cov_from_gram([(1.0, G[0], cs[0])], shift32, n)
        return mean, C
    import torch.distributed as dist

    def allreduce(ts):
        for t in ts:
            dist.all_reduce(t, group=group)

    shift32 = engine.common_shift(Z, None, n, allreduce)
    if n > 0:
        G, cs = engine.gram(Z, None, [0, n], shift32)
        packed = engine.gram_pack(G[0], cs[0], torch.zeros_like(shift32), n)
    else:
        packed = torch.zeros(d * (d + 1) // 2 + d + 1, dtype=torch.float64, device=Z.device)
    dist.all_reduce(packed, group=group)
    C, dvec = engine.cov_from_packed(packed, d)
    return dvec + shift32.to(torch.float64), C


def latent_T2(Z: torch.Tensor, mean64: torch.Tensor, A: torch.Tensor) -> torch.Tensor:
    """T²_i = (z_i − μ)ᵀ A (z_i − μ) (fp64) by the SIMCA scoring kernel with P = I."""
    n, d = Z.shape
    if n == 0:
        return torch.empty(0, dtype=torch.float64, device=Z.device)
    eye = torch.eye(d, dtype=torch.float64, device=Z.device)
    return engine.score(Z, None, n, eye, mean64, A, want_T2=True, want_Q=False)["T2"]


def qhf_device(x: torch.Tensor, x_rec: torch.Tensor, z: torch.Tensor):
    """vae_model.compute_q_h_f on the GPU: returns (q f32, h f32, f f32,
    q_crit, h_crit, f_crit) with the reference's per-batch statistics."""
    xf = engine.as_device_f32(x)
    xr = engine.as_device_f32(x_rec, xf.device)
    zf = engine.as_device_f32(z, xf.device)
    q = engine.rowsq_residual(xf, xr)
    q0, sq, _ = _moments(q)
    Nq = 2 * (q0 / sq) ** 2
    n = zf.shape[0]
    mean, C = _latent_cov(zf)
    A = engine.sym_pinv(C) / (n - 1)
    h64 = latent_T2(zf, mean, A)
    h0, sh, _ = _moments(h64)
    Nh = 2 * (h0 / sh) ** 2
    f = (h64 / h0 * Nh + q.to(torch.float64) / q0 * Nq).to(torch.float32)
    return (q, h64.to(torch.float32), f, stats.chi2.ppf(0.95, df=Nq), stats.chi2.ppf(0.95, df=Nh),
            stats.chi2.ppf(0.95, df=Nh + Nq))


def latent_stats(mus: torch.Tensor, q_cal: torch.Tensor, ridge: float = 1e-6, pct: float = 95.0, group=None):
    """utils/final_vaesimca.py:428-442: (latent mean f64, (cov + ridge·I)⁻¹ f64,
    T² threshold, Q threshold) of the calibration latents / residuals — of
    every rank's rows when ``group`` spans several ranks (all-reduced latent
    Gram, distributed radix-select percentiles)."""
    from .dist import percentile_sharded

    Z = engine.as_device_f32(mus)
    mean, C = _latent_cov(Z, group)
    C.diagonal().add_(ridge)
    inv = engine.sym_pinv(C)  # SPD: the pseudo-inverse is the inverse (np.linalg.inv at :431)
    T2 = latent_T2(Z, mean, inv)
    qd = q_cal if q_cal.dtype in (torch.float32, torch.float64) else q_cal.to(torch.float32)
    if _world(group) > 1:
        import torch.distributed as dist

        cnt = torch.tensor([float(Z.shape[0])], dtype=torch.float64, device=Z.device)
        dist.all_reduce(cnt, group=group)
        n = int(round(float(cnt.item())))
        return mean, inv, percentile_sharded(T2, pct, n, group), percentile_sharded(qd.contiguous(), pct, n, group)
    return mean, inv, engine.percentile(T2, pct), engine.percentile(qd.contiguous(), pct)


def full_distance_decision(mus_test: torch.Tensor, latent_mean: torch.Tensor, q: torch.Tensor, alpha=0.05,
                           group=None):
    """utils/final_vaesimca.py:510-533: accept (bool, device), f (f64), f_crit.
    With ``group`` the test set is the concatenation of every rank's rows: the
    h / q moments are global (one all-gather of 3 doubles each), the decision local."""
    Z = engine.as_device_f32(mus_test)
    h = engine.rowsq_residual(Z, engine.as_device_f32(latent_mean, Z.device).reshape(-1))
    h0, _, sh = _moments(h, group)
    q0, _, sq = _moments(q, group)
    Nh = 2 * (h0 / sh) ** 2
    Nq = 2 * (q0 / sq) ** 2
    f = h.to(torch.float64) / h0 * Nh + q.to(torch.float64) / q0 * Nq
    fcrit = stats.chi2.ppf(1 - alpha, Nh + Nq)
    return f <= fcrit, f, fcrit


def _inv(x) -> float:
    """1/x with NumPy semantics (a zero limit gives inf, as Q/0 in the reference)."""
    with np.errstate(divide="ignore"):
        return float(np.float64(1.0) / np.float64(x))


class VAESIMCA:
    """SIMCA limits on VAE latents (VAE_SIMCA.py:215-382), device-resident.

    ``fit_thresholds(loader, class_label)`` / ``predict(loader)`` keep the
    reference's signatures (loader yields tuples whose first item is a batch
    of spectra) and its percentile-variant limits; ``predict`` returns
    (y_pred bool, T2 f64, Q f32) NumPy arrays like the reference."""

    def __init__(self, vae, type="alt", t2lim="Fdist", t2cl=0.95, qlim="jm", qcl=0.95, dcl=0.95, device="cpu",
                 verbose=True):
        self.vae = vae
        self.device = device
        self.type, self.t2lim, self.t2cl = type, t2lim, t2cl
        self.qlim, self.qcl, self.dcl = qlim, qcl, dcl
        self.verbose = verbose
        self._model = {}
        self.model_class = None

    # -- latent pass ------------------------------------------------------
    @torch.no_grad()
    def _latents(self, loader):
        """μ and the round trip ẑ = enc(dec(μ)) for every batch (device f32)."""
        v = self.vae
        mus, zhats = [], []
        for xb in loader:
            x = xb[0].to(self.device)
            mu, _ = v.encode((x - v.spec_mean) / v.spec_std)
            z_hat, _ = v.encode((v.decode(mu) - v.spec_mean) / v.spec_std)
            mus.append(mu.float())
            zhats.append(z_hat.float())
        return torch.cat(mus).contiguous(), torch.cat(zhats).contiguous()

    @torch.no_grad()
    def fit_thresholds(self, loader, class_label=0):
        self.vae.eval()
        Z, Zh = self._latents(loader)
        self.fit_latents(Z, Zh, class_label)

    def fit_latents(self, Z: torch.Tensor, Zh: torch.Tensor, class_label=0):
        """The statistics part of ``fit_thresholds`` on given latents μ and
        round trips ẑ (device or host arrays, (n, d))."""
        self.model_class = [class_label]
        Z = engine.as_device_f32(Z)
        Zh = engine.as_device_f32(Zh, Z.device)
        n, nc = Z.shape
        mean, C = _latent_cov(Z)
        C.diagonal().add_(1e-12)
        invcov = engine.sym_pinv(C)
        T2 = latent_T2(Z, mean, invcov)
        Q = engine.rowsq_residual(Z, Zh)
        T2_limit, t2dof, t2scfact = self._t2_limit(T2, nc)
        Q_limit, qdof, qscfact = self._q_limit(Q)
        D_limit = self._d_limit(T2_limit, Q_limit, Q, nc, t2dof, qdof)
        self._model[class_label] = {
            "latent_mean": mean.cpu().numpy(), "invcovT": invcov.cpu().numpy(), "T2": T2.cpu().numpy(),
            "Q": Q.cpu().numpy(), "T2_limit": T2_limit, "Q_limit": Q_limit, "D_limit": D_limit, "T2dof": t2dof,
            "T2scfact": t2scfact, "Qdof": qdof, "Qscfact": qscfact, "n_components": nc,
            "_mean_dev": mean, "_invcov_dev": invcov,
        }

    # -- limits (VAE_SIMCA.py:281-346) -----------------------------------
    def _t2_limit(self, T2, nc):
        if self.t2lim not in ("perc", "chi2", "Fdist", "chi2pom"):
            raise ValueError(f"T2 limit type {self.t2lim} not implemented")
        n = T2.numel()
        if self.t2lim in ("perc", "chi2"):
            return engine.percentile(T2, self.t2cl * 100), None, None
        if self.t2lim == "Fdist":
            F_value = engine.percentile(T2, self.t2cl * 100)
            return nc * (n - 1) / (n - nc) * F_value, None, None
        if self.t2lim == "chi2pom":
            h0, sd, _ = _moments(T2)
            var = sd * sd if n > 1 else 0.0
            Nh = max(int(np.round(2 * (h0 ** 2) / var)) if var > 0 else 1, 1)
            return h0 * engine.percentile(T2, self.t2cl * 100) / Nh, Nh, h0
        raise ValueError(f"T2 limit type {self.t2lim} not implemented")

    def _q_limit(self, Q):
        if self.qlim == "perc":
            return engine.percentile(Q, self.qcl * 100), None, None
        if self.qlim == "jm":
            qd = Q.to(torch.float64)
            th = torch.stack([qd.sum(), (qd ** 2).sum(), (qd ** 3).sum()]).cpu().numpy()
            th1, th2, th3 = (float(v) for v in th)
            if th1 == 0:
                return 0, None, None
            h0 = max(1 - (2 * th1 * th3) / (3 * th2 ** 2), 1e-3)
            ca = np.sqrt(2) * special.erfinv(2 * self.qcl - 1)
            h1 = ca * np.sqrt(2 * th2 * h0 ** 2) / th1
            h2 = th2 * h0 * (h0 - 1) / (th1 ** 2)
            return th1 * (1 + h1 + h2) ** (1 / h0), None, None
        if self.qlim == "chi2pom":
            v0, sd, _ = _moments(Q)
            Nv = max(round(2 * (v0 ** 2) / (sd * sd)), 1)
            return v0 * engine.percentile(Q, self.qcl * 100) / Nv, Nv, v0
        raise ValueError(f"Q limit type {self.qlim} not implemented")

    def _d_limit(self, T2_limit, Q_limit, Q, nc, t2dof, qdof):
        if self.type == "sim":
            return 1
        if self.type == "alt":
            return np.sqrt(2)
        if self.type == "ci":
            qd = Q.to(torch.float64)
            s = torch.stack([qd.sum(), (qd ** 2).sum()]).cpu().numpy()
            tr1 = nc / T2_limit + float(s[0]) / Q_limit
            tr2 = nc / T2_limit ** 2 + float(s[1]) / Q_limit ** 2
            return tr2 / tr1 * engine.percentile(Q, self.dcl * 100)
        if self.type == "dd":
            if t2dof is None or qdof is None:
                raise ValueError("t2dof/qdoff must be set for dd")
            return t2dof + qdof
        raise ValueError(f"D type {self.type} not implemented")

    # -- decision (VAE_SIMCA.py:348-382) --------------------------------
    @torch.no_grad()
    def predict(self, loader):
        self.vae.eval()
        Z, Zh = self._latents(loader)
        return self.predict_latents(Z, Zh)

    def predict_latents(self, Z: torch.Tensor, Zh: torch.Tensor):
        """The decision part of ``predict`` on given latents μ / round trips ẑ."""
        info = self._model[self.model_class[0]]
        Z = engine.as_device_f32(Z)
        Zh = engine.as_device_f32(Zh, Z.device)
        T2 = latent_T2(Z, info["_mean_dev"], info["_invcov_dev"])
        Q = engine.rowsq_residual(Z, Zh)
        if self.type == "alt":
            dec = engine.make_decision("alt", _inv(info["T2_limit"]), _inv(info["Q_limit"]), info["D_limit"])
        elif self.type == "dd":
            dec = engine.make_decision("dd", info["T2dof"] / info["T2scfact"], info["Qdof"] / info["Qscfact"],
                                       info["D_limit"])
        else:  # sim and ci both take max(T2/T2lim, Q/Qlim) here (VAE_SIMCA.py:377-378)
            dec = engine.make_decision("sim", _inv(info["T2_limit"]), _inv(info["Q_limit"]), info["D_limit"])
        acc = torch.empty(Z.shape[0], dtype=torch.float64, device=Z.device)
        engine.decide(T2, Q, dec, want_red=False, accept_out=acc)
        return acc.cpu().numpy() > 0.5, T2.cpu().numpy(), Q.cpu().numpy()
