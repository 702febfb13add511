"""Importable pieces of the reference's cheese VAE sweep, utils/final_vaesimca.py.

The reference script is not importable (it loads a private ``.mat`` at import,
utils/final_vaesimca.py:230-231); what a driver reuses from it lives here with
the same names and semantics, on the MI355X engine:

* ``ConvVAE1D`` — the script's own copy of the network (:72-193): the
  vae_model network with its buffer layout, ``threshold`` and ``q_threshold``
  (:95-96) instead of ``threshold_q/h/f``, so a checkpoint the script saves
  (``VAE_class0_best.pth``, :445) loads strictly;
* the three losses (:198-224): ``beta_vae_cosine_loss``,
  ``beta_vae_euclidean_loss`` and ``beta_vae_bce_loss`` — the script's BCE is
  a PROBABILITY BCE of the min-max scaled reconstruction, unlike
  vae_model.beta_vae_bce_loss (BCE-with-logits); the graph-captured trainer
  takes them as ``loss="cosine" | "euclidean" | "bce_prob"``
  (ocm.vae_train.GraphedVAETrainer);
* ``rec_error`` — the calibration / test Q (:417-425, :484-492): the per-sample
  min-max scaled residual for ``"X_bce"`` (libocm ``ocm_rowsq_minmax_f32``),
  the plain one otherwise (``ocm_rowsq_residual_f32``);
* ``calibrate`` — the best-epoch latent statistics (:406-442): latent mean,
  (cov + 1e-6·I)⁻¹, the 95th-percentile Mahalanobis threshold and Q threshold,
  written into the network's buffers;
* ``score`` — the test pass and the full-distance decision (:474-533).
"""
from __future__ import annotations

import numpy as np
import torch

import vae_model as _vm
from ocm import engine
from ocm.vae import full_distance_decision, latent_stats, latent_T2

__all__ = ["ConvVAE1D", "beta_vae_cosine_loss", "beta_vae_euclidean_loss", "beta_vae_bce_loss", "rec_error",
           "calibrate", "score", "LOSS_FOR"]

# the script's loss_type names → the trainer's loss names
LOSS_FOR = {"X_cosine": "cosine", "X_euclidean": "euclidean", "X_bce": "bce_prob"}


class ConvVAE1D(_vm.ConvVAE1D):
    """utils/final_vaesimca.py:72-193 (same constructor and network as
    vae_model.ConvVAE1D; buffers ``threshold``, ``q_threshold``)."""

    THRESHOLD_BUFFERS = ("threshold", "q_threshold")


def beta_vae_cosine_loss(x, x_recon, mu, logvar, beta=1.0, eps=1e-8):
    """utils/final_vaesimca.py:198-206 (= vae_model's)."""
    return _vm.beta_vae_cosine_loss(x, x_recon, mu, logvar, beta=beta, eps=eps)


def beta_vae_euclidean_loss(x, x_recon, mu, logvar, beta=1.0):
    """utils/final_vaesimca.py:208-211: MSE + β·KL."""
    recon = _vm.mse_recon_term(x, x_recon)
    kl = _vm.kl_term(mu, logvar)
    return recon + beta * kl, recon.detach().cpu().item(), kl.detach().cpu().item()


def beta_vae_bce_loss(x, x_recon, mu, logvar, beta=1.0, eps=1e-8):
    """utils/final_vaesimca.py:213-224: probability BCE of the min-max scaled
    reconstruction (clamped to [0, 1]) + β·KL."""
    recon = _vm.bce_prob_recon_term(x, x_recon, eps)
    kl = _vm.kl_term(mu, logvar)
    return recon + beta * kl, recon.detach().cpu().item(), kl.detach().cpu().item()


def rec_error(x: torch.Tensor, x_rec: torch.Tensor, loss_type: str) -> torch.Tensor:
    """Per-row reconstruction error Q (float32, device): min-max scaled for
    ``"X_bce"`` (:417-423, :484-490), plain Σ(x − x̂)² otherwise (:425, :492)."""
    xf = engine.as_device_f32(x)
    xr = engine.as_device_f32(x_rec, xf.device)
    if loss_type == "X_bce":
        return engine.rowsq_minmax(xf, xr, 1e-8)
    return engine.rowsq_residual(xf, xr)


def _batches(X, batch):
    n = X.shape[0]
    for a in range(0, n, batch):
        yield X[a:a + batch]


@torch.no_grad()
def _latents_and_q(vae, X, loss_type, batch):
    """μ of every row (encoder on the standardised spectra) and the Q of the
    network's own (stochastic, as the reference's eval-mode forward) reconstruction."""
    Xd = engine.as_device_f32(X, next(vae.parameters()).device)
    mus, qs = [], []
    for x in _batches(Xd, batch):
        mu, _ = vae.encode((x - vae.spec_mean) / vae.spec_std)
        x_rec, _, _ = vae(x)
        mus.append(mu.float())
        qs.append(rec_error(x, x_rec.float(), loss_type))
    return torch.cat(mus), torch.cat(qs)


def calibrate(vae, X_cal, loss_type: str = "X_bce", batch: int = 512, group=None):
    """utils/final_vaesimca.py:406-442 on the device: the calibration latents'
    mean and (cov + 1e-6·I)⁻¹, the 95th percentiles of their Mahalanobis T² and
    of Q; written to the buffers ``latent_mean``, ``latent_cov_inv``,
    ``threshold``, ``q_threshold`` (float32, as the script copies them).
    Returns (mean f64, cov_inv f64, threshold, q_threshold)."""
    vae.eval()
    mus, q = _latents_and_q(vae, X_cal, loss_type, batch)
    mean, inv, thr, qthr = latent_stats(mus, q, ridge=1e-6, pct=95.0, group=group)
    with torch.no_grad():
        vae.latent_mean.copy_(mean.to(torch.float32))
        vae.latent_cov_inv.copy_(inv.to(torch.float32))
        vae.threshold.copy_(torch.tensor(thr, dtype=torch.float32))
        if hasattr(vae, "q_threshold"):
            vae.q_threshold.copy_(torch.tensor(qthr, dtype=torch.float32))
    return mean, inv, thr, qthr


def score(vae, X_test, loss_type: str = "X_bce", batch: int = 512, alpha: float = 0.05, group=None):
    """utils/final_vaesimca.py:474-533: the test Mahalanobis d² against the
    stored latent statistics (buffers, float32 as the script reads them), the
    test Q, and the full-distance decision (Euclidean h, test-set moments).
    Returns dict(d2, q, accept, f, fcrit) with device tensors (fcrit a float)."""
    vae.eval()
    mus, q = _latents_and_q(vae, X_test, loss_type, batch)
    mean32 = vae.latent_mean.to(torch.float64)
    inv32 = vae.latent_cov_inv.to(torch.float64).contiguous()
    d2 = latent_T2(mus, mean32, inv32)
    accept, f, fcrit = full_distance_decision(mus, vae.latent_mean, q, alpha=alpha, group=group)
    return {"d2": d2, "q": q, "accept": accept, "f": f, "fcrit": float(fcrit), "mu": mus}


def as_numpy(out: dict) -> dict:
    return {k: (v.cpu().numpy() if isinstance(v, torch.Tensor) else np.asarray(v)) for k, v in out.items()}
