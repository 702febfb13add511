"""Synthetic spectra generated in HBM, shard by shard.

C5 (VAE-SIMCA DDP, 10M × 4096 fp32 = 164 GB) does not fit in host RAM, so
each rank generates its own contiguous row block on its GPU with torch's
device generator (counter-based Philox4x32-10).  Rows come in fixed chunks
whose generator seed depends only on (seed, chunk index): the global matrix
is the same for any world size, and a rank only generates the chunks that
overlap its rows.

The model is the survey's (§8d synthetic inputs): rank-``rank_count``
Gaussian absorption bands (shared loadings, from ``seed``), scores with a
gap at ``k`` (s = linspace(20, 8, k) ++ linspace(2, 0.5, r − k)), σ-noise
and a sloped baseline 1 + 0.3·λ.
"""
from __future__ import annotations

import torch

__all__ = ["shard_bounds", "spectra_shard", "band_loadings"]

CHUNK = 65536  # rows per generator chunk (the unit of reproducibility)


def shard_bounds(n_total: int, rank: int, world: int) -> tuple[int, int]:
    """Contiguous, balanced row block [lo, hi) of ``rank``."""
    base, extra = divmod(n_total, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def band_loadings(p: int, seed: int, device, rank_count: int = 40) -> torch.Tensor:
    """(rank_count, p) unit-norm Gaussian bands, identical on every rank."""
    g = torch.Generator(device=device).manual_seed(seed)
    wl = torch.linspace(0.0, 1.0, p, device=device, dtype=torch.float64)
    centers = torch.rand(rank_count, generator=g, device=device, dtype=torch.float64) * 0.9 + 0.05
    widths = torch.rand(rank_count, generator=g, device=device, dtype=torch.float64) * 0.07 + 0.01
    L = torch.exp(-0.5 * ((wl[None, :] - centers[:, None]) / widths[:, None]) ** 2)
    return (L / L.norm(dim=1, keepdim=True)).float()


def spectra_shard(n_total: int, p: int, rank: int, world: int, device, seed: int = 1234, k: int = 20,
                  rank_count: int = 40, noise: float = 0.05, out: torch.Tensor | None = None) -> torch.Tensor:
    """This rank's rows [lo, hi) of the global synthetic matrix (float32, HBM)."""
    lo, hi = shard_bounds(n_total, rank, world)
    L = band_loadings(p, seed, device, rank_count)
    s = torch.cat([torch.linspace(20, 8, k), torch.linspace(2, 0.5, rank_count - k)]).to(device)
    base = (1.0 + 0.3 * torch.linspace(0.0, 1.0, p, device=device, dtype=torch.float64)).float()
    X = out if out is not None else torch.empty((hi - lo, p), dtype=torch.float32, device=device)
    g = torch.Generator(device=device)
    for c in range(lo // CHUNK, (hi + CHUNK - 1) // CHUNK):
        c0, c1 = c * CHUNK, min((c + 1) * CHUNK, n_total)
        a, b = max(c0, lo), min(c1, hi)
        if a >= b:
            continue
        g.manual_seed(seed * 1_000_003 + c + 1)  # depends on (seed, chunk) only
        S = torch.randn((c1 - c0, rank_count), generator=g, device=device) * s
        E = torch.randn((c1 - c0, p), generator=g, device=device)
        blk = torch.addmm(base.expand(c1 - c0, p), S, L).add_(E, alpha=noise)
        X[a - lo:b - lo] = blk[a - c0:b - c0]
    return X
