"""Drop-in for the reference's ``vae_model`` (vae_model.py:1-182).

``ConvVAE1D``, ``beta_vae_bce_loss``, ``beta_vae_cosine_loss`` and
``compute_q_h_f`` keep the reference's names, signatures, buffers and
state_dict layout (a checkpoint written by either loads into the other), and
the same seeded initialisation.  The network stays a PyTorch-ROCm module
(narrow Conv1d / BN / ELU / Linear layers are launch-bound,
not MFMA targets); its convolutions (``ocm.conv``) and training-mode batch
norms (``ocm.bn``) run libocm's direct HIP kernels on the GPU instead of
MIOpen, with the stock modules' parameters and state_dict keys; the training
step is captured in a HIP graph by ``ocm.vae_train``.  The latent statistics of ``compute_q_h_f`` (residual q,
leverage h) run on libocm's HIP kernels when the tensors live on the GPU
(``ocm.vae.qhf_device``): the same Gram / pseudo-inverse / quadratic-form
kernels as SIMCA at p = d.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from ocm.bn import FastBatchNorm1d
from ocm.conv import FastConv1d, FastConvTranspose1d

__all__ = ["ConvVAE1D", "beta_vae_cosine_loss", "beta_vae_bce_loss", "compute_q_h_f"]


def _conv_out_len(n: int, k: int, s: int, pad: int) -> int:
    return (n + 2 * pad - (k - 1) - 1) // s + 1


def _optional_dropout(p: float) -> nn.Module:
    return nn.Dropout(p) if p > 0 else nn.Identity()


class ConvVAE1D(nn.Module):
    """1-D convolutional β-VAE on standardised spectra (vae_model.py:6-129).

    Encoder: ``conv_blocks`` × [Conv1d (stride 1 for the first block, then
    ``stride``) → BN → act (→ Dropout)], filters doubling (≤ 1024) → flatten →
    Linear(hidden_fc) → act → μ, logσ².  Decoder mirrors it with
    ConvTranspose1d (stride on all but the last block, filters halving, ≥
    n_filters) and a final 1×1 Conv1d, cropped / zero-padded to
    ``input_length``.  ``forward`` standardises with the ``spec_mean`` /
    ``spec_std`` buffers, samples z = μ + ε·exp(½logσ²) (also in eval, as the
    reference) and de-standardises the reconstruction.
    """

    # decision thresholds travel with checkpoints (vae_model.py:29-32); the
    # copy in utils/final_vaesimca.py:95-96 carries ("threshold", "q_threshold")
    THRESHOLD_BUFFERS = ("threshold", "threshold_q", "threshold_h", "threshold_f")

    def __init__(self, input_length, latent_dim, mean, std, conv_blocks=3, n_filters=32, kernel_size=9, stride=2,
                 hidden_fc=256, activation="elu", dropout=0.0, use_batchnorm=True, beta=1.0):
        super().__init__()
        self.input_length = input_length
        self.latent_dim = latent_dim
        self.beta = beta
        self.dropout = dropout
        self.use_batchnorm = use_batchnorm
        for name in self.THRESHOLD_BUFFERS:
            self.register_buffer(name, torch.tensor(0.0))

        act_cls = nn.ELU if activation == "elu" else nn.GELU
        pad = kernel_size // 2

        # ---- encoder convolutions: channel plan and output length ----
        layers, chans, length, c_in = [], n_filters, input_length, 1
        for b in range(conv_blocks):
            s_b = 1 if b == 0 else stride
            layers += self._block(FastConv1d(c_in, chans, kernel_size, stride=s_b, padding=pad), chans, act_cls)
            c_in, length = chans, _conv_out_len(length, kernel_size, s_b, pad)
            chans = min(chans * 2, 1024)
        self.encoder_conv = nn.Sequential(*layers)
        self._enc_out_channels = c_in
        self._enc_out_length = length
        flat = c_in * length

        # ---- bottleneck ----
        self.fc = nn.Sequential(nn.Linear(flat, hidden_fc), act_cls(), _optional_dropout(dropout))
        self.fc_mu = nn.Linear(hidden_fc, latent_dim)
        self.fc_logvar = nn.Linear(hidden_fc, latent_dim)
        self.fc_dec = nn.Sequential(nn.Linear(latent_dim, hidden_fc), act_cls(), _optional_dropout(dropout),
                                    nn.Linear(hidden_fc, flat), act_cls())

        # ---- decoder transposed convolutions ----
        layers, chans = [], c_in
        for b in range(conv_blocks):
            nxt = max(chans // 2, n_filters)
            s_b = stride if b < conv_blocks - 1 else 1
            layers += self._block(FastConvTranspose1d(chans, nxt, kernel_size, stride=s_b, padding=pad,
                                                      output_padding=s_b - 1), nxt, act_cls)
            chans = nxt
        layers.append(FastConv1d(chans, 1, kernel_size=1))
        self.decoder_conv = nn.Sequential(*layers)

        self.register_buffer("spec_mean", torch.tensor(mean, dtype=torch.float32))
        self.register_buffer("spec_std", torch.tensor(std, dtype=torch.float32))
        self.register_buffer("latent_mean", torch.zeros(latent_dim))
        self.register_buffer("latent_cov_inv", torch.eye(latent_dim))
        self._init_weights()

    def _block(self, conv: nn.Module, chans: int, act_cls) -> list:
        mods = [conv]
        if self.use_batchnorm and act_cls is nn.ELU:
            # nn.BatchNorm1d + ELU in libocm's training kernels on HIP tensors; the
            # Identity keeps the ELU's slot, so the state_dict keys do not move
            mods += [FastBatchNorm1d(chans).fuse_elu(), nn.Identity()]
        elif self.use_batchnorm:
            mods += [FastBatchNorm1d(chans), act_cls()]
        else:
            mods.append(act_cls())
        if self.dropout > 0:
            mods.append(nn.Dropout(self.dropout))
        return mods

    def _init_weights(self):
        """Kaiming-normal (gain 1) weights, zero biases (vae_model.py:90-96)."""
        for mod in self.modules():
            if isinstance(mod, (nn.Conv1d, nn.ConvTranspose1d, nn.Linear)):
                nn.init.kaiming_normal_(mod.weight, nonlinearity="linear")
                if mod.bias is not None:
                    nn.init.zeros_(mod.bias)

    def encode(self, x):
        h = self.encoder_conv(x.unsqueeze(1)).flatten(1)
        h = self.fc(h)
        return self.fc_mu(h), self.fc_logvar(h)

    def reparameterize(self, mu, logvar):
        return mu + torch.randn_like(mu) * torch.exp(0.5 * logvar)

    def decode(self, z):
        h = self.fc_dec(z).view(z.shape[0], self._enc_out_channels, self._enc_out_length)
        x = self.decoder_conv(h).squeeze(1)
        L = self.input_length
        if x.shape[-1] > L:
            x = x[..., :L]
        elif x.shape[-1] < L:
            x = F.pad(x, (0, L - x.shape[-1]))
        return x

    def forward(self, x):
        mu, logvar = self.encode((x - self.spec_mean) / self.spec_std)
        x_rec_std = self.decode(self.reparameterize(mu, logvar))
        return x_rec_std * self.spec_std + self.spec_mean, mu, logvar


# ---------------------------------------------------------------------------
# losses (vae_model.py:136-158): the tensor-valued parts are shared with the
# graph-captured trainer (ocm/vae_train.py), which must not call .item()
# ---------------------------------------------------------------------------

def kl_term(mu, logvar):
    """−½ · mean_B Σ_d (1 + logσ² − μ² − σ²)."""
    return -0.5 * torch.mean(torch.sum(1 + logvar - mu.pow(2) - logvar.exp(), dim=1))


def bce_recon_term(x, x_recon, eps=1e-8):
    """BCE-with-logits of the (de-standardised) reconstruction against the
    per-sample min-max scaled input."""
    lo = x.min(dim=1, keepdim=True)[0]
    hi = x.max(dim=1, keepdim=True)[0]
    target = ((x - lo) / (hi - lo + eps)).clamp(0.0, 1.0)
    return F.binary_cross_entropy_with_logits(x_recon.reshape(x_recon.shape[0], -1),
                                              target.reshape(target.shape[0], -1), reduction="mean")


def _minmax_scaled(x, v, eps):
    lo = x.min(dim=1, keepdim=True)[0]
    hi = x.max(dim=1, keepdim=True)[0]
    return ((v - lo) / (hi - lo + eps)).clamp(0.0, 1.0)


def bce_prob_recon_term(x, x_recon, eps=1e-8):
    """utils/final_vaesimca.py:213-221: probability BCE of the reconstruction
    and the input, both min-max scaled by the input's per-sample range."""
    return F.binary_cross_entropy(_minmax_scaled(x, x_recon, eps), _minmax_scaled(x, x, eps), reduction="mean")


def mse_recon_term(x, x_recon):
    """utils/final_vaesimca.py:208-209: mean squared error."""
    return F.mse_loss(x_recon, x, reduction="mean")


def cosine_recon_term(x, x_recon, eps=1e-8):
    """mean_B √(2(1 − cos θ)) with cos θ clamped to (−1+eps, 1−eps)."""
    a = F.normalize(x.reshape(x.shape[0], -1), p=2, dim=1)
    b = F.normalize(x_recon.reshape(x_recon.shape[0], -1), p=2, dim=1)
    cos = torch.clamp((a * b).sum(dim=1), -1.0 + eps, 1.0 - eps)
    return torch.mean(torch.sqrt(2.0 * (1.0 - cos)))


def beta_vae_cosine_loss(x, x_recon, mu, logvar, beta=1.0, eps=1e-8):
    recon = cosine_recon_term(x, x_recon, eps)
    kl = kl_term(mu, logvar)
    return recon + beta * kl, recon.detach().cpu().item(), kl.detach().cpu().item()


def beta_vae_bce_loss(x, x_recon, mu, logvar, beta=1.0, eps=1e-8):
    recon = bce_recon_term(x, x_recon, eps)
    kl = kl_term(mu, logvar)
    return recon + beta * kl, recon.detach().cpu().item(), kl.detach().cpu().item()


# ---------------------------------------------------------------------------
# χ² distances (vae_model.py:162-182)
# ---------------------------------------------------------------------------

def compute_q_h_f(x, x_rec, z):
    """q = Σ(x − x̂)², leverage h of the column-standardised latent, f = h/h0·Nh
    + q/q0·Nq and the χ²₀.₉₅ criticals with moment-matched dof (unbiased
    std).  Per-batch statistics, as the reference.  The arithmetic runs on
    libocm (ocm.vae.qhf_device); host tensors are copied to the device and
    the per-row results come back to the host, like the reference's own
    return device.  There is no CPU path: without a HIP device this raises."""
    from ocm.vae import qhf_device

    host = not x.is_cuda
    q, h, f, q_crit, h_crit, f_crit = qhf_device(x, x_rec, z)
    if host:
        q, h, f = q.cpu(), h.cpu(), f.cpu()
    return q, h, f, q_crit, h_crit, f_crit
