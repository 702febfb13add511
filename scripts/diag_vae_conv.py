"""Diagnostic: encoder μ of the drop-in ConvVAE1D on the GPU vs the reference
network's μ on the CPU (tests/golden/vae_*.npz) under different convolution
backend settings."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
import vae_model as V  # noqa: E402

for name in ("vae_a.npz", "vae_b.npz"):
    g = dict(np.load(os.path.join(REPO, "tests", "golden", name)))
    cfg = json.loads(str(g["config_json"]))
    L, d = cfg.pop("input_length"), cfg.pop("latent_dim")
    m = V.ConvVAE1D(L, d, g["mean"], g["std"], **cfg)
    m.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd/")})
    m = m.cuda().eval()
    xs = torch.from_numpy(g["x_cal"]).cuda()
    ref = g["mu_cal"]
    for label, setup in [("default", {}), ("no_tf32", {"allow_tf32": False}),
                         ("deterministic", {"allow_tf32": False, "deterministic": True, "benchmark": False}),
                         ("cudnn_off", {"enabled": False})]:
        saved = {k: getattr(torch.backends.cudnn, k) for k in ("enabled", "allow_tf32", "deterministic", "benchmark")}
        for k, v in setup.items():
            setattr(torch.backends.cudnn, k, v)
        with torch.no_grad():
            h = m.encoder_conv(((xs - m.spec_mean) / m.spec_std).unsqueeze(1))
            mu, _ = m.encode((xs - m.spec_mean) / m.spec_std)
        # conv-only check against the same layers on the CPU
        with torch.no_grad():
            hc = m.cpu().encoder_conv(((xs.cpu() - m.spec_mean) / m.spec_std).unsqueeze(1))
        m.cuda()
        err = np.abs(mu.cpu().numpy() - ref).max() / np.abs(ref).max()
        herr = (h.cpu() - hc).abs().max().item() / hc.abs().max().item()
        print(f"{name} {label:14s} mu rel err {err:.3e}  encoder_conv rel err {herr:.3e}")
        for k, v in saved.items():
            setattr(torch.backends.cudnn, k, v)
