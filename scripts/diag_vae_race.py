"""Diagnostic: bench-style VAE graph training with different host sync
cadences; reports the first non-finite loss step."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
import vae_model as V  # noqa: E402
from bench import synth_device  # noqa: E402
from ocm.vae_train import GraphedVAETrainer  # noqa: E402

dev = torch.device("cuda", 0)
B, L, nb = 512, 2048, 16
X = synth_device(B * nb, L, 20, seed=99, device=dev)
mean = X.mean(0).cpu().numpy()
std = X.std(0).cpu().numpy() + 1e-6
for sync_every in (1, 25, 1000):
    for graph in (True, False):
        torch.manual_seed(0)
        m = V.ConvVAE1D(L, 32, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
        tr = GraphedVAETrainer(m, B, lr=1e-3, dtype=torch.bfloat16, graph=graph)
        losses = torch.zeros(210, device=dev)
        for i in range(210):
            out = tr.step(X[(i % nb) * B:(i % nb + 1) * B])
            losses[i].copy_(out[0])
            if (i + 1) % sync_every == 0:
                torch.cuda.synchronize()
        l = losses.cpu()
        bad = torch.nonzero(~torch.isfinite(l)).flatten()
        b0 = int(bad[0]) if len(bad) else None
        print(f"sync_every={sync_every} graph={graph} first_nonfinite={b0} loss[9]={float(l[9]):.4f} "
              f"loss[-1]={float(l[-1]):.4f} around={[round(float(v), 3) for v in l[max(0, (b0 or 0) - 3):(b0 or 0) + 2]]}",
              flush=True)
