"""Diagnostic: VAE training loss trajectory on the GPU in four modes
(fp32 / bf16 autocast × eager / HIP-graph) on the bench's C4 network."""
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
for dtype, graph, restore in ((torch.float32, False, True), (torch.float32, True, True), (torch.float32, True, False),
                              (torch.bfloat16, False, True), (torch.bfloat16, True, True),
                              (torch.bfloat16, True, False)):
    if True:
        torch.manual_seed(0)
        m = V.ConvVAE1D(L, 32, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
        tr = GraphedVAETrainer(m, B, lr=1e-3, dtype=dtype, graph=graph, restore=restore)
        traj = []
        for i in range(400):
            out = tr.step(X[(i % nb) * B:(i % nb + 1) * B])
            if i % 25 == 0 or i == 399:
                traj.append(round(float(out[0]), 4))
        bad = [n for n, p in m.named_parameters() if not torch.isfinite(p).all()]
        print(f"{str(dtype):15s} graph={graph!s:5s} restore={restore!s:5s} loss {traj}  nonfinite params: {bad[:4]}", flush=True)
