"""Diagnostic: count non-finite VAE graph-training runs (bench shape) under a
mode: 'base', 'foreach_zero' (grads zeroed by a foreach kernel instead of
memset nodes)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
import vae_model as V  # noqa: E402
from bench import synth_device  # noqa: E402
import ocm.vae_train as vt  # noqa: E402

mode = sys.argv[1]
if mode == "foreach_zero":
    def zg(self, set_to_none=False):
        gs = [p.grad for g in self.param_groups for p in g["params"] if p.grad is not None]
        if gs:
            torch._foreach_zero_(gs)
    torch.optim.Adam.zero_grad = zg
dev = torch.device("cuda", 0)
B, L, nb = 512, 2048, 16
X = synth_device(B * nb, L, 20, seed=99, device=dev)
mean = X.mean(0).cpu().numpy()
std = X.std(0).cpu().numpy() + 1e-6
res = []
for rep in range(6):
    torch.manual_seed(0)
    m = V.ConvVAE1D(L, 32, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
    tr = vt.GraphedVAETrainer(m, B, lr=1e-3, dtype=torch.bfloat16)
    losses = torch.zeros(210, device=dev)
    for i in range(210):
        out = tr.step(X[(i % nb) * B:(i % nb + 1) * B])
        losses[i].copy_(out[0])
        if i == 9 or (rep % 2 and (i + 1) % 25 == 0):
            torch.cuda.synchronize()
    l = losses.cpu()
    bad = torch.nonzero(~torch.isfinite(l)).flatten()
    res.append(int(bad[0]) if len(bad) else None)
print(mode, os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE"), "first non-finite per rep:", res, flush=True)
