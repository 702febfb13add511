"""Diagnostic: does the SIMCA phase of bench.py disturb the VAE that trains
after it in the same process?  mode: "vae" (VAE only), "simca+vae" (bench
order), "canary" (SIMCA with 1 GiB canary tensors allocated around it,
checked afterwards, then the VAE)."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
from bench import synth_device, vae_bench  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
if mode in ("simca+vae", "canary"):
    from ocm.dist import ShardedSIMCA

    can = []
    if mode == "canary":
        can.append(torch.full((1 << 28,), 1.2345, device=dev))
    X = synth_device(1_000_000, 2048, 20, seed=4321, device=dev)
    if mode == "canary":
        can.append(torch.full((1 << 28,), 1.2345, device=dev))
    pred = torch.empty(1_000_000, dtype=torch.float64, device=dev)
    for _ in range(3):
        m = ShardedSIMCA(n_components=20, type="alt", t2lim="Fdist", qlim="jm").fit(X)
        m.predict(X, out=pred)
    torch.cuda.synchronize()
    print("simca T2_limit", m.T2_limit, "Q_limit", m.Q_limit, "accept", float(pred.mean()), "iters", m.fit_.eig_iters)
    for i, c in enumerate(can):
        print("canary", i, "intact", bool((c == 1.2345).all()))
    del X, pred
r = vae_bench(dev, 200, 10)
print(mode, {k: r[k] for k in ("value", "loss_after_warmup", "final_loss", "params_finite")}, flush=True)
