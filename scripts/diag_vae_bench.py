"""Diagnostic: call bench.vae_bench itself, with GraphedVAETrainer.step
wrapped to record every loss on the device."""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
import bench  # noqa: E402
import ocm.vae_train as vt  # noqa: E402

dev = torch.device("cuda", 0)
records = []
orig = vt.GraphedVAETrainer.step


def step(self, x=None):
    out = orig(self, x)
    buf = records[-1]
    buf.append(out[0].detach().clone())
    return out


vt.GraphedVAETrainer.step = step
for rep in range(2):
    records.append([])
    r = bench.vae_bench(dev, 200, 10)
    losses = torch.stack(records[-1]).cpu()
    bad = torch.nonzero(~torch.isfinite(losses)).flatten()
    b0 = int(bad[0]) if len(bad) else None
    print(f"rep {rep}: final {r['final_loss']} finite {r['params_finite']} first_nonfinite_step {b0} "
          f"around {[round(float(v), 4) for v in losses[max(0, (b0 or 0) - 4):(b0 or 0) + 1]]}", flush=True)
