#!/usr/bin/env python3
"""A/B of the bf16 VAE step's bottleneck Linear layers: vae_fused.linear_act
(one libocm launch for each layer's ELU + bias gradient) against torch's
autocast Linear + ELU (ocm.vae_train.LINEAR_FUSED = False), the bench's VAE
line (C4, B = 512, L = 2048, HIP graph) in alternating child processes.

    python scripts/vae_linear_ab.py [--steps 300] [--rounds 2]
"""
import argparse
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = """
import json, os, sys
sys.path.insert(0, {repo!r}); sys.path.insert(0, os.path.join({repo!r}, "ocm-vae-simca_amd"))
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")
import ocm.vae_train as vt
vt.LINEAR_FUSED = {fused}
import torch
from bench import vae_bench
r = vae_bench(torch.device("cuda", 0), {steps}, 10, latent_rows=0)
print(json.dumps({{"linear_fused": {fused}, "steps_per_s": r["value"] if "value" in r else r}}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    for _ in range(a.rounds):
        for fused in (True, False):
            code = CHILD.format(repo=REPO, fused=fused, steps=a.steps)
            r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
            if r.returncode != 0:
                sys.exit(r.stderr[-3000:])
            print(r.stdout.strip().splitlines()[-1], flush=True)


if __name__ == "__main__":
    main()
