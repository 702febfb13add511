"""Profiling driver: the Gram (default mode, or OCM_GRAM_MODE) on the bench
workload (1M×2048 fp32 in HBM), --reps launches."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=1_000_000)
ap.add_argument("--p", type=int, default=2048)
ap.add_argument("--reps", type=int, default=3)
args = ap.parse_args()
import torch  # noqa: E402

from bench import synth_device  # noqa: E402
from ocm import engine  # noqa: E402

X = synth_device(args.rows, args.p, 20, seed=7, device=torch.device("cuda", 0))
shift = engine.cast_f32(engine.colmean(X, None, 4096))
for _ in range(args.reps):
    G, cs = engine.gram(X, None, [0, args.rows], shift)
torch.cuda.synchronize()
print("ok", float(G[0].diagonal().sum()))
