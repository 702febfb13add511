#!/usr/bin/env python3
"""Eigensolver (ocm_eig_topk) timing on the bench's covariance: C of a
65,536-row sample of the 1M × 2048 synthetic spectra, k = 20, θ1..θ3 (jm).
``--spectrum nuts``: the same rows after the nuts preprocessing (SNV +
Savitzky–Golay w 5, p 2, deriv 1: simca_nuts.py:47-52), whose slow spectral
decay takes many iterations; ``geom``: a 2048-point geometric spectrum
100 … 0.01 in a random basis.

    python scripts/bench_eig.py [--reps 20] [--spectrum bench|nuts|geom]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--spectrum", default="bench", choices=["bench", "nuts", "geom"])
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm import engine

    dev = torch.device("cuda", 0)
    if args.spectrum == "geom":
        g = torch.Generator(device="cpu").manual_seed(3)
        Q, _ = torch.linalg.qr(torch.randn(2048, 2048, generator=g, dtype=torch.float64))
        lam = torch.logspace(2, -2, 2048, dtype=torch.float64)
        C = ((Q * lam) @ Q.T).to(dev)
        C = 0.5 * (C + C.T)
    else:
        X = synth_device(65536, 2048, args.k, seed=5, device=dev)
        if args.spectrum == "nuts":
            from ocm.preprocess import snv_savgol

            X = snv_savgol(X, 5, 2, deriv=1, snv=True)
        Y = X.double() - X.double().mean(0)
        C = (Y.T @ Y) / (X.shape[0] - 1)
    engine.eig_topk(C, args.k, 2)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        ev, _, th, it = engine.eig_topk(C, args.k, 2)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.reps
    ref = torch.linalg.eigvalsh(C).flip(0)
    print(json.dumps({"lib": os.path.basename(os.environ.get("OCM_LIB", "libocm.so")), "spectrum": args.spectrum,
                      "ms": round(dt * 1e3, 4),
                      "iters": int(it), "max_rel_eval": float(((ev - ref[:args.k]).abs() / ref[:args.k]).max()),
                      "theta1_rel": float(abs(th[0] - ref[args.k:].sum()) / ref[args.k:].sum())}), flush=True)


if __name__ == "__main__":
    main()
