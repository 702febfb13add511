#!/usr/bin/env python3
"""Eigensolver (ocm_eig_topk) timing on the bench's covariance: C of a
65,536-row sample of the 1M × 2048 synthetic spectra, k = 20, θ1..θ3 (jm).

    python scripts/bench_eig.py [--reps 20]
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
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm import engine

    dev = torch.device("cuda", 0)
    X = synth_device(65536, 2048, args.k, seed=5, device=dev)
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
    print(json.dumps({"lib": os.path.basename(os.environ.get("OCM_LIB", "libocm.so")), "ms": round(dt * 1e3, 4),
                      "iters": int(it), "max_rel_eval": float(((ev - ref[:args.k]).abs() / ref[:args.k]).max()),
                      "theta1_rel": float(abs(th[0] - ref[args.k:].sum()) / ref[args.k:].sum())}), flush=True)


if __name__ == "__main__":
    main()
