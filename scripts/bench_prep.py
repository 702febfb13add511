#!/usr/bin/env python3
"""SNV + Savitzky–Golay preprocessing throughput (ocm_snv_savgol_f32) on a
1M×2048 fp32 matrix in HBM: rows/s and algorithmic GB/s (read + write 4p B
per row), for the nuts (w = 5, polyorder 2, deriv 1) and cheese (w = 15)
filters and SNV alone.

    python scripts/bench_prep.py [--rows 1000000] [--p 2048]
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
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm.preprocess import snv_savgol

    dev = torch.device("cuda", 0)
    X = synth_device(args.rows, args.p, 20, seed=3, device=dev)
    out = torch.empty_like(X)
    for name, kw in [("snv+sg5d1", dict(window_length=5, polyorder=2, deriv=1)),
                     ("snv+sg15d1", dict(window_length=15, polyorder=2, deriv=1)), ("snv", dict())]:
        snv_savgol(X, out=out, **kw)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.reps):
            snv_savgol(X, out=out, **kw)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / args.reps
        gbs = 2 * X.numel() * 4 / dt / 1e9
        print(json.dumps({"filter": name, "rows": args.rows, "p": args.p, "ms": round(dt * 1e3, 3),
                          "rows_per_s": round(args.rows / dt, 1), "GBs": round(gbs, 1),
                          "hbm_frac": round(gbs / 8000.0, 4)}), flush=True)


if __name__ == "__main__":
    main()
