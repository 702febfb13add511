#!/usr/bin/env python3
"""Latent-encoding throughput of the C4/C5 network (eval mode, no grad):
encode + decode + row residual per batch, for several batch sizes and
precisions.  Prints one JSON line per variant (rows/s).

    python scripts/bench_encode.py [--length 4096] [--rows 65536]
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--length", type=int, default=4096)
    ap.add_argument("--rows", type=int, default=65536)
    ap.add_argument("--batches", default="512,2048,8192")
    ap.add_argument("--dtypes", default="bf16,f32")
    ap.add_argument("--train-steps", type=int, default=0, help="HIP-graph train steps before encoding")
    args = ap.parse_args()
    import torch

    import vae_model as V
    from ocm import engine

    dev = torch.device("cuda", 0)
    L = args.length
    torch.manual_seed(0)
    X = torch.randn(args.rows, L, device=dev)
    m = V.ConvVAE1D(L, 32, torch.zeros(L).numpy(), torch.ones(L).numpy(), conv_blocks=3, n_filters=3,
                    kernel_size=7, hidden_fc=64).to(dev)
    if args.train_steps:
        from ocm.vae_train import GraphedVAETrainer

        tr = GraphedVAETrainer(m, 512, lr=1e-3, dtype=torch.bfloat16)
        for i in range(args.train_steps):
            tr.step(X[(i % 8) * 512:(i % 8 + 1) * 512])
        torch.cuda.synchronize()
    m.eval()
    for dt in args.dtypes.split(","):
        for bs in (int(b) for b in args.batches.split(",")):
            ctx = torch.autocast("cuda", dtype=torch.bfloat16, enabled=(dt == "bf16"))

            def run(n):
                with torch.no_grad(), ctx:
                    for a in range(0, n, bs):
                        xb = X[a:a + bs]
                        mu, _ = m.encode((xb - m.spec_mean) / m.spec_std)
                        xr = m.decode(mu).float() * m.spec_std + m.spec_mean
                        engine.rowsq_residual(xb, xr.contiguous())

            run(2 * bs)  # kernel selection for this shape
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            run(args.rows)
            torch.cuda.synchronize()
            dt_s = time.perf_counter() - t0
            print(json.dumps({"dtype": dt, "batch": bs, "rows": args.rows, "L": L, "s": round(dt_s, 4),
                              "rows_per_s": round(args.rows / dt_s, 1)}), flush=True)


if __name__ == "__main__":
    main()
