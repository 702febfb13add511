#!/usr/bin/env python3
"""A/B the scoring kernel variants in ONE process on the bench workload
(1M×2048 fp32, k=20): GB/s of single-pass bytes and output agreement."""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="f64,direct,lds")
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm import engine
    from ocm._lib import Context

    dev = torch.device("cuda", 0)
    X = synth_device(args.rows, args.p, args.k, seed=7, device=dev)
    g = torch.Generator(device=dev).manual_seed(1)
    Pm = torch.linalg.qr(torch.randn(args.p, args.k, generator=g, device=dev, dtype=torch.float64))[0].T.contiguous()
    P32 = Pm.contiguous()
    mu = X[:4096].double().mean(0).contiguous()
    A = torch.diag(torch.linspace(1.0, 0.1, args.k, device=dev, dtype=torch.float64)).contiguous()
    ctx = Context.get(0)
    res, outs = {}, {}
    for r in range(args.rounds):
        for v in args.variants.split(","):
            os.environ["OCM_SCORE_VARIANT"] = v
            engine.score(X, None, args.rows, P32, mu, A)
            torch.cuda.synchronize()
            ctx.read_timing(1)
            ctx.set_timing(True)
            o = engine.score(X, None, args.rows, P32, mu, A, want_T=True)
            ctx.set_timing(False)
            ms, _ = ctx.read_timing(1)
            res.setdefault(v, []).append(args.rows * args.p * 4 / (ms / 1e3) / 1e9)
            if r == 0:
                outs[v] = o
    first = args.variants.split(",")[0]
    for v, vals in res.items():
        dq = ((outs[v]["Q"].double() - outs[first]["Q"].double()).abs() / outs[first]["Q"].double().abs()).max().item()
        dt = ((outs[v]["T2"] - outs[first]["T2"]).abs() / outs[first]["T2"].abs()).max().item()
        print(f"{v:8s} GB/s median {sorted(vals)[len(vals)//2]:8.1f} ms {args.rows*args.p*4/sorted(vals)[len(vals)//2]/1e6:.3f}"
              f"  maxrel Q {dq:.2e} T2 {dt:.2e}", flush=True)


if __name__ == "__main__":
    main()
