#!/usr/bin/env python3
"""A/B the Gram kernel variants in ONE process (interleaved rounds), on the
bench workload (1M×2048 fp32 in HBM).  Prints TFLOP/s (symmetric count) per
variant and the max relative difference of G between variants."""
import argparse
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
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="bf16x3:256x32:2048,i8x3:128x32:4096,i8x3:128x32:2048,i8x3:128x32:1024")
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm import engine
    from ocm._lib import Context

    dev = torch.device("cuda", 0)
    X = synth_device(args.rows, args.p, 20, seed=7, device=dev)
    shift = engine.cast_f32(engine.colmean(X, None, 4096))
    ctx = Context.get(0)
    variants = [v.split(":") for v in args.variants.split(",")]
    res = {":".join(v): [] for v in variants}
    Gs = {}
    flop = args.rows * args.p * (args.p + 1)
    for r in range(args.rounds):
        for mode, name, chunk in variants:
            os.environ["OCM_GRAM_MODE"] = "bf16x3" if mode.startswith("bf16x3") else mode[:4] if mode.startswith("i8x3") else mode
            # i8x3 kernel variants: i8x3 (default) | i8x3d (direct) | i8x3s[N] (shared LDS, N-slot ring)
            var = {"i8x3d": "direct"}.get(mode) or ("shared" + mode[5:] if mode.startswith("i8x3s") else None)
            if var:
                os.environ["OCM_GRAM8_VARIANT"] = var
            else:
                os.environ.pop("OCM_GRAM8_VARIANT", None)
            if mode == "bf16x3pk":
                os.environ["OCM_GRAM3_PK"] = "1"
            else:
                os.environ.pop("OCM_GRAM3_PK", None)
            os.environ["OCM_GRAM_TILE"], os.environ["OCM_GRAM_BK"] = name.split("x")
            os.environ["OCM_GRAM_CHUNK"] = chunk
            key = f"{mode}:{name}:{chunk}"
            engine.gram(X, None, [0, args.rows], shift)  # warm (workspace)
            torch.cuda.synchronize()
            ctx.read_timing(0)
            ctx.set_timing(True)
            G, cs = engine.gram(X, None, [0, args.rows], shift)
            ctx.set_timing(False)
            ms, cnt = ctx.read_timing(0)
            res[key].append(flop / (ms / 1e3) / 1e12)
            if r == 0:
                Gs[key] = G[0].clone()
    # exact reference for the error column: fp64 Gram of a row sample (first 65536 rows)
    ns = min(args.rows, 65536)
    Y = (X[:ns].double() - shift.double())
    Gref = Y.T @ Y
    os.environ.pop("OCM_GRAM3_PK", None)
    os.environ.pop("OCM_GRAM8_VARIANT", None)
    for mode in sorted({v[0][:4] if v[0].startswith("i8x3") else v[0] for v in variants} - {"bf16x3pk"}):
        os.environ["OCM_GRAM_MODE"] = mode
        Gm, _ = engine.gram(X, None, [0, ns], shift)
        print(f"{mode:8s} sample Gram max rel err vs fp64: {((Gm[0] - Gref).abs().max() / Gref.abs().max()).item():.2e}")
    ref = next(iter(Gs.values()))
    for key, vals in res.items():
        d = ((Gs[key] - ref).abs().max() / ref.abs().max()).item()
        print(f"{key:24s} TFLOP/s median {sorted(vals)[len(vals)//2]:7.2f}  all {[round(v,1) for v in vals]}  "
              f"maxrel vs first {d:.2e}", flush=True)


if __name__ == "__main__":
    main()
