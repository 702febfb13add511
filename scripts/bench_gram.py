#!/usr/bin/env python3
"""A/B the Gram arithmetic modes (ocm_gram_f32_ex) in ONE process
(interleaved rounds) on the bench workload (1M×2048 fp32 in HBM).  Prints
TFLOP/s (symmetric count n·p(p+1)) per mode/chunk and the max relative error
of each mode against an fp64 Gram of a row sample.

    python scripts/bench_gram.py [--variants i8x3:0,f32:0,bf16x3:0,i8x3:0:packed] [--outliers 0.005]

A third field sets OCM_GRAM8_ORDER for that variant (k_gram8e block order),
a fourth OCM_GRAM8_PIECES (quantiser / Gram overlap), a fifth OCM_Q8_CG
(column groups per quantiser row block on consecutive workgroups), a sixth
OCM_GRAM8_XCD (0: no XCD remap of the Gram workgroups).  "wall" is the whole
call (guard, quantiser, Gram, reduce) between two device synchronisations.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
QUANT_ID = 2  # include/ocm.h OCM_KERNEL_QUANT
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="i8x3:0,bf16x3:0,f32:0", help="mode:chunk_rows[:order] (0 = automatic)")
    ap.add_argument("--outliers", type=float, default=0.0, help="fraction of rows scaled x100..x1000")
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm import engine
    from ocm._lib import Context

    dev = torch.device("cuda", 0)
    X = synth_device(args.rows, args.p, 20, seed=7, device=dev)
    if args.outliers > 0:
        g = torch.Generator(device=dev).manual_seed(3)
        m = int(args.outliers * args.rows)
        idx = torch.randperm(args.rows, generator=g, device=dev)[:m]
        mu = X[:4096].mean(0)
        X[idx] = mu + (X[idx] - mu) * (100 + 900 * torch.rand(m, 1, generator=g, device=dev))
    shift = engine.cast_f32(engine.colmean(X, None, 4096))
    ctx = Context.get(0)
    import time

    variants = [tuple(v.split(":")[:2]) + tuple((v.split(":") + ["", "", "", ""])[2:6]) for v in args.variants.split(",")]
    variants = [(m, int(c), o, pc, cg, xr) for m, c, o, pc, cg, xr in variants]
    res = {":".join(map(str, v)): [] for v in variants}
    wall = {k: [] for k in res}
    quant = {k: [] for k in res}
    flop = args.rows * args.p * (args.p + 1)
    for _ in range(args.rounds):
        for mode, chunk, order, pcs, qcg, xr in variants:
            key = ":".join(map(str, (mode, chunk, order, pcs, qcg, xr)))
            for var, val in (("OCM_GRAM8_ORDER", order), ("OCM_GRAM8_PIECES", pcs), ("OCM_Q8_CG", qcg),
                             ("OCM_GRAM8_XCD", xr)):
                if val:
                    os.environ[var] = val
                else:
                    os.environ.pop(var, None)
            engine.gram(X, None, [0, args.rows], shift, mode=mode, chunk_rows=chunk)  # warm (workspace)
            torch.cuda.synchronize()
            ctx.read_timing(0)
            ctx.read_timing(QUANT_ID)
            ctx.set_timing(True)
            t0 = time.perf_counter()
            engine.gram(X, None, [0, args.rows], shift, mode=mode, chunk_rows=chunk)
            torch.cuda.synchronize()
            t1 = time.perf_counter()
            ctx.set_timing(False)
            ms, _ = ctx.read_timing(0)
            qms, _ = ctx.read_timing(QUANT_ID)
            res[key].append(flop / (ms / 1e3) / 1e12)
            wall[key].append((t1 - t0) * 1e3)
            quant[key].append(qms)
    print("guard marks (last i8x3 call):", engine.last_gram_marks(0))
    ns = min(args.rows, 65536)
    Y = X[:ns].double() - shift.double()
    Gref = Y.T @ Y
    os.environ.pop("OCM_GRAM8_ORDER", None)
    os.environ.pop("OCM_GRAM8_PIECES", None)
    os.environ.pop("OCM_Q8_CG", None)
    os.environ.pop("OCM_GRAM8_XCD", None)
    for mode in sorted({v[0] for v in variants}):
        Gm, _ = engine.gram(X, None, [0, ns], shift, mode=mode)
        err = ((Gm[0] - Gref).abs().max() / Gref.abs().max()).item()
        print(f"{mode:8s} sample Gram max rel err vs fp64: {err:.2e}")
    for key, vals in res.items():
        w = sorted(wall[key])
        qq = sorted(quant[key])
        print(f"{key:18s} TFLOP/s median {sorted(vals)[len(vals) // 2]:7.2f}  all {[round(v, 1) for v in vals]}  "
              f"wall ms median {w[len(w) // 2]:7.3f}  quantise ms median {qq[len(qq) // 2]:6.3f}", flush=True)


if __name__ == "__main__":
    main()
