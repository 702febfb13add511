#!/usr/bin/env python3
"""Time the SIMCA scoring kernels on the bench workload (1M×2048 fp32 in HBM)
in ONE process: ocm_score_f32_diag (single HBM pass for the SIMCA shapes) and
ocm_score_f32 (two sweeps), for each k.  hipEvents around the launches on the
launch stream; prints ms per launch and the algorithmic HBM rate (4p B/row).

    python scripts/bench_score.py [--k 16,20] [--reps 10] [--kernels diag,full]
The library is $OCM_LIB (default: the in-tree libocm.so), so an experiment
build (make -C ocm-vae-simca_amd/csrc exp) can be A/B'd against the product."""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--k", default="16,20")
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--kernels", default="diag,full")
    ap.add_argument("--gram", action="store_true", help="also time the i8x3 Gram (quantiser + Gram) per view")
    ap.add_argument("--prep", default="none", help="comma list of none, snv (SNV only), snv5 (SNV + w 5 d 1), "
                    "sg15 (w 15 d 1): score lazy views (diag kernel)")
    ap.add_argument("--tag", default=os.path.basename(os.environ.get("OCM_LIB", "libocm.so")))
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm import engine

    dev = torch.device("cuda", 0)
    n, p = args.rows, args.p
    X = synth_device(n, p, 20, 7, dev)
    mean = X[:4096].double().mean(0)
    from ocm import preprocess

    views = {"none": X, "snv": preprocess.snv_savgol(X, None, lazy=True),
             "snv5": preprocess.snv_savgol(X, 5, 2, 1, lazy=True),
             "sg15": preprocess.snv_savgol(X, 15, 2, 1, snv=False, lazy=True)}
    for pv in args.prep.split(","):
        if pv == "none":
            continue
        Xv = views[pv]
        Xv.rowstat()
        for k in [int(v) for v in args.k.split(",")]:
            P, _ = torch.linalg.qr(torch.randn(p, k, dtype=torch.float64, device=dev))
            P = P.T.contiguous()
            inv = torch.linspace(1.0, 0.1, k, dtype=torch.float64, device=dev)
            outv = engine.score(Xv, None, n, P, mean, inv, want_stats=True)
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.reps):
                engine.score(Xv, None, n, P, mean, inv, want_stats=True)
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            extra = {}
            if os.environ.get("OCM_STAMPS"):
                tiles = (n + 15) // 16
                extra["cycles_per_tile"] = [round(v / tiles, 1) for v in outv["stats"].cpu().tolist()]
            print(json.dumps({**extra, "lib": args.tag, "kernel": "diag", "prep": pv, "k": k, "p": p, "rows": n,
                              "ms": round(ms, 4), "GBs_alg": round(4 * p * n / ms / 1e6, 1)}), flush=True)
    if args.gram:
        from ocm import _lib

        ctx = _lib.Context.get(0)
        for pv in args.prep.split(","):
            Xv = views[pv]
            if pv != "none":
                Xv.rowstat()
            shift = engine.cast_f32(engine.colmean(Xv, None, 4096))
            engine.gram(Xv, None, [0, n], shift)
            torch.cuda.synchronize()
            for kid in range(3):
                ctx.read_timing(kid)
            ctx.set_timing(True)
            for _ in range(3):
                engine.gram(Xv, None, [0, n], shift)
            torch.cuda.synchronize()
            ctx.set_timing(False)
            t = {nm: ctx.read_timing(kid) for kid, nm in enumerate(("gram", "score", "quant"))}
            print(json.dumps({"kernel": "gram_i8x3", "prep": pv, "rows": n, "p": p,
                              "quant_ms": round(t["quant"][0] / max(1, t["quant"][1]), 4),
                              "gram_ms": round(t["gram"][0] / max(1, t["gram"][1]), 4),
                              "marks": engine.last_gram_marks(0)}), flush=True)
    for k in [int(v) for v in args.k.split(",")]:
        P, _ = torch.linalg.qr(torch.randn(p, k, dtype=torch.float64, device=dev))
        P = P.T.contiguous()
        inv = torch.linspace(1.0, 0.1, k, dtype=torch.float64, device=dev)
        ref = None
        for kern in args.kernels.split(","):
            A = inv if kern == "diag" else torch.diag(inv)
            out = engine.score(X, None, n, P, mean, A, want_stats=True)  # warm-up
            torch.cuda.synchronize()
            if ref is None:
                ref = out["Q"].double()
            err = float(((out["Q"].double() - ref).abs() / ref.abs().clamp_min(1e-30)).max())
            st = torch.cuda.current_stream()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(st)
            for _ in range(args.reps):
                engine.score(X, None, n, P, mean, A, want_stats=True)
            e1.record(st)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / args.reps
            extra = {}
            if os.environ.get("OCM_STAMPS"):  # diagnostic build: stats carry Σ cycles per phase (wave 0)
                tiles = (n + 15) // 16
                extra["cycles_per_tile"] = [round(v / tiles, 1) for v in out["stats"].cpu().tolist()]
            print(json.dumps({**extra, "lib": args.tag, "kernel": kern, "k": k, "p": p, "rows": n, "ms": round(ms, 4),
                              "GBs_alg": round(4 * p * n / ms / 1e6, 1), "maxrel_Q_vs_first": err}), flush=True)


if __name__ == "__main__":
    main()
