#!/usr/bin/env python3
"""Quantiser A/B between two libocm builds (run once per library, OCM_LIB):
the i8×3 Gram of the bench workload (1M × 2048) — quantiser and Gram times
from the library's hipEvent timing — and a hash of the fp64 Gram, so two
builds whose digit planes agree print the same hash.

    python scripts/quant_ab.py [--rows N] [--reps R]
"""
import argparse
import hashlib
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    import torch

    from bench import synth_device
    from ocm import _lib, engine

    dev = torch.device("cuda", 0)
    X = synth_device(args.rows, 2048, 20, 7, dev)
    shift = engine.cast_f32(engine.colmean(X, None, 4096))
    ctx = _lib.Context.get(0)
    G, cs = engine.gram(X, None, [0, args.rows], shift)
    torch.cuda.synchronize()
    h = hashlib.sha256(G.cpu().numpy().tobytes() + cs.cpu().numpy().tobytes()).hexdigest()[:16]
    ctx.set_timing(True)
    ctx.read_timing(0)
    ctx.read_timing(2)
    for _ in range(args.reps):
        engine.gram(X, None, [0, args.rows], shift)
    torch.cuda.synchronize()
    tg, ng = ctx.read_timing(0)
    tq, nq = ctx.read_timing(2)
    ctx.set_timing(False)
    print(json.dumps({"lib": os.path.basename(os.environ.get("OCM_LIB", "libocm.so")), "gram_hash": h,
                      "quant_ms": round(tq / max(nq, 1), 4), "gram_ms": round(tg / max(ng, 1), 4), "n": [nq, ng]}),
          flush=True)


if __name__ == "__main__":
    main()
