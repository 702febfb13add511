"""End-to-end drop-in rate from host memory (PCIe-inclusive), for DESIGN.md.

The headline ``bench.py`` value has the spectra resident in HBM.  Here the
caller holds a NumPy float32 matrix in host RAM, exactly as the reference's
drivers do (simca_nuts.py:186-189): ``utils.SIMCA(...).fit(X, y)`` then
``.predict(X)``, so the H2D copy of X (twice: fit and predict each receive
the host array) and the D2H of the (n, 1) float64 predictions are inside the
timed region.

    python scripts/bench_e2e.py [--rows 1000000] [--p 2048] [--k 20]
"""
import argparse
import contextlib
import io
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (REPO, os.path.join(REPO, "ocm-vae-simca_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--p", type=int, default=2048)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--reps", type=int, default=3)
    args = ap.parse_args()

    import numpy as np
    import torch

    from bench import synth_device
    from utils import SIMCA

    dev = torch.device("cuda", 0)
    Xd = synth_device(args.rows, args.p, args.k, 4321, dev)
    X = Xd.cpu().numpy()  # host copy (pageable, like a NumPy array from a driver script)
    del Xd
    y = np.zeros(args.rows, dtype=np.int64)

    def run():
        with contextlib.redirect_stdout(io.StringIO()):
            est = SIMCA(n_components=args.k, model_class=0, type="alt", t2lim="Fdist", qlim="jm", verbose=False)
            est.fit(X, y)
            pred = est.predict(X)
        return pred

    run()
    times = []
    for _ in range(args.reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        pred = run()
        torch.cuda.synchronize()
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    # raw H2D bandwidth of the same array (pageable → HBM)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    _ = torch.from_numpy(X).to(dev)
    torch.cuda.synchronize()
    h2d = time.perf_counter() - t0
    print(json.dumps({"metric": "drop-in SIMCA fit+predict from host NumPy (PCIe-inclusive)",
                      "value": round(args.rows / t, 1), "unit": "spectra/s", "seconds": round(t, 4),
                      "rows": args.rows, "p": args.p, "k": args.k, "accept_rate": float(np.mean(pred)),
                      "h2d_GBs": round(X.nbytes / h2d / 1e9, 2), "h2d_s": round(h2d, 4)}))


if __name__ == "__main__":
    main()
