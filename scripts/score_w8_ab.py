#!/usr/bin/env python3
"""Same-process A/B of k_score_1p with four waves per workgroup (one per SIMD,
the product) against eight (two per SIMD, WV = 8) on the bench workload
(1M × 2048 fp32 in HBM, k = 20): an exp build with -DOCM_S1P_W8 holds both,
OCM_S1P_W8_ON=0/1 picks one per call.  Prints ms per launch of each (pairs
alternated), and the largest T² / Q differences between the two.

    OCM_ALLOW_EXP_LIB=1 OCM_LIB=.../build/exp/libocm_w8.so python scripts/score_w8_ab.py
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)


def main():
    import torch

    from bench import synth_device
    from ocm import engine

    dev = torch.device("cuda", 0)
    n, p, reps = int(os.environ.get("ROWS", 1_000_000)), 2048, int(os.environ.get("REPS", 10))
    X = synth_device(n, p, 20, 7, dev)
    mean = X[:4096].double().mean(0)
    res = {}
    for k in (20, 16):
        P, _ = torch.linalg.qr(torch.randn(p, k, dtype=torch.float64, device=dev))
        P = P.T.contiguous()
        inv = torch.linspace(1.0, 0.1, k, dtype=torch.float64, device=dev)
        outs, times = {}, {"w4": [], "w8": []}
        for rnd in range(3):
            for tag, on in (("w4", "0"), ("w8", "1")) if rnd % 2 == 0 else (("w8", "1"), ("w4", "0")):
                os.environ["OCM_S1P_W8_ON"] = on
                outs[tag] = engine.score(X, None, n, P, mean, inv, want_T=True, want_stats=True)
                st = torch.cuda.current_stream()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    engine.score(X, None, n, P, mean, inv, want_stats=True)
                e1.record(st)
                torch.cuda.synchronize()
                times[tag].append(e0.elapsed_time(e1) / reps)
        a, b = outs["w4"], outs["w8"]
        d = {key: float(((a[key].double() - b[key].double()).abs() / a[key].double().abs().clamp_min(1e-30)).max())
             for key in ("T2", "Q", "T")}
        res[k] = {"ms_w4": [round(t, 4) for t in times["w4"]], "ms_w8": [round(t, 4) for t in times["w8"]],
                  "GBs_w4": round(4 * p * n / min(times["w4"]) / 1e6, 1),
                  "GBs_w8": round(4 * p * n / min(times["w8"]) / 1e6, 1), "max_rel_diff": d}
        print(json.dumps({"k": k, **res[k]}), flush=True)


if __name__ == "__main__":
    main()
