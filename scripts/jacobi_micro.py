"""One 32×32 Jacobi eigensolve per call (ocm_eig_topk at p = 32 runs
k_jacobi_1b once, without the Rayleigh–Ritz test): with a `make exp`
build carrying OCM_JACOBI_STAMPS each call prints its phase stamps.

    OCM_ALLOW_EXP_LIB=1 OCM_LIB=.../libocm_jstamp.so python scripts/jacobi_micro.py [--reps 4]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=4)
    args = ap.parse_args()
    import numpy as np
    import torch

    from ocm import engine

    rng = np.random.default_rng(0)
    lam = np.concatenate([np.linspace(60, 8, 20), np.geomspace(2.0, 1e-3, 12)])
    Q, _ = np.linalg.qr(rng.standard_normal((32, 32)))
    C = torch.from_numpy(0.5 * ((Q * lam) @ Q.T + ((Q * lam) @ Q.T).T)).cuda()
    for _ in range(args.reps):
        ev, _, _, _ = engine.eig_topk(C, 5, 0)
        torch.cuda.synchronize()
    print("top eigenvalues", ev.cpu().numpy()[:3], "want", lam[:3])


if __name__ == "__main__":
    main()
