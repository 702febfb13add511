"""Child process of tests/test_gpu_eig_wait.py (GPU): one SIMCA class fit
whose eigensolve runs the Rayleigh–Ritz test fused into the Jacobi, with S
from side stream B taken in flight (theta_mode 2: the deflation and θ3 chain
on the side streams).  The parent runs it with the product library, with
AMD_SERIALIZE_KERNEL=3 (every launch waits for the previous one), and with a
``make exp`` build whose wait gives up at once (OCM_JACOBI_WAIT_SPINS=0), so
every test takes the re-run path.  Prints one JSON line."""
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "ocm-vae-simca_amd"))
sys.path.insert(0, REPO)
import ocm  # noqa: E402,F401
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from ocm import _lib, engine
    from oracle import simca_oracle as O

    X = torch.from_numpy(O.synth_spectra(20000, 512, 20, rank=48, seed=9, outlier_frac=0.02)).cuda()
    fit = engine.fit_class(X, None, X.shape[0], 20, 2, want_T=False)
    torch.cuda.synchronize()
    n = ctypes.c_int64(0)
    _lib.check(_lib.load().ocm_eig_test_reruns(_lib.Context.get(0).handle, ctypes.byref(n)), "ocm_eig_test_reruns")
    print(json.dumps({"evals": fit.evals_host.tolist(), "thetas": list(fit.thetas), "iters": fit.eig_iters,
                      "P": np.abs(fit.P64.cpu().numpy()).sum(1).tolist(), "reruns": int(n.value),
                      "lib": _lib.LIB_PATH}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
