"""Diagnose the k = 96 (two component blocks) fit against the fp64 oracle:
eigenvalues, loadings subspace, and T² recomputed on the host from the
device's own loadings (separates eigensolver error from scoring error)."""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..",
                                                                             "ocm-vae-simca_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle import simca_oracle as O  # noqa: E402
from utils import SIMCA  # noqa: E402

n, p, k = 20_000, 2048, int(sys.argv[1]) if len(sys.argv) > 1 else 96
kgen = int(sys.argv[2]) if len(sys.argv) > 2 else k
X = O.synth_spectra(n + 4000, p, kgen, rank=140, seed=4242, outlier_frac=800 / 24_000, loadings="random")[:n]
y = np.zeros(n, dtype=np.int64)
est = SIMCA(n_components=k, model_class=0, verbose=False).fit(X, y)
fit = est._fits[0]
mean, C = O.covariance_chunked(X.astype(np.float64))
ev, Vt = O.eig_desc(C)
evd = fit.evals.cpu().numpy()
print("eig iters", fit.eig_iters)
print("oracle evals around k:", ev[k - 4:k + 4])
if fit.C is not None:
    Cd = fit.C.cpu().numpy()
    print("C dev vs oracle: max abs", np.abs(Cd - C).max(), "rel to max", np.abs(Cd - C).max() / np.abs(C).max())
    evC = np.linalg.eigvalsh(Cd)[::-1]
    print("eigh(C dev) vs device evals max rel", np.max(np.abs(evC[:k] - fit.evals.cpu().numpy()) / evC[:k]))
    print("eigh(C dev) vs oracle evals max rel", np.max(np.abs(evC[:k] - ev[:k]) / ev[:k]))
print("evals max rel err", np.max(np.abs(evd - ev[:k]) / ev[:k]), "argmax", np.argmax(np.abs(evd - ev[:k]) / ev[:k]))
Pd = fit.P64.cpu().numpy()
print("P orthonormality", np.abs(Pd @ Pd.T - np.eye(k)).max())
cosv = np.abs(np.sum(Pd * Vt[:k], axis=1))
print("per-comp |cos| min", cosv.min(), "argmin", cosv.argmin(), "first 5 worst", np.argsort(cosv)[:5], np.sort(cosv)[:5])
s = np.linalg.svd(Pd @ Vt[:k].T, compute_uv=False)
print("subspace cos min", s.min())
Y = X.astype(np.float64) - fit.mean64.cpu().numpy()
Th = Y @ Pd.T
T2h = (Th ** 2 / evd).sum(1)
T2d = fit.T2.cpu().numpy()
print("device T2 vs host T2 (device P) max rel", np.max(np.abs(T2d - T2h) / T2h))
To = Y @ Vt[:k].T
T2o = (To ** 2 / ev[:k]).sum(1)
print("host T2 (device P) vs oracle max rel", np.max(np.abs(T2h - T2o) / T2o))
Td = fit.T.cpu().numpy()
print("device T vs host T (device P): max abs by comp block", np.abs(Td[:, :64] - Th[:, :64]).max(),
      np.abs(Td[:, 64:] - Th[:, 64:]).max() if k > 64 else 0, "scale", np.abs(Th).max())
Qd = fit.Q.cpu().numpy().astype(np.float64)
Qh = (Y ** 2).sum(1) - (Th ** 2).sum(1)
print("device Q vs host Q max rel", np.max(np.abs(Qd - Qh) / Qh))
