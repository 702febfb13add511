"""Parity at the north-star shape (BASELINE.json config C2):
p = 2048 wavelengths, k = 20 components, default i8×3 Gram.

* against the REFERENCE (tests/golden/simca_ns.npz, made by make_golden.py
  from /root/reference at 8000 fit rows + 2000 test rows);
* against the fp64 oracle (Gram + eigh, ``precision='gram'``) at the C2 size,
  100k × 2048, for alt/Fdist/jm, sim/perc/perc and dd/chi2pom/chi2pom;
* on outlier-bearing data (0.5–1 % of rows scaled ×100–×1000, spread over the
  1536-row scale blocks) against the fp64 oracle: the i8×3 outlier guard must
  keep θ-based (jm) and F limits and the decisions;
* float64 input: the drop-in computes in float64 on the GPU (fp64-MFMA Gram,
  fp64 scoring, as sklearn's PCA follows the input dtype) and is compared
  with the reference's float64 run.

Tolerances: T², Q rtol 1e-4 with an absolute floor of
1e-5·median; limits rtol 1e-5 (percentile / moment limits 1e-4); decisions
identical outside |dred − D_lim| < 1e-4·D_lim."""
import contextlib
import io
import json
import os

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

BAND = 1e-4


def _load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name), allow_pickle=False))


def close(a, b, rtol=1e-4, floor=1e-5):
    b = np.asarray(b)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=floor * float(np.median(np.abs(b))))


def _lim_rtol(t2):
    return 1e-4 if t2 in ("perc", "chi2pom") else 1e-5


def _regen(g):
    from oracle.simca_oracle import synth_spectra

    c = json.loads(str(g["config_json"]))
    if "n_test" in c:
        X = synth_spectra(c["n_fit"] + c["n_test"], c["p"], c["k"], rank=c["rank"], seed=c["seed"],
                          outlier_frac=c["outlier_frac"])
        return X[:c["n_fit"]], X[c["n_fit"]:], c["k"]
    X = synth_spectra(c["n"], c["p"], c["k"], rank=c["rank"], seed=c["seed"], outlier_frac=c["outlier_frac"],
                      dtype=np.float64)
    return X[:c["n_fit"]], X[c["n_fit"]:], c["k"]


def _check_vs_reference(g, X_fit, X_test, k, arrays=True):
    from oracle import simca_oracle as O
    from utils import SIMCA

    y = np.zeros(len(X_fit), dtype=np.int64)
    n_checked = 0
    for ci, combo in enumerate(g["combos"]):
        ty, t2, ql = str(combo).split("|")
        est = SIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql, verbose=False)
        with contextlib.redirect_stdout(io.StringIO()):
            est.fit(X_fit, y)
            pred = est.predict(X_test)[:, 0]
        m = est._model[0]
        if arrays and ci == 0:
            np.testing.assert_allclose(m["xmean"], g["xmean"], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(m["eigs_all"][:k], g["eigs_all"][:k], rtol=1e-5)
            close(m["T2"], g["fit_T2"])
            close(m["Q"], g["fit_Q"])
            T2, _, Q, _ = est.transform(X_test)
            close(T2, g["test_T2"], rtol=2e-4)
            close(Q, g["test_Q"], rtol=2e-4)
        np.testing.assert_allclose(m["T2_limit"], g["T2_limit"][ci], rtol=_lim_rtol(t2), err_msg=str(combo))
        np.testing.assert_allclose(m["Q_limit"], g["Q_limit"][ci], rtol=1e-4, err_msg=str(combo))
        np.testing.assert_allclose(m["D_limit"], g["D_limit"][ci], rtol=1e-4, err_msg=str(combo))
        orc = O.OracleSIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql)
        orc.fit(X_fit, y)
        d = orc.dred(X_test, 0)
        dl = orc._model[0]["D_limit"]
        clear = np.abs(d - dl) > BAND * abs(dl)
        np.testing.assert_array_equal(pred[clear], g["pred"][ci][clear].astype(np.float64), err_msg=str(combo))
        n_checked += int(clear.sum())
    assert n_checked > 0


def test_north_star_shape_vs_reference(golden_dir):
    """p = 2048, k = 20 through the drop-in, against the reference's own run."""
    g = _load(golden_dir, "simca_ns.npz")
    X_fit, X_test, k = _regen(g)
    _check_vs_reference(g, X_fit, X_test, k)


def test_theta_tail_sums_at_north_star(golden_dir):
    """θ1..θ3 from the deflated-trace kernel vs the reference's eigenvalue tail sums."""
    import torch
    from ocm import engine

    g = _load(golden_dir, "simca_ns.npz")
    X_fit, _, k = _regen(g)
    fit = engine.fit_class(torch.from_numpy(X_fit).cuda(), None, len(X_fit), k, 2)
    np.testing.assert_allclose(fit.thetas, g["thetas"], rtol=1e-4)


def test_float64_input_vs_reference(golden_dir):
    """float64 X.  The reference then runs its PCA in float64, and so does the
    drop-in (k_gram_f64 + k_score_f64, T and Q returned as float64): limits,
    T²/Q and decisions agree at the stated tolerances."""
    g = _load(golden_dir, "simca_f64.npz")
    X_fit, X_test, k = _regen(g)
    assert X_fit.dtype == np.float64
    _check_vs_reference(g, X_fit, X_test, k)


def _c2_data(n, p, k, seed, outliers=None):
    from oracle.simca_oracle import synth_spectra

    X = synth_spectra(n, p, k, rank=40, seed=seed)
    if outliers is not None:
        frac, lo, hi = outliers
        rng = np.random.default_rng(seed + 1)
        idx = np.sort(rng.choice(n, int(round(frac * n)), replace=False))
        mu = X.mean(0)
        X[idx] = (mu + (X[idx] - mu) * rng.uniform(lo, hi, len(idx))[:, None]).astype(np.float32)
    return X


def _check_vs_oracle(X, Xt, k, combos):
    """drop-in utils.SIMCA vs the fp64 oracle (Gram + eigh) on the same rows."""
    from oracle import simca_oracle as O
    from utils import SIMCA

    y = np.zeros(len(X), dtype=np.int64)
    base = None
    n_checked = 0
    for ty, t2, ql in combos:
        est = SIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql, verbose=False)
        with contextlib.redirect_stdout(io.StringIO()):
            est.fit(X, y)
            pred = est.predict(Xt)[:, 0]
        orc = O.OracleSIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql, precision="gram")
        orc.fit(X, y)
        m, mo = est._model[0], orc._model[0]
        if base is None:
            close(m["T2"], mo["T2"])
            close(m["Q"], mo["Q"])
            np.testing.assert_allclose(m["eigs_all"][:k], mo["eigs_all"][:k], rtol=1e-6)
            base = True
        for key in ("T2_limit", "Q_limit", "D_limit"):
            rt = _lim_rtol(t2) if key != "Q_limit" else (1e-4 if ql in ("perc", "chi2pom") else 1e-5)
            np.testing.assert_allclose(m[key], mo[key], rtol=rt, err_msg=f"{ty}|{t2}|{ql} {key}")
        d = orc.dred(Xt, 0)
        dl = mo["D_limit"]
        clear = np.abs(d - dl) > BAND * abs(dl)
        ref = (d < dl).astype(np.float64)
        np.testing.assert_array_equal(pred[clear], ref[clear], err_msg=f"{ty}|{t2}|{ql}")
        n_checked += int(clear.sum())
        assert 0 < ref.sum() < len(ref)  # both decisions occur
    assert n_checked > 0


@pytest.mark.timeout(300)
def test_c2_100k_x_2048_vs_fp64_oracle():
    """BASELINE.json config C2: 100k × 2048, k = 20 (default i8×3 Gram); the
    test rows come from the same generator (same loadings), the last 2000 of
    them carry the out-of-class band."""
    from oracle.simca_oracle import synth_spectra

    n, p, k = 100_000, 2048, 20
    X = synth_spectra(n + 20_000, p, k, rank=40, seed=1234, outlier_frac=2000 / 120_000)
    _check_vs_oracle(X[:n], X[n:], k, [("alt", "Fdist", "jm"), ("sim", "perc", "perc"),
                                       ("dd", "chi2pom", "chi2pom")])


@pytest.mark.timeout(300)
@pytest.mark.parametrize("frac,lo,hi", [(0.005, 100.0, 1000.0), (0.01, 100.0, 300.0)])
def test_outlier_rows_limits_vs_fp64_oracle(frac, lo, hi):
    """outlier rows spread over the 1536-row scale blocks.
    The guard screens them out of the digit planes and adds them back exactly;
    jm (θ tail sums), F and chi2box limits and the decisions (on every 5th
    training row, outliers included) follow the fp64 oracle."""
    import torch
    from ocm import engine

    n, p, k = 30_000, 512, 10
    X = _c2_data(n, p, k, seed=77, outliers=(frac, lo, hi))
    _check_vs_oracle(X, X[::5].copy(), k, [("alt", "Fdist", "jm"), ("ci", "chi2", "chi2box")])
    # the guard engaged on the fix-up path (no bf16×3 fallback at this outlier rate)
    Xd = torch.from_numpy(X).cuda()
    shift = engine.cast_f32(engine.colmean(Xd, None, 4096))
    engine.gram(Xd, None, [0, n], shift)
    assert 0 < engine.last_gram_marks(0)


@pytest.mark.timeout(300)
def test_k96_wide_block_vs_fp64_oracle():
    """n_components beyond one 64-wide block (k = 96 at
    p = 2048, the reference allows any k ≤ min(n, p), utils/SIMCA.py:34-40):
    the eigensolver's 144-column block with host b×b steps, and scoring in two
    component blocks (64 + 32), against the fp64 oracle.  Orthonormal random
    loadings: 96 independent directions with the gap at k (band loadings this
    wide stop at ≈70, and noise-floor eigenvalues 1e-5 of λ₁ are beyond any
    float32 method, the reference's SVD included)."""
    from oracle.simca_oracle import synth_spectra

    n, p, k = 20_000, 2048, 96
    X = synth_spectra(n + 4000, p, k, rank=140, seed=4242, outlier_frac=800 / 24_000, loadings="random")
    _check_vs_oracle(X[:n], X[n:], k, [("alt", "Fdist", "jm"), ("ci", "chi2", "chi2box")])


def test_eig_not_converged_raises():
    """A covariance with no gap at k (a nearly flat spectrum) cannot converge in
    a short iteration budget: with ``dense_fallback=False`` the engine raises
    OcmNotConverged instead of handing on an unconverged subspace."""
    import torch

    from ocm import OcmNotConverged, engine

    p, k = 256, 20
    rng = np.random.default_rng(9)
    Qm, _ = np.linalg.qr(rng.standard_normal((p, p)))
    lam = np.linspace(1.0, 0.995, p)
    C = torch.from_numpy((Qm * lam) @ Qm.T).cuda()
    with pytest.raises(OcmNotConverged):
        engine.eig_topk(C, k, 2, max_iter=30, dense_fallback=False)
    # the same call with a gap converges
    lam[:k] *= 10
    C = torch.from_numpy((Qm * lam) @ Qm.T).cuda()
    ev, _, _, it = engine.eig_topk(C, k, 2, max_iter=30)
    np.testing.assert_allclose(ev.cpu().numpy(), np.sort(lam)[::-1][:k], rtol=1e-10)


def test_eig_not_converged_dense_fallback():
    """on a flat tail the default path does not abort (the
    reference's full SVD always returns): the dense eigensolver gives the
    top-k, θ1..θ3 from the eigenvalue tail, with a RuntimeWarning — and a
    SIMCA fit on spectra whose noise floor is flat at k completes and matches
    the fp64 oracle's limits."""
    import torch

    from ocm import engine

    p, k = 256, 20
    rng = np.random.default_rng(9)
    Qm, _ = np.linalg.qr(rng.standard_normal((p, p)))
    lam = np.linspace(1.0, 0.995, p)
    C = (Qm * lam) @ Qm.T
    with pytest.warns(RuntimeWarning, match="dense eigensolver"):
        ev, vec, th, _ = engine.eig_topk(torch.from_numpy(C).cuda(), k, 2, max_iter=30)
    w = np.sort(np.linalg.eigvalsh(C))[::-1]
    np.testing.assert_allclose(ev.cpu().numpy(), w[:k], rtol=1e-12)
    tail = w[k:]
    np.testing.assert_allclose(th.cpu().numpy(), [tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()], rtol=1e-12)
    V = vec.cpu().numpy()
    np.testing.assert_allclose(V @ V.T, np.eye(k), atol=1e-10)
    np.testing.assert_allclose(V @ C, ev.cpu().numpy()[:, None] * V, atol=1e-10)


@pytest.mark.parametrize("p,k", [(2048, 20), (300, 7), (3, 2), (1, 1), (64, 64)])
def test_eigh_dense_vs_numpy(p, k):
    """ocm_eigh_f64 (Householder tridiagonalisation on the GPU, QL + inverse
    iteration on the host): all eigenvalues vs numpy.linalg.eigvalsh, the top-k
    vectors orthonormal with residuals at fp64 level and the svd_flip sign;
    a covariance with repeated eigenvalues included."""
    import torch

    from ocm import engine

    rng = np.random.default_rng(p)
    if p >= 64:
        Qm, _ = np.linalg.qr(rng.standard_normal((p, p)))
        lam = np.concatenate([np.linspace(50, 10, min(k, p)), np.full(max(p - k, 0), 0.5)])[:p]
        lam[k // 2: k // 2 + 3] = lam[k // 2]  # a repeated eigenvalue inside the top k
        C = (Qm * lam) @ Qm.T
    else:
        A = rng.standard_normal((p, p))
        C = A @ A.T
    ev, vec = engine.eigh_dense(torch.from_numpy(C).cuda(), k)
    ev = ev.cpu().numpy()
    w = np.sort(np.linalg.eigvalsh(C))[::-1]
    np.testing.assert_allclose(ev, w, rtol=0, atol=1e-12 * np.abs(w).max() * max(1, p // 64))
    V = vec.cpu().numpy()
    np.testing.assert_allclose(V @ V.T, np.eye(k), atol=1e-9)
    np.testing.assert_allclose(V @ C, ev[:k, None] * V, atol=1e-9 * np.abs(w).max())
    idx = np.argmax(np.abs(V), axis=1)
    assert np.all(V[np.arange(k), idx] > 0)


def test_eigs_all_from_libocm(golden_dir):
    """`_model[cls]['eigs_all']` (utils/SIMCA.py:88): the whole spectrum from
    ocm_eigh_f64, against the reference's values at the north-star shape."""
    from utils import SIMCA

    g = _load(golden_dir, "simca_ns.npz")
    X_fit, _, k = _regen(g)
    est = SIMCA(n_components=k, model_class=0, verbose=False)
    with contextlib.redirect_stdout(io.StringIO()):
        est.fit(X_fit, np.zeros(len(X_fit), dtype=np.int64))
    got = est._model[0]["eigs_all"]
    ref = g["eigs_all"]
    assert got.shape == ref.shape
    np.testing.assert_allclose(got[:k], ref[:k], rtol=1e-5)
    # the float32 SVD's tail is noise-level: compare to its scale
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-5 * ref[0])
