"""float64 spectra: the PCA precision follows the input
dtype as in the reference (utils/SIMCA.py:64-66 — sklearn runs the SVD in
float64 for float64 X; its scores, residuals and Q are then float64).  The
fp64-MFMA Gram, the fp64 scoring kernel and the drop-in on float64 X against
float64 NumPy / the fp64 oracle at fp64-grade tolerances."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n,p", [(5, 64 + 1), (777, 128), (5000, 300), (3001, 1000), (20000, 2048)])
def test_gram_f64_matches_numpy(n, p):
    from ocm import engine

    rng = np.random.default_rng(n + p)
    X = rng.standard_normal((n, p)) * rng.uniform(0.1, 3, p) + 2.0
    Xd = _dev(X)
    shift = X[: min(n, 17)].mean(0).astype(np.float32)
    G, cs = engine.gram(Xd, None, [0, n], _dev(shift))
    Y = X - shift.astype(np.float64)
    Gref = Y.T @ Y
    np.testing.assert_allclose(G[0].cpu().numpy(), Gref, rtol=1e-12, atol=1e-12 * np.abs(Gref).max())
    np.testing.assert_allclose(cs[0].cpu().numpy(), Y.sum(0), rtol=1e-12, atol=1e-12 * np.abs(Y).sum(0).max())


def test_gram_f64_segments_and_rows():
    import torch

    from ocm import engine

    rng = np.random.default_rng(3)
    n, p = 6000, 200
    X = rng.standard_normal((n, p))
    rows = np.sort(rng.choice(n, 4500, replace=False))
    seg = [0, 1000, 1000, 2603, 4500]  # an empty segment, ragged lengths
    shift = torch.zeros(p, dtype=torch.float32, device="cuda")
    G, cs = engine.gram(_dev(X), _dev(rows.astype(np.int64)), seg, shift)
    Xs = X[rows]
    for s in range(len(seg) - 1):
        Y = Xs[seg[s]:seg[s + 1]]
        np.testing.assert_allclose(G[s].cpu().numpy(), Y.T @ Y, rtol=1e-12, atol=1e-11)
        np.testing.assert_allclose(cs[s].cpu().numpy(), Y.sum(0), rtol=1e-12, atol=1e-11)


@pytest.mark.parametrize("n,p,k", [(3001, 256, 7), (5000, 300, 20), (4097, 2048, 20), (2000, 512, 40),
                                   (1500, 1000, 96)])
def test_score_f64_matches_numpy(n, p, k):
    import torch

    from ocm import engine

    rng = np.random.default_rng(k + p)
    X = rng.standard_normal((n, p)) + 1.5
    Pm, _ = np.linalg.qr(rng.standard_normal((p, k)))
    P = Pm.T.copy()
    mu = X.mean(0)
    lam = np.sort(rng.uniform(0.5, 5, k))[::-1]
    out = engine.score(_dev(X), None, n, _dev(P), _dev(mu), _dev(1.0 / lam), want_T=True, want_stats=True)
    Y = X - mu
    T = Y @ P.T
    T2 = (T * T / lam).sum(1)
    Q = ((Y - T @ P) ** 2).sum(1)
    assert out["T"].dtype == torch.float64 and out["Q"].dtype == torch.float64
    np.testing.assert_allclose(out["T"].cpu().numpy(), T, rtol=1e-11, atol=1e-11 * np.abs(T).max())
    np.testing.assert_allclose(out["T2"].cpu().numpy(), T2, rtol=1e-11)
    np.testing.assert_allclose(out["Q"].cpu().numpy(), Q, rtol=1e-10)
    st = out["stats"].cpu().numpy()
    np.testing.assert_allclose(st, [T2.sum(), (T2 ** 2).sum(), Q.sum(), (Q ** 2).sum()], rtol=1e-10)


def test_score_f64_rows_and_decision():
    import torch

    from ocm import engine

    rng = np.random.default_rng(9)
    n, p, k = 5000, 384, 12
    X = rng.standard_normal((n, p))
    rows = np.sort(rng.choice(n, 3333, replace=False)).astype(np.int64)
    P = np.linalg.qr(rng.standard_normal((p, k)))[0].T.copy()
    mu = X.mean(0)
    lam = np.linspace(3, 1, k)
    T2l, Ql = 20.0, 380.0
    dec = engine.make_decision("alt", 1.0 / T2l, 1.0 / Ql, np.sqrt(2))
    acc = torch.full((3333, 2), -1.0, dtype=torch.float64, device="cuda")
    out = engine.score(_dev(X), _dev(rows), 3333, _dev(P), _dev(mu), _dev(1.0 / lam), decision=dec,
                       accept_out=acc[:, 1:], accept_stride=2)
    Y = X[rows] - mu
    T = Y @ P.T
    T2 = (T * T / lam).sum(1)
    Q = ((Y - T @ P) ** 2).sum(1)
    np.testing.assert_allclose(out["T2"].cpu().numpy(), T2, rtol=1e-11)
    np.testing.assert_allclose(out["Q"].cpu().numpy(), Q, rtol=1e-10)
    d = np.sqrt((T2 / T2l) ** 2 + (Q / Ql) ** 2)
    clear = np.abs(d - np.sqrt(2)) > 1e-9
    a = acc.cpu().numpy()
    assert np.all(a[:, 0] == -1.0)
    np.testing.assert_array_equal(a[clear, 1], (d < np.sqrt(2))[clear].astype(float))
    t2r, qr, dr = engine.decide(out["T2"], out["Q"], dec, want_dred=True)
    np.testing.assert_allclose(dr.cpu().numpy(), d, rtol=1e-10)


@pytest.mark.timeout(300)
def test_drop_in_float64_vs_fp64_oracle():
    """SIMCA(...).fit / predict / transform on float64 X (p = 2048, k = 20):
    the fit runs in fp64 end to end, so it meets the fp64 oracle far inside the
    float32 tolerances — eigenvalues 1e-10, limits 1e-9, T²/Q 1e-8 — and the
    ``_model`` arrays are float64 as the reference's."""
    from oracle import simca_oracle as O
    from utils import SIMCA

    X = O.synth_spectra(12000, 2048, 20, rank=40, seed=77, outlier_frac=0.1).astype(np.float64)
    Xf, Xt = X[:10000], X[10000:]
    y = np.zeros(len(Xf), dtype=np.int64)
    est = SIMCA(n_components=20, model_class=0, verbose=False).fit(Xf, y)
    orc = O.OracleSIMCA(n_components=20, model_class=0, precision="gram").fit(Xf, y)
    m, mo = est._model[0], orc._model[0]
    for key in ("T", "P", "Q", "xmean"):
        assert m[key].dtype == np.float64, key
    np.testing.assert_allclose(m["eigs_all"][:20], mo["eigs_all"][:20], rtol=1e-10)
    np.testing.assert_allclose([m["T2_limit"], m["Q_limit"]], [mo["T2_limit"], mo["Q_limit"]], rtol=1e-9)
    np.testing.assert_allclose(m["T2"], mo["T2"], rtol=1e-8)
    np.testing.assert_allclose(m["Q"], mo["Q"], rtol=1e-8)
    pred = est.predict(Xt)[:, 0]
    d = orc.dred(Xt, 0)
    dl = mo["D_limit"]
    clear = np.abs(d - dl) > 1e-7 * dl
    np.testing.assert_array_equal(pred[clear], (d < dl)[clear].astype(float))
    T2, _, Q, _ = est.transform(Xt)
    assert Q.dtype == np.float64


def _near_low_rank(n=6000, p=512, k=20, seed=31):
    """Rank-k spectra (λ₁ ≈ 100) plus an isotropic tail of λ ≈ 1e-8 = 1e-10·λ₁,
    on a baseline of 3: ‖y‖² is ~1e10 × Q, so Q = ‖y‖² − ‖t‖² would keep only
    ≈ 6 of its 16 digits (eps·‖y‖²/Q ≈ 1e-6)."""
    rng = np.random.default_rng(seed)
    scores = rng.standard_normal((n, k)) * np.geomspace(10, 1, k)
    basis = np.linalg.qr(rng.standard_normal((p, k)))[0].T
    return scores @ basis + 1e-4 * rng.standard_normal((n, p)) + 3.0


def test_score_f64_q_is_explicit_residual_near_low_rank():
    """on nearly exact low-rank data Q is the explicit residual
    Σ(x − (t·P + μ))² (utils/SIMCA.py:67-68, 71) to 1e-8 relative — the
    identity ‖y‖² − ‖t‖² misses that by orders of magnitude here."""
    from ocm import engine

    X = _near_low_rank()
    k = 20
    mu = X.mean(0)
    Y = X - mu
    P = np.linalg.svd(Y, full_matrices=False)[2][:k].copy()
    lam = (Y @ P.T).var(0, ddof=1)
    out = engine.score(_dev(X), None, X.shape[0], _dev(P), _dev(mu), _dev(1.0 / lam), want_T=True)
    T = Y @ P.T
    Q = ((Y - T @ P) ** 2).sum(1)
    q_ident = (Y ** 2).sum(1) - (T ** 2).sum(1)
    assert np.max(np.abs(q_ident - Q) / Q) > 1e-7  # the identity is NOT good enough on this data
    np.testing.assert_allclose(out["Q"].cpu().numpy(), Q, rtol=1e-8)
    np.testing.assert_allclose(out["T2"].cpu().numpy(), (T * T / lam).sum(1), rtol=1e-10)


@pytest.mark.timeout(300)
def test_drop_in_float64_near_low_rank_vs_oracle():
    """The drop-in's float64 fit and predict on the same data against the fp64
    oracle (explicit residuals): Q at rtol 1e-6, T² 1e-8, both limits."""
    from oracle import simca_oracle as O
    from utils import SIMCA

    X = _near_low_rank()
    Xf, Xt = X[:5000], X[5000:]
    y = np.zeros(len(Xf), dtype=np.int64)
    est = SIMCA(n_components=20, model_class=0, verbose=False).fit(Xf, y)
    orc = O.OracleSIMCA(n_components=20, model_class=0, precision="gram").fit(Xf, y)
    m, mo = est._model[0], orc._model[0]
    np.testing.assert_allclose(m["Q"], mo["Q"], rtol=1e-6)
    np.testing.assert_allclose(m["T2"], mo["T2"], rtol=1e-8)
    np.testing.assert_allclose([m["T2_limit"], m["Q_limit"]], [mo["T2_limit"], mo["Q_limit"]], rtol=1e-6)
    T2, _, Q, _ = est.transform(Xt)
    _, T2o, Qo = orc._scores(Xt, mo)
    np.testing.assert_allclose(Q, Qo, rtol=1e-6)
    np.testing.assert_allclose(T2, T2o, rtol=1e-8)
