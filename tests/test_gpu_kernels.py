"""Kernel-level parity on the GPU: every libocm entry point against the CPU
oracle / a float64 NumPy reference of the same op, on seeded inputs."""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]


@pytest.fixture(scope="module")
def eng():
    from ocm import engine

    return engine


@pytest.fixture(params=["f32", "bf16x3", "i8x3", "i8x3k32"])
def gram_mode(request):
    """All Gram kernels: FP32 MFMA, the bf16×3 split on bf16 MFMA and the int8
    digit split on integer MFMA (the default; on the 32x32x32 and on the
    16x16x64 instruction), chosen through the explicit mode argument of
    ocm_gram_f32_ex."""
    from ocm import engine

    prev = engine.set_gram_mode(request.param)
    yield request.param
    engine.set_gram_mode(prev)


def _dev(a):
    import torch

    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


@pytest.mark.parametrize("n,p", [(5000, 300), (777, 128), (4100, 96), (3000, 1000)])
def test_gram_matches_fp64(eng, gram_mode, n, p):
    rng = np.random.default_rng(n + p)
    X = (rng.standard_normal((n, p)) * rng.uniform(0.1, 3, p) + 2.0).astype(np.float32)
    Xd = _dev(X)
    shift = _dev(X[:17].mean(0).astype(np.float32))
    G, cs = eng.gram(Xd, None, [0, n], shift)
    Y = X.astype(np.float64) - shift.cpu().numpy().astype(np.float64)
    Gref = Y.T @ Y
    np.testing.assert_allclose(G[0].cpu().numpy(), Gref, rtol=2e-6, atol=2e-6 * np.abs(Gref).max())
    np.testing.assert_allclose(cs[0].cpu().numpy(), Y.sum(0), rtol=1e-6, atol=1e-6 * np.abs(Y).sum(0).max())


def test_gram_segments_and_rows(eng, gram_mode):
    import torch

    rng = np.random.default_rng(3)
    n, p = 6000, 200
    X = rng.standard_normal((n, p)).astype(np.float32)
    rows = np.sort(rng.choice(n, 4500, replace=False))
    seg = [0, 1000, 1000, 2600, 4500]  # includes an empty segment
    Xd = _dev(X)
    shift = torch.zeros(p, dtype=torch.float32, device="cuda")
    G, cs = eng.gram(Xd, _dev(rows.astype(np.int64)), seg, shift)
    Xs = X[rows].astype(np.float64)
    for s in range(len(seg) - 1):
        Y = Xs[seg[s]:seg[s + 1]]
        ref = Y.T @ Y
        np.testing.assert_allclose(G[s].cpu().numpy(), ref, rtol=2e-6, atol=2e-6 * max(np.abs(ref).max(), 1))
        np.testing.assert_allclose(cs[s].cpu().numpy(), Y.sum(0), rtol=1e-6, atol=1e-7 * np.abs(Y).sum(0).max())


def test_cov_and_mean(eng, gram_mode):
    from oracle.simca_oracle import synth_spectra

    X = synth_spectra(4000, 300, 8, rank=20, seed=5)
    Xd = _dev(X)
    shift = eng.cast_f32(eng.colmean(Xd, None, 64))
    G, cs = eng.gram(Xd, None, [0, 4000], shift)
    C, mean = eng.cov_from_gram([(1.0, G[0], cs[0])], shift, 4000)
    Xf = X.astype(np.float64)
    # y = x − shift is formed in float32 (≤ 6e-8·|y| per element) before the f64
    # sums; the reference's own float32 mean (sklearn) is no better than 1e-7
    np.testing.assert_allclose(mean.cpu().numpy(), Xf.mean(0), rtol=0, atol=2e-7)
    Cref = np.cov(Xf, rowvar=False)
    np.testing.assert_allclose(C.cpu().numpy(), Cref, rtol=1e-5, atol=1e-6 * np.abs(Cref).max())


@pytest.mark.parametrize("p,k", [(300, 8), (256, 20), (48, 5), (1000, 12)])
def test_eig_topk_and_thetas(eng, p, k):
    rng = np.random.default_rng(p * 31 + k)
    # spectrum with a gap at k and a long tail
    lam = np.concatenate([np.linspace(50, 10, k), np.geomspace(1.0, 1e-3, p - k)])
    Qm, _ = np.linalg.qr(rng.standard_normal((p, p)))
    C = (Qm * lam) @ Qm.T
    C = 0.5 * (C + C.T)
    Cd = _dev(C)
    evals, evecs, theta, iters = eng.eig_topk(Cd, k, 2)
    w, V = np.linalg.eigh(C)
    w, V = w[::-1], V[:, ::-1]
    np.testing.assert_allclose(evals.cpu().numpy(), w[:k], rtol=1e-10)
    P = evecs.cpu().numpy()
    for i in range(k):
        v = V[:, i] * np.sign(V[np.argmax(np.abs(V[:, i])), i])
        np.testing.assert_allclose(P[i], v, atol=1e-7)
    tail = w[k:]
    np.testing.assert_allclose(theta.cpu().numpy(), [tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()],
                               rtol=1e-8)


@pytest.mark.parametrize("rank", [12, 25])
def test_eig_rank_deficient_block(eng, rank):
    """C of rank < b = 32 (fewer spectra than the block width): the plain
    iterations' CholQR meets zero columns, which the factor replaces by
    pseudo-random ones — including in the launch that would otherwise hand
    its Gram to the next one (k_cvq32<true>, round 5).  Eigenpairs and θ as
    eigh's; the zero tail contributes nothing."""
    rng = np.random.default_rng(100 + rank)
    p, k = 256, 6
    lam = np.concatenate([np.linspace(40, 20, k), np.geomspace(1.0, 1e-2, rank - k)])
    Qm, _ = np.linalg.qr(rng.standard_normal((p, rank)))
    C = (Qm * lam) @ Qm.T
    C = 0.5 * (C + C.T)
    evals, evecs, theta, iters = eng.eig_topk(_dev(C), k, 2)
    w, V = np.linalg.eigh(C)
    w, V = w[::-1], V[:, ::-1]
    np.testing.assert_allclose(evals.cpu().numpy(), w[:k], rtol=1e-10)
    P = evecs.cpu().numpy()
    for i in range(k):
        v = V[:, i] * np.sign(V[np.argmax(np.abs(V[:, i])), i])
        np.testing.assert_allclose(P[i], v, atol=1e-7)
    tail = lam[k:]
    np.testing.assert_allclose(theta.cpu().numpy(), [tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()],
                               rtol=1e-8)


def test_eig_no_gap_converges(eng):
    rng = np.random.default_rng(9)
    p, k = 512, 10
    A = rng.standard_normal((2000, p))
    C = np.cov(A, rowvar=False)
    evals, evecs, theta, iters = eng.eig_topk(_dev(C), k, 2)
    w = np.linalg.eigvalsh(C)[::-1]
    np.testing.assert_allclose(evals.cpu().numpy(), w[:k], rtol=1e-8)
    tail = w[k:]
    np.testing.assert_allclose(theta.cpu().numpy()[:2], [tail.sum(), (tail ** 2).sum()], rtol=1e-8)


def test_eig_slow_decay_adaptive_rayleigh_ritz(eng):
    """A spectrum whose k-th / (b+1)-th eigenvalue ratio is close to 1 (the
    derivative spectra of the nuts preprocessing converge in ~30 iterations):
    the predicted Rayleigh–Ritz schedule must still stop only at the tolerance,
    with eigenpairs and θ equal to eigh's."""
    rng = np.random.default_rng(21)
    p, k = 512, 20
    lam = np.geomspace(100.0, 0.01, p) * (1 + 0.01 * rng.random(p))
    lam = np.sort(lam)[::-1]
    Qm, _ = np.linalg.qr(rng.standard_normal((p, p)))
    C = (Qm * lam) @ Qm.T
    C = 0.5 * (C + C.T)
    evals, evecs, theta, iters = eng.eig_topk(_dev(C), k, 2)
    assert iters > 6  # the slow case really took the adaptive path
    w, V = np.linalg.eigh(C)
    w, V = w[::-1], V[:, ::-1]
    np.testing.assert_allclose(evals.cpu().numpy(), w[:k], rtol=1e-9)
    P = evecs.cpu().numpy()
    for i in range(k):
        v = V[:, i] * np.sign(V[np.argmax(np.abs(V[:, i])), i])
        np.testing.assert_allclose(P[i], v, atol=1e-6)
    tail = w[k:]
    np.testing.assert_allclose(theta.cpu().numpy(), [tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()],
                               rtol=1e-8)


def test_eig_chebyshev_filter_iterations(eng):
    """Round 6: after a failed Rayleigh–Ritz test the eigensolver switches to
    Chebyshev-filtered iterations bounded by that test's Ritz values.  On a
    2048-point geometric spectrum (100 … 0.01) the filter converges in 102
    iterations where plain subspace iteration takes 349
    (profiles/r06j_eig_cheb_ab.jsonl); the bound 160 keeps the filter from
    silently switching off.  Eigenpairs and θ as eigh's."""
    rng = np.random.default_rng(3)
    p, k = 2048, 20
    lam = np.geomspace(100.0, 0.01, p)
    Qm, _ = np.linalg.qr(rng.standard_normal((p, p)))
    C = (Qm * lam) @ Qm.T
    C = 0.5 * (C + C.T)
    evals, evecs, theta, iters = eng.eig_topk(_dev(C), k, 2)
    print("chebyshev iterations:", iters)
    assert 6 < iters <= 160
    w, V = np.linalg.eigh(C)
    w, V = w[::-1], V[:, ::-1]
    np.testing.assert_allclose(evals.cpu().numpy(), w[:k], rtol=1e-9)
    P = evecs.cpu().numpy()
    for i in range(k):
        v = V[:, i] * np.sign(V[np.argmax(np.abs(V[:, i])), i])
        np.testing.assert_allclose(P[i], v, atol=1e-6)
    tail = w[k:]
    np.testing.assert_allclose(theta.cpu().numpy(), [tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()],
                               rtol=1e-8)


def test_inv_evals_pinv_cutoff(eng):
    """ocm_inv_evals_f64 = the diagonal of np.linalg.pinv(diag(λ)) (rcond 1e-15
    relative to max |λ|): tiny and zero eigenvalues map to 0."""
    import torch

    lam = np.array([5.0, 1.0, 3e-15, 6e-15, 0.0, -2.0, 1e-3])
    got = eng.inv_evals(torch.from_numpy(lam).cuda()).cpu().numpy()
    want = np.diag(np.linalg.pinv(np.diag(lam), rcond=1e-15))
    np.testing.assert_allclose(got, want, rtol=1e-14, atol=0)
    assert got[2] == 0.0 and got[4] == 0.0 and got[3] != 0.0


@pytest.mark.parametrize("k", [4, 20, 40])
def test_score_matches_oracle(eng, k):
    import torch
    from oracle.simca_oracle import project_scores, synth_spectra

    n, p = 3000, 520
    X = synth_spectra(n, p, min(k, 20), rank=max(k + 5, 30), seed=k, outlier_frac=0.1)
    Xf = X.astype(np.float64)
    mean = Xf.mean(0)
    w, V = np.linalg.eigh(np.cov(Xf, rowvar=False))
    P = V[:, ::-1][:, :k].T.copy()
    lam = w[::-1][:k]
    A = np.diag(1 / lam)
    T_ref, T2_ref, Q_ref = project_scores(X, P, mean, A)
    out = eng.score(_dev(X), None, n, _dev(P), _dev(mean), _dev(A), want_T=True, want_stats=True)
    np.testing.assert_allclose(out["T"].cpu().numpy(), T_ref, rtol=1e-4, atol=1e-4 * np.abs(T_ref).max())
    np.testing.assert_allclose(out["T2"].cpu().numpy(), T2_ref, rtol=2e-5, atol=1e-6 * np.median(T2_ref))
    np.testing.assert_allclose(out["Q"].cpu().numpy(), Q_ref, rtol=2e-5, atol=1e-6 * np.median(Q_ref))
    st = out["stats"].cpu().numpy()
    np.testing.assert_allclose(st, [T2_ref.sum(), (T2_ref ** 2).sum(), Q_ref.astype(np.float64).sum(),
                                    (Q_ref.astype(np.float64) ** 2).sum()], rtol=1e-6)
    # row-index path (gather) and fused decision
    rows = np.arange(n - 1, -1, -3)
    acc = torch.zeros((len(rows), 2), dtype=torch.float64, device="cuda")
    dec = eng.make_decision("alt", 1 / np.percentile(T2_ref, 90), 1 / np.percentile(Q_ref, 90), np.sqrt(2))
    out2 = eng.score(_dev(X), _dev(rows.astype(np.int64)), len(rows), _dev(P), _dev(mean), _dev(A),
                     decision=dec, accept_out=acc[:, 1:], accept_stride=2)
    np.testing.assert_allclose(out2["Q"].cpu().numpy(), Q_ref[rows], rtol=2e-5, atol=1e-6 * np.median(Q_ref))
    d = np.sqrt((T2_ref[rows] * dec.t2_scale) ** 2 + (Q_ref[rows].astype(np.float64) * dec.q_scale) ** 2)
    clear = np.abs(d - np.sqrt(2)) > 1e-4
    np.testing.assert_array_equal(acc[:, 1].cpu().numpy()[clear], (d < np.sqrt(2))[clear].astype(float))
    assert np.all(acc[:, 0].cpu().numpy() == 0)


@pytest.mark.parametrize("n,p,k", [(5003, 2048, 20), (4097, 2048, 16), (1000, 1024, 17), (777, 512, 10),
                                   (300, 256, 1), (33, 2048, 20), (1, 512, 5), (2000, 520, 20), (1500, 2048, 24)])
def test_score_diag_matches_oracle(eng, n, p, k):
    """ocm_score_f32_diag (A = diag(1/λ), the SIMCA case): the single-pass
    kernel k_score_1p for p ∈ {256, 512, 1024, 2048}, k ≤ 20, and the two-sweep
    fallback for the rest (p = 520, k = 24); ragged tails (m mod 16 ≠ 0, m < 16),
    the row-index gather, the fused decision and the moment partials."""
    import torch
    from oracle.simca_oracle import project_scores, synth_spectra

    X = synth_spectra(n + 64, p, min(k, 20), rank=max(k + 5, 30), seed=n + k, outlier_frac=0.1)
    Xf = X.astype(np.float64)
    mean = Xf.mean(0)
    w, V = np.linalg.eigh(np.cov(Xf, rowvar=False))
    P = V[:, ::-1][:, :k].T.copy()
    lam = w[::-1][:k]
    inv = 1 / lam
    T_ref, T2_ref, Q_ref = project_scores(X[:n], P, mean, np.diag(inv))
    Xd = _dev(X)
    out = eng.score(Xd, None, n, _dev(P), _dev(mean), _dev(inv), want_T=True, want_stats=True)
    np.testing.assert_allclose(out["T"].cpu().numpy(), T_ref, rtol=1e-4, atol=1e-4 * np.abs(T_ref).max())
    np.testing.assert_allclose(out["T2"].cpu().numpy(), T2_ref, rtol=2e-5, atol=1e-6 * np.median(T2_ref))
    np.testing.assert_allclose(out["Q"].cpu().numpy(), Q_ref, rtol=2e-5, atol=1e-6 * np.median(Q_ref))
    q64 = Q_ref.astype(np.float64)
    np.testing.assert_allclose(out["stats"].cpu().numpy(),
                               [T2_ref.sum(), (T2_ref ** 2).sum(), q64.sum(), (q64 ** 2).sum()], rtol=1e-6)
    # same as the general two-sweep kernel with the full matrix
    full = eng.score(Xd, None, n, _dev(P), _dev(mean), _dev(np.diag(inv)), want_T=True)
    np.testing.assert_allclose(out["Q"].cpu().numpy(), full["Q"].cpu().numpy(), rtol=2e-5,
                               atol=1e-6 * np.median(Q_ref))
    # gather + fused decision at a stride, T2/Q/T outputs off
    rows = np.arange(n + 63, -1, -3)[: max(1, (n + 64) // 3)]
    _, T2r, Qr = project_scores(X[rows], P, mean, np.diag(inv))
    acc = torch.zeros((len(rows), 2), dtype=torch.float64, device="cuda")
    dec = eng.make_decision("alt", 1 / np.percentile(T2r, 90), 1 / np.percentile(Qr, 90), np.sqrt(2))
    eng.score(Xd, _dev(rows.astype(np.int64)), len(rows), _dev(P), _dev(mean), _dev(inv), want_T2=False,
              want_Q=False, decision=dec, accept_out=acc[:, 1:], accept_stride=2)
    d = np.sqrt((T2r * dec.t2_scale) ** 2 + (Qr.astype(np.float64) * dec.q_scale) ** 2)
    clear = np.abs(d - np.sqrt(2)) > 1e-4
    np.testing.assert_array_equal(acc[:, 1].cpu().numpy()[clear], (d < np.sqrt(2))[clear].astype(float))
    assert np.all(acc[:, 0].cpu().numpy() == 0)


@pytest.mark.parametrize("offset", [0, 1])
def test_score_diag_strided_and_offset_rows(eng, offset):
    """X a column slice of a wider matrix (ldx > p); offset 1 breaks the 16-B
    alignment and takes the two-sweep kernel.  Data with a large common mean
    (μ ≈ 50σ) checks that the centring happens before the f32 projection."""
    from oracle.simca_oracle import project_scores

    rng = np.random.default_rng(5 + offset)
    n, p, k = 2000, 1024, 12
    W = (rng.standard_normal((n, p + 8)) * 0.02 + 1.0).astype(np.float32)
    W[:, :p] += (rng.standard_normal((n, k)) @ rng.standard_normal((k, p)) * 0.05).astype(np.float32)
    X = W[:, offset:offset + p]
    Xf = X.astype(np.float64)
    mean = Xf.mean(0)
    w, V = np.linalg.eigh(np.cov(Xf, rowvar=False))
    P = V[:, ::-1][:, :k].T.copy()
    inv = 1 / w[::-1][:k]
    T_ref, T2_ref, Q_ref = project_scores(np.ascontiguousarray(X), P, mean, np.diag(inv))
    Wd = _dev(W)
    out = eng.score(Wd[:, offset:offset + p], None, n, _dev(P), _dev(mean), _dev(inv), want_T=True)
    np.testing.assert_allclose(out["T2"].cpu().numpy(), T2_ref, rtol=2e-5, atol=1e-6 * np.median(T2_ref))
    np.testing.assert_allclose(out["Q"].cpu().numpy(), Q_ref, rtol=2e-5, atol=1e-6 * np.median(Q_ref))


def test_decide_types(eng):
    import torch

    rng = np.random.default_rng(1)
    m = 1000
    T2 = rng.gamma(3, 1, m)
    Q = rng.gamma(5, 1, m).astype(np.float32)
    for ty in ["sim", "alt", "ci", "dd"]:
        dec = eng.make_decision(ty, 0.3, 0.2, 1.3)
        acc = torch.zeros(m, dtype=torch.float64, device="cuda")
        t2r, qr, dr = eng.decide(_dev(T2), _dev(Q), dec, want_dred=True, accept_out=acc)
        t, q = T2 * 0.3, Q.astype(np.float64) * 0.2
        ref = {"sim": np.maximum(t, q), "alt": np.sqrt(t * t + q * q), "ci": t + q, "dd": t + q}[ty]
        np.testing.assert_allclose(dr.cpu().numpy(), ref, rtol=1e-14)
        np.testing.assert_array_equal(acc.cpu().numpy(), (ref < 1.3).astype(float))


@pytest.mark.parametrize("n", [1, 2, 7, 1000, 100003])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_percentile(eng, n, dtype):
    rng = np.random.default_rng(n)
    v = (rng.standard_normal(n) * 10).astype(dtype)
    v[: n // 3] = np.abs(v[: n // 3])  # mixed signs, duplicates below
    if n > 10:
        v[5:9] = v[4]
    for pct in [0, 5, 50, 95, 99.9, 100]:
        got = eng.percentile(_dev(v), pct)
        # numpy evaluates the interpolation in the array dtype; so does ocm_percentile
        np.testing.assert_allclose(got, np.percentile(v, pct), rtol=1e-7 if dtype == np.float32 else 1e-15)


def test_sym_pinv(eng):
    rng = np.random.default_rng(2)
    for d in [3, 17, 32, 64]:
        B = rng.standard_normal((d + 5, d))
        A = B.T @ B
        np.testing.assert_allclose(eng.sym_pinv(_dev(A)).cpu().numpy(), np.linalg.pinv(A), rtol=1e-8, atol=1e-10)
    A = np.diag([3.0, 2.0, 0.0])  # rank-deficient -> pseudo-inverse
    np.testing.assert_allclose(eng.sym_pinv(_dev(A)).cpu().numpy(), np.linalg.pinv(A), atol=1e-14)


def test_rowsq_residual(eng):
    rng = np.random.default_rng(4)
    x = rng.standard_normal((777, 333)).astype(np.float32)
    xh = x + 0.01 * rng.standard_normal(x.shape).astype(np.float32)
    q = eng.rowsq_residual(_dev(x), _dev(xh)).cpu().numpy()
    np.testing.assert_allclose(q, ((x.astype(np.float64) - xh) ** 2).sum(1), rtol=1e-6)


def test_rowsq_residual_broadcast_and_strided(eng):
    """ldxh = 0 broadcasts one row (Euclidean latent distance about a mean,
    utils/final_vaesimca.py:510-512); a strided x view is honoured."""
    rng = np.random.default_rng(6)
    z = rng.standard_normal((1001, 32)).astype(np.float32)
    mu = rng.standard_normal(32).astype(np.float32)
    h = eng.rowsq_residual(_dev(z), _dev(mu)).cpu().numpy()
    np.testing.assert_allclose(h, ((z.astype(np.float64) - mu) ** 2).sum(1), rtol=1e-6)
    big = _dev(rng.standard_normal((50, 100)).astype(np.float32))
    view = big[:, 10:42]
    q = eng.rowsq_residual(view, _dev(mu)).cpu().numpy()
    np.testing.assert_allclose(q, ((view.cpu().numpy().astype(np.float64) - mu) ** 2).sum(1), rtol=1e-6)


@pytest.mark.parametrize("n,p", [(9000, 257), (300, 2048)])
def test_gram_i8_digit_split_edge_cases(eng, n, p):
    """i8x3 fixed-point split: per-(1536-row block, column) power-of-two scales
    must cope with zero / constant columns, a far-off shift, ragged
    chunk/block tails, p not a multiple of the 128 tile, a 1e-20-scale column
    and a single huge value (3e5 among N(0, 0.25) values).  The huge value is
    screened by the outlier guard and added back exactly, so the other rows
    of its block keep full precision: the error is normalised by the Gram of
    the rows WITHOUT the outlier (an outer(d, d) over all rows would let the
    outlier hide the loss)."""
    rng = np.random.default_rng(p)
    X = rng.standard_normal((n, p)).astype(np.float32) * np.float32(0.5)
    X[:, 3] = 0.0
    X[:, 5] = 7.25
    X[:, 7] += np.float32(1e4)
    X[n // 3, 11] = np.float32(3e5)
    X[:, -1] = np.float32(1e-20) * rng.standard_normal(n).astype(np.float32)
    Xd = _dev(X)
    shift = _dev(X[:5].mean(0).astype(np.float32))
    G, cs = eng.gram(Xd, None, [0, n], shift, mode="i8x3", chunk_rows=512)
    assert eng.last_gram_marks(0) >= 1
    Y = X.astype(np.float64) - shift.cpu().numpy().astype(np.float64)
    Gref = Y.T @ Y
    Y0 = np.delete(Y, n // 3, axis=0)
    d = np.sqrt(np.maximum(np.einsum("ij,ij->j", Y0, Y0), 1e-300))
    err = np.abs(G[0].cpu().numpy() - Gref) / np.outer(d, d)
    assert err.max() < 2e-6, err.max()
    np.testing.assert_allclose(cs[0].cpu().numpy(), Y.sum(0), rtol=1e-6, atol=1e-6 * np.abs(Y).sum(0).max())


@pytest.mark.parametrize("n,p,chunk", [(20000, 2048, 0), (9000, 257, 512), (5000, 300, 4608)])
def test_gram_i8_kernels_bit_identical(eng, n, p, chunk):
    """k_gram8e (16x16x64, the default launch) and k_gram8d (32x32x32) sum the
    same exact int32 digit products and flush them to f32 in the same order:
    the Grams are bit for bit equal, with segments, a gather list and outlier
    rows.  (The A/B launch variants of k_gram8e live in `make exp` builds only.)"""
    import torch

    rng = np.random.default_rng(p + n)
    X = (rng.standard_normal((n, p)) * rng.uniform(0.1, 3, p) + 1.0).astype(np.float32)
    X[n // 5] *= np.float32(800.0)  # one screened row (exact fix-up in both)
    Xd = _dev(X)
    shift = eng.cast_f32(eng.colmean(Xd, None, 4096))
    rows = _dev(np.sort(rng.choice(n, n - 100, replace=False)).astype(np.int64))
    m = n - 100
    for r, seg in ((None, [0, n]), (rows, [0, m // 3, m // 3, m])):
        Ga, ca = eng.gram(Xd, r, seg, shift, mode="i8x3", chunk_rows=chunk)
        Gb, cb = eng.gram(Xd, r, seg, shift, mode="i8x3k32", chunk_rows=chunk)
        assert torch.equal(Ga, Gb)
        assert torch.equal(ca, cb)


def _outlier_rows(rng, n, frac, lo=100.0, hi=1000.0):
    """Row indices spread over the matrix (one or more per 1536-row block) and
    their scale factors in [lo, hi]."""
    m = max(1, int(round(frac * n)))
    idx = np.sort(rng.choice(n, m, replace=False))
    return idx, rng.uniform(lo, hi, m)


@pytest.mark.parametrize("frac", [0.005, 0.01])
def test_gram_i8_outlier_rows(eng, frac):
    """0.5–1 % of the rows scaled ×100–×1000, spread so that most 1536-row
    blocks hold several: the guarded i8×3 Gram must match fp64 to the same
    relative accuracy (normalised by the clean rows' scale) as on clean data,
    and agree with the FP32-MFMA Gram."""
    from oracle.simca_oracle import synth_spectra

    rng = np.random.default_rng(int(frac * 1e4))
    n, p = 20000, 384
    X = synth_spectra(n, p, 8, rank=24, seed=17)
    idx, f = _outlier_rows(rng, n, frac)
    mu = X.mean(0)
    X[idx] = (mu + (X[idx] - mu) * f[:, None]).astype(np.float32)
    Xd = _dev(X)
    shift = eng.cast_f32(eng.colmean(Xd, None, 4096))
    G, cs = eng.gram(Xd, None, [0, n], shift, mode="i8x3")
    marks = eng.last_gram_marks(0)
    assert 0 < marks <= n // 8
    Y = X.astype(np.float64) - shift.cpu().numpy().astype(np.float64)
    Gref = Y.T @ Y
    clean = np.setdiff1d(np.arange(n), idx)
    d = np.sqrt(np.einsum("ij,ij->j", Y[clean], Y[clean]))
    err = np.abs(G[0].cpu().numpy() - Gref) / np.outer(d, d)
    assert err.max() < 1e-6, err.max()


def test_gram_i8_clean_data_marks_nothing(eng):
    from oracle.simca_oracle import synth_spectra

    X = synth_spectra(12000, 256, 8, rank=24, seed=3, outlier_frac=0.1)
    Xd = _dev(X)
    shift = eng.cast_f32(eng.colmean(Xd, None, 4096))
    eng.gram(Xd, None, [0, 12000], shift, mode="i8x3")
    assert eng.last_gram_marks(0) == 0


def test_gram_i8_heavy_marking_falls_back_to_bf16x3(eng):
    """Scale drift after the sample rows (every later row ×200): more than n/8
    marked rows, so the call recomputes on the bf16×3 split; the result is
    still the Gram."""
    rng = np.random.default_rng(8)
    n, p = 12000, 192
    X = rng.standard_normal((n, p)).astype(np.float32)
    X[5000:] *= np.float32(200.0)
    Xd = _dev(X)
    shift = _dev(np.zeros(p, np.float32))
    G, _ = eng.gram(Xd, None, [0, n], shift, mode="i8x3")
    assert eng.last_gram_marks(0) > n // 8
    Y = X.astype(np.float64)
    Gref = Y.T @ Y
    np.testing.assert_allclose(G[0].cpu().numpy(), Gref, rtol=2e-6, atol=2e-6 * np.abs(Gref).max())


def test_gram_i8_outliers_in_segments_and_gather(eng):
    """The fix-up adds each marked row to its own segment (CV folds) and
    follows the row-index list."""
    rng = np.random.default_rng(21)
    n, p = 9000, 160
    X = rng.standard_normal((n, p)).astype(np.float32)
    rows = np.sort(rng.choice(n, 7000, replace=False)).astype(np.int64)
    hot = rows[[10, 2500, 2501, 5999]]
    X[hot] *= np.float32(500.0)
    seg = [0, 2000, 2000, 4700, 7000]
    Xd = _dev(X)
    import torch

    shift = torch.zeros(p, dtype=torch.float32, device="cuda")
    G, cs = eng.gram(Xd, _dev(rows), seg, shift, mode="i8x3", chunk_rows=1536)
    assert eng.last_gram_marks(0) > 0
    Xs = X[rows].astype(np.float64)
    for s in range(len(seg) - 1):
        Y = Xs[seg[s]:seg[s + 1]]
        ref = Y.T @ Y
        keep = ~np.isin(rows[seg[s]:seg[s + 1]], hot)
        d = np.sqrt(np.maximum(np.einsum("ij,ij->j", Y[keep], Y[keep]), 1e-300))
        if Y.shape[0] == 0:
            assert np.all(G[s].cpu().numpy() == 0)
            continue
        err = np.abs(G[s].cpu().numpy() - ref) / np.outer(d, d)
        assert err.max() < 2e-6, (s, err.max())
        np.testing.assert_allclose(cs[s].cpu().numpy(), Y.sum(0), rtol=1e-6, atol=1e-6 * np.abs(Y).sum(0).max())
