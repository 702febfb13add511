"""Lazy preprocessed views.

The drivers run SNV then Savitzky–Golay right before SIMCA (simca_nuts.py:47-52
w = 5, p = 2, deriv 1; simca_new_cheese.py:37-39 w = 15 alone;
utils/data_utils.py:57-61).  ``ocm.preprocess.snv_savgol(X, ..., lazy=True)``
returns a view whose transform runs inside the kernels that read it: the
i8×3 quantiser (halo columns through LDS), k_score_1p (the row tile
transformed in registers), the shift / threshold samples and the fix-up.

* the view's values (ocm_prep_apply_f32) = the CPU restatement of the shared
  float32 formula (oracle.prep_fused_f32) and the drivers' NumPy/SciPy calls;
* the fused Gram and the fused scores are BIT-identical to the same kernels
  run on the materialised view (every fused kernel forms the same float32
  values), with gather lists, segments, outlier rows, the row ends and every
  fused window; the fused paths materialise nothing (ocm_prep_materialised);
* the fallback shapes / windows / even-derivative filters (materialised
  inside libocm) give the same results too;
* the drop-in SIMCA on a view vs the fp64 oracle on SciPy-preprocessed X at
  C2 (100k × 2048, k = 20) for (w 5, p 2, d 1, SNV) and (w 15, p 2, d 1,
  no SNV): T², Q rtol 1e-4, limits 1e-5, decisions outside the 1e-4 band.
"""
import contextlib
import io

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

DRIVERS = [(True, 5, 2, 1), (False, 15, 2, 1)]
OTHERS = [(True, 15, 2, 1), (True, None, 0, 0), (True, 5, 2, 0), (False, 5, 2, 2), (True, 9, 2, 1),
          (False, 7, 3, 0)]


def _fused_form(snv, w, d):
    """The forms the fused load paths implement (csrc PrepArgs::fused_form):
    SNV alone, or an odd-derivative filter of window 5 or 15 (every driver's
    deriv 1), SNV optional; the rest is materialised inside libocm."""
    return (w is None and snv) or (w in (5, 15) and d % 2 == 1)


def _spectra(n, p, seed=5, base=1.0):
    from oracle.simca_oracle import synth_spectra

    X = synth_spectra(n, p, 8, rank=24, seed=seed, outlier_frac=0.1)
    return (X + np.float32(base - 1.0)).astype(np.float32)


def _view(Xd, snv, w, po, d):
    from ocm import preprocess

    return preprocess.snv_savgol(Xd, w, po, d, 1.0, snv=snv, lazy=True)


@pytest.mark.parametrize("snv,w,po,d", DRIVERS + OTHERS)
@pytest.mark.parametrize("p", [2048, 300])
def test_view_values(snv, w, po, d, p):
    import torch

    from ocm.preprocess import savgol_taps
    from oracle.simca_oracle import prep_fused_f32, preprocess_reference

    X = _spectra(777, p, base=30.0)
    v = _view(torch.from_numpy(X).cuda(), snv, w, po, d)
    got = v.materialize().cpu().numpy()
    emu = prep_fused_f32(X, w or 0, savgol_taps(w, po, d) if w else None, d, snv)
    ref = preprocess_reference(X, w, po, d, 1.0, snv)
    scale = np.abs(ref).max()
    np.testing.assert_allclose(got, emu, rtol=0, atol=1e-6 * scale)
    np.testing.assert_allclose(got, ref, rtol=0, atol=3e-6 * scale)
    rows = torch.arange(776, -1, -3, device="cuda")
    np.testing.assert_array_equal(v.materialize(rows).cpu().numpy(), got[rows.cpu().numpy()])


def _gram_pair(v, rows, seg, outlier=False):
    import torch

    from ocm import engine

    Y = v.materialize()
    sa = engine.cast_f32(engine.colmean(v, rows, min(4096, seg[-1])))
    sb = engine.cast_f32(engine.colmean(Y, rows, min(4096, seg[-1])))
    assert torch.equal(sa, sb)
    Ga, ca = engine.gram(v, rows, seg, sa)
    ma = engine.last_gram_marks(0)
    Gb, cb = engine.gram(Y, rows, seg, sb)
    mb = engine.last_gram_marks(0)
    assert ma == mb and (ma > 0 or not outlier)
    return Ga, ca, Gb, cb


@pytest.mark.parametrize("snv,w,po,d", DRIVERS + OTHERS)
@pytest.mark.parametrize("n,p", [(20000, 2048), (7000, 512), (5000, 300)])
def test_view_gram_bit_identical(snv, w, po, d, n, p):
    """The quantiser's fused transform = the materialised rows, to the bit:
    identical digits, identical Grams and column sums (contiguous rows and a
    gather list with segments)."""
    import torch

    from ocm.prepview import materialised_count

    X = _spectra(n, p)
    v = _view(torch.from_numpy(X).cuda(), snv, w, po, d)
    fused = p % 4 == 0 and _fused_form(snv, w, d)
    c0 = materialised_count(0)
    Ga, ca, Gb, cb = _gram_pair(v, None, [0, n])
    assert torch.equal(Ga, Gb) and torch.equal(ca, cb)
    rng = np.random.default_rng(n)
    rows = torch.from_numpy(np.sort(rng.choice(n, n - 333, replace=False))).cuda()
    m = n - 333
    Ga, ca, Gb, cb = _gram_pair(v, rows, [0, m // 3, m // 3, m])
    assert torch.equal(Ga, Gb) and torch.equal(ca, cb)
    assert (materialised_count(0) == c0) == fused


def test_view_gram_outlier_rows_bit_identical():
    """Rows the guard screens out are added back by the fix-up, which reads
    the view through the same formula."""
    import torch

    n, p = 20000, 1024
    X = _spectra(n, p)
    X[[7, 4000, 15000]] *= np.float32(400.0)
    X[9000, 100:140] += np.float32(5000.0)
    v = _view(torch.from_numpy(X).cuda(), False, 5, 2, 1)
    Ga, ca, Gb, cb = _gram_pair(v, None, [0, n], outlier=True)
    assert torch.equal(Ga, Gb) and torch.equal(ca, cb)


@pytest.mark.parametrize("snv,w,po,d", DRIVERS + OTHERS)
@pytest.mark.parametrize("n,p", [(20000, 2048), (5000, 300)])
def test_write_through_gram_and_xprime_bit_identical(snv, w, po, d, n, p):
    """Write-through views (lazy="write"): the quantiser
    writes X′ as a side output of the pass that forms it.  X′ = the no-copy
    view's materialised rows to the bit, the Gram and column sums = the
    materialised Gram (segments too), the view then reads as X′ everywhere,
    and nothing is materialised on the fused forms (the others run the eager
    pass into X′ inside ocm_gram_f32_prep_write)."""
    import torch

    from ocm import engine, preprocess
    from ocm.prepview import materialised_count

    X = _spectra(n, p, seed=n + p)
    Xd = torch.from_numpy(X).cuda()
    Y = _view(Xd, snv, w, po, d).materialize()
    for seg in ([0, n], [0, n // 3, n // 3, n]):
        vw = preprocess.snv_savgol(Xd, w, po, d, 1.0, snv=snv, lazy="write")
        sh = engine.cast_f32(engine.colmean(vw, None, 4096))
        assert torch.equal(sh, engine.cast_f32(engine.colmean(Y, None, 4096)))
        c0 = materialised_count(0)
        Ga, ca = engine.gram(vw, None, seg, sh)
        assert materialised_count(0) == c0
        assert vw.written() is not None and torch.equal(vw.written(), Y)
        Gb, cb = engine.gram(Y, None, seg, sh)
        assert torch.equal(Ga, Gb) and torch.equal(ca, cb)
        assert torch.equal(vw.materialize(), Y) and torch.equal(vw[5:9], Y[5:9])
    # a gather list does not write: the view stays lazy
    rows = torch.arange(0, n, 2, device="cuda")
    vw = preprocess.snv_savgol(Xd, w, po, d, 1.0, snv=snv, lazy="write")
    sh = engine.cast_f32(engine.colmean(Y, rows, min(4096, rows.numel())))
    Ga, ca = engine.gram(vw, rows, [0, rows.numel()], sh)
    Gb, cb = engine.gram(Y, rows, [0, rows.numel()], sh)
    assert vw.written() is None and torch.equal(Ga, Gb) and torch.equal(ca, cb)


@pytest.mark.parametrize("frac", [0.002, 0.2])
def test_write_through_outlier_rows(frac):
    """Screened rows on a write-through view: the exact fix-up (few rows) and
    the bf16×3 recompute past n/8 marked rows (which runs on the X′ the
    quantiser has written) = the materialised Gram."""
    import torch

    from ocm import engine, preprocess

    n, p = 8000, 1024
    X = _spectra(n, p, seed=77)
    rng = np.random.default_rng(4)
    bad = rng.choice(n, int(frac * n), replace=False)
    X[bad] *= np.float32(400.0)
    Xd = torch.from_numpy(X).cuda()
    Y = _view(Xd, False, 5, 2, 1).materialize()
    vw = preprocess.snv_savgol(Xd, 5, 2, 1, 1.0, snv=False, lazy="write")
    sh = engine.cast_f32(engine.colmean(Y, None, 4096))
    Ga, ca = engine.gram(vw, None, [0, n], sh)
    ma = engine.last_gram_marks(0)
    Gb, cb = engine.gram(Y, None, [0, n], sh)
    assert ma == engine.last_gram_marks(0) and ma > 0
    assert torch.equal(vw.written(), Y)
    assert torch.equal(Ga, Gb) and torch.equal(ca, cb)


def _score_pair(v, rows, m, k, seed=3):
    import torch

    from ocm import engine

    p = v.shape[1]
    rng = np.random.default_rng(seed)
    P = torch.from_numpy(np.linalg.qr(rng.standard_normal((p, k)))[0].T.copy()).cuda()
    mu = torch.from_numpy(rng.standard_normal(p) * 0.01).cuda()
    A = torch.from_numpy(rng.uniform(0.5, 2.0, k)).cuda()
    dec = engine.make_decision("alt", 0.05, 0.03, 1.4142135623730951)
    acc_a = torch.zeros(m, dtype=torch.float64, device="cuda")
    acc_b = torch.zeros_like(acc_a)
    a = engine.score(v, rows, m, P, mu, A, want_T=True, decision=dec, accept_out=acc_a, want_stats=True)
    Y = v.materialize()
    b = engine.score(Y, rows, m, P, mu, A, want_T=True, decision=dec, accept_out=acc_b, want_stats=True)
    return a, b, acc_a, acc_b


@pytest.mark.parametrize("snv,w,po,d", DRIVERS + OTHERS)
@pytest.mark.parametrize("p,k", [(2048, 20), (2048, 12), (1024, 20), (512, 10), (256, 16)])
def test_view_score_bit_identical(snv, w, po, d, p, k):
    """k_score_1p's in-register transform (neighbour lanes by ds_bpermute,
    halo quads at the wave slices, edge rows at the row ends) = the
    materialised rows: T, T², Q, decisions and moments to the bit."""
    import torch

    from ocm.prepview import materialised_count

    n = 5003
    X = _spectra(n, p, seed=p + k)
    v = _view(torch.from_numpy(X).cuda(), snv, w, po, d)
    c0 = materialised_count(0)
    a, b, acc_a, acc_b = _score_pair(v, None, n, k)
    for key in ("T", "T2", "Q", "stats"):
        assert torch.equal(a[key], b[key]), key
    assert torch.equal(acc_a, acc_b)
    fused = _fused_form(snv, w, d)
    assert (materialised_count(0) == c0) == fused
    rows = torch.arange(n - 1, 0, -2, device="cuda")
    a, b, acc_a, acc_b = _score_pair(v, rows, rows.numel(), k)
    for key in ("T", "T2", "Q", "stats"):
        assert torch.equal(a[key], b[key]), key
    assert torch.equal(acc_a, acc_b)


def _c2_vs_oracle(snv, w, po, d, n=100_000, p=2048, k=20):
    import torch

    from oracle import simca_oracle as O
    from oracle.simca_oracle import preprocess_reference, synth_spectra
    from utils import SIMCA

    X = synth_spectra(n + 20_000, p, k, rank=40, seed=1234, outlier_frac=2000 / 120_000)
    Xp = preprocess_reference(X, w, po, d, 1.0, snv).astype(np.float32)
    Xd = torch.from_numpy(X).cuda()
    fit_v = _view(Xd[:n], snv, w, po, d)
    test_v = _view(Xd[n:], snv, w, po, d)
    y = np.zeros(n, dtype=np.int64)
    for ty, t2, ql in (("alt", "Fdist", "jm"), ("ci", "chi2", "chi2box")):
        est = SIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql, verbose=False)
        with contextlib.redirect_stdout(io.StringIO()):
            est.fit(fit_v, y)
            pred = est.predict(test_v)[:, 0].cpu().numpy()
            orc = O.OracleSIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql, precision="gram")
            orc.fit(Xp[:n], y)
        m, mo = est._model[0], orc._model[0]
        for key in ("T2", "Q"):
            a, b = m[key], mo[key]
            np.testing.assert_allclose(a, b, rtol=1e-4, atol=1e-5 * np.median(b), err_msg=key)
        for key in ("T2_limit", "Q_limit", "D_limit"):
            np.testing.assert_allclose(m[key], mo[key], rtol=1e-5, err_msg=f"{ty} {key}")
        dd = orc.dred(Xp[n:], 0)
        dl = mo["D_limit"]
        clear = np.abs(dd - dl) > 1e-4 * abs(dl)
        np.testing.assert_array_equal(pred[clear], (dd < dl)[clear].astype(np.float64))
        assert 0 < pred.sum() < len(pred)


@pytest.mark.timeout(400)
@pytest.mark.parametrize("snv,w,po,d", DRIVERS)
def test_c2_view_vs_fp64_oracle(snv, w, po, d):
    """C2 (100k × 2048, k = 20) on lazy views of raw X against the fp64
    oracle on SciPy-preprocessed X, the two driver settings."""
    from ocm.prepview import materialised_count

    c0 = materialised_count(0)
    _c2_vs_oracle(snv, w, po, d)
    assert materialised_count(0) == c0  # fit and predict ran on the fused paths


@pytest.mark.parametrize("fast", [True, False])
def test_cv_grid_on_view(fast):
    """cross_validate_simca_grid on a lazy view (fold engine, and the generic
    refit loop slicing X[rows, :]) = the same on the materialised rows."""
    import torch

    from utils import SIMCA, ClasswiseKFoldWithExternalVal, cross_validate_simca_grid
    import utils.CVSIMCA as CVmod

    n, p = 6000, 512
    X = _spectra(n, p, seed=21)
    y = np.zeros(n, dtype=np.int64)
    y[::7] = 1
    v = _view(torch.from_numpy(X).cuda(), True, 5, 2, 1)
    outs = []
    for data in (v, v.materialize()):
        saved = CVmod._fast_grid
        if not fast:
            CVmod._fast_grid = lambda *a, **k: (None, None)
        try:
            with contextlib.redirect_stdout(io.StringIO()):
                outs.append(cross_validate_simca_grid(
                    SIMCA(verbose=False), data, y, ClasswiseKFoldWithExternalVal(n_splits=4, cls_label=0),
                    LV_min=3, LV_max=6, param_grid={"type": ["alt", "sim"]}, print_summary=False,
                    store_predictions=True))
        finally:
            CVmod._fast_grid = saved
    a, b = outs
    assert [(r["LV"], r["spec"], r["sens"]) for r in a["results"]] == \
        [(r["LV"], r["spec"], r["sens"]) for r in b["results"]]
    assert a["best_LV"] == b["best_LV"]
