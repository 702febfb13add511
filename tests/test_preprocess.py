"""Spectral preprocessing (ocm/preprocess.py, ocm_snv_savgol_f32).

CPU: the Savitzky–Golay tap tables reproduce scipy.signal.savgol_filter
(mode='interp', incl. edges) for the drivers' settings and others.
GPU: SNV + SG on the device vs NumPy SNV in float32 + SciPy savgol_filter
(the drivers' exact calls): rtol 1e-5 of the output scale.
"""
import numpy as np
import pytest
from scipy.signal import savgol_filter

from conftest import gpu_available
from ocm.preprocess import savgol_taps

SETTINGS = [(5, 2, 1, 1.0), (15, 2, 1, 1.0), (7, 3, 2, 0.5), (9, 2, 0, 1.0), (1, 0, 0, 1.0), (11, 4, 3, 2.0)]


def _apply_taps(x, w, tp):
    p = x.shape[1]
    h = w // 2
    inner, L, R = tp[:w], tp[w:w + h * w].reshape(h, w), tp[w + h * w:].reshape(h, w)
    out = np.empty(x.shape, dtype=np.float64)
    for j in range(p):
        if j < h:
            out[:, j] = x[:, :w] @ L[j]
        elif j >= p - h:
            out[:, j] = x[:, p - w:] @ R[j - (p - h)]
        else:
            out[:, j] = x[:, j - h:j - h + w] @ inner
    return out


@pytest.mark.parametrize("w,po,d,delta", SETTINGS)
def test_savgol_taps_match_scipy(w, po, d, delta):
    x = np.random.default_rng(w).standard_normal((3, 70)).astype(np.float32)
    ref = savgol_filter(x, w, po, deriv=d, delta=delta, axis=1)
    got = _apply_taps(x.astype(np.float64), w, savgol_taps(w, po, d, delta))
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-6 * np.abs(ref).max())


def test_savgol_taps_errors():
    with pytest.raises(ValueError):
        savgol_taps(4, 2)
    with pytest.raises(ValueError):
        savgol_taps(5, 5)


def _snv_ref(x):
    return (x - np.mean(x, axis=1, keepdims=True)) / (np.std(x, axis=1, keepdims=True) + 1e-8)


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")
@pytest.mark.parametrize("snv,setting", [(True, (5, 2, 1, 1.0)), (False, (15, 2, 1, 1.0)), (True, (15, 2, 1, 1.0)),
                                         (True, None), (False, (11, 4, 3, 2.0))])
@pytest.mark.parametrize("p", [517, 2048, 1028, 36, 4096])
def test_snv_savgol_device(snv, setting, p):
    """p = 517: the general one-workgroup-per-row kernel; p % 4 == 0 with the
    drivers' filters (none, w = 5, w = 15): the wave-per-row kernel, with a
    partial last 256-column segment (1028), a tiny row (36) and a partial last
    group of four rows (301 rows); p = 4096 (C5 spectra): 67 KB of dynamic LDS
    at w = 15."""
    import torch
    from ocm import preprocess

    rng = np.random.default_rng(3)
    wl = np.linspace(0, 1, p)
    x = (1.0 + 0.4 * wl + 0.3 * np.sin(9 * wl) + 0.02 * rng.standard_normal((301, p))).astype(np.float32)
    ref = _snv_ref(x) if snv else x
    if setting is not None:
        w, po, d, delta = setting
        ref = savgol_filter(ref, w, po, deriv=d, delta=delta, axis=1)
        got = preprocess.snv_savgol(torch.from_numpy(x).cuda(), w, po, d, delta, snv=snv)
    else:
        got = preprocess.snv(torch.from_numpy(x).cuda())
    got = got.cpu().numpy()
    assert got.dtype == np.float32
    np.testing.assert_allclose(got, ref, rtol=0, atol=1e-5 * np.abs(ref).max())


@pytest.mark.gpu
@pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")
def test_mahalanobis_outlier_mask_device():
    """vs the drivers' NumPy/sklearn screen (exact fp64 PCA here): identical
    keep-masks outside a 1e-6 band around the threshold."""
    import torch
    from ocm import preprocess
    from oracle import simca_oracle as O

    X = O.synth_spectra(3000, 256, 10, rank=24, seed=8, outlier_frac=0.05)
    mask, thr = preprocess.mahalanobis_outlier_mask(torch.from_numpy(X).cuda(), 10)
    Xc = X.astype(np.float64) - X.mean(0, dtype=np.float64)
    w, V = np.linalg.eigh(Xc.T @ Xc / (len(X) - 1))
    P = V[:, ::-1][:, :10]
    T = Xc @ P
    d = T - T.mean(0)
    md = np.sqrt(np.einsum("ij,jk,ik->i", d, np.linalg.pinv(np.cov(T, rowvar=False)), d))
    ref_thr = np.percentile(md, 95)
    np.testing.assert_allclose(thr, ref_thr, rtol=1e-5)
    band = np.abs(md - ref_thr) > 1e-5 * ref_thr
    np.testing.assert_array_equal(mask.cpu().numpy()[band], (md <= ref_thr)[band])
    assert abs(int(mask.sum()) - int(0.95 * len(X))) <= 2


@pytest.mark.parametrize("snv,setting", [(True, (5, 2, 1, 1.0)), (False, (15, 2, 1, 1.0)), (True, (15, 2, 1, 1.0)),
                                         (True, (9, 2, 0, 1.0)), (False, (7, 3, 2, 0.5)), (True, None)])
def test_lazy_view_formula_matches_scipy(snv, setting):
    """The float32 formula every fused kernel applies (include/ocm.h ocm_prep,
    restated in oracle.prep_fused_f32) is the drivers' SNV + savgol_filter to
    float32 rounding: 2e-6 of the output scale, on spectra with a large
    baseline (the raw differences keep it from costing precision)."""
    from oracle.simca_oracle import prep_fused_f32, preprocess_reference

    rng = np.random.default_rng(11)
    p = 300
    wl = np.linspace(0, 1, p)
    x = (50.0 + 4 * wl + 0.3 * np.sin(9 * wl) + 0.02 * rng.standard_normal((64, p))).astype(np.float32)
    if setting is None:
        w, po, d, delta = 0, 0, 0, 1.0
        tp = None
    else:
        w, po, d, delta = setting
        tp = savgol_taps(w, po, d, delta)
    ref = preprocess_reference(x.astype(np.float64), w, po, d, delta, snv)
    got = prep_fused_f32(x, w, tp, d, snv)
    np.testing.assert_allclose(got, ref, rtol=0, atol=2e-6 * np.abs(ref).max())
