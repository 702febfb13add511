"""Drop-in SIMCA on the GPU against the reference's golden vectors and the
CPU oracle (same inputs).  Tolerances: Q, T² rtol 1e-4 (with
an absolute floor of 1e-5·median for rows near zero), limits rtol 1e-5
(percentile/moment-based 1e-4), decisions identical outside the band
|dred − D_lim| < 1e-4·D_lim."""
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


def _est(g, **kw):
    from utils import SIMCA

    classes = list(g["classes"])
    ks = [int(g[f"c{i}_k"]) for i in range(len(classes))]
    return SIMCA(n_components=ks if len(classes) > 1 else ks[0],
                 model_class=None if len(classes) > 1 else int(classes[0]), verbose=False, **kw), classes, ks


@pytest.mark.parametrize("name", ["simca_a.npz", "simca_b.npz", "simca_multi.npz"])
def test_fit_arrays_vs_reference(golden_dir, name):
    g = _load(golden_dir, name)
    est, classes, ks = _est(g)
    est.fit(g["X_fit"], g["y_fit"])
    for i, cls in enumerate(classes):
        m = est._model[cls]
        k = ks[i]
        np.testing.assert_allclose(m["xmean"], g[f"c{i}_xmean"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(m["eigs_all"][:k], g[f"c{i}_eigs_all"][:k], rtol=1e-5)
        np.testing.assert_allclose(m["P"], g[f"c{i}_P"], atol=2e-4)
        np.testing.assert_allclose(m["T"], g[f"c{i}_T"], rtol=1e-4, atol=1e-3)
        close(m["T2"], g[f"c{i}_T2"])
        close(m["Q"], g[f"c{i}_Q"])
        assert m["Q"].dtype == np.float32 and m["T2"].dtype == np.float64
        assert m["n_samples"] == int(g[f"c{i}_n"]) and m["n_components"] == k


@pytest.mark.parametrize("name", ["simca_a.npz", "simca_b.npz", "simca_multi.npz"])
def test_limits_and_decisions_all_combos(golden_dir, name):
    from oracle import simca_oracle as O

    g = _load(golden_dir, name)
    n_checked = 0
    for ci, combo in enumerate(g["combos"]):
        ty, t2, ql = str(combo).split("|")
        est, classes, ks = _est(g, type=ty, t2lim=t2, qlim=ql)
        with contextlib.redirect_stdout(io.StringIO()):
            est.fit(g["X_fit"], g["y_fit"])
            pred = est.predict(g["X_test"])
        assert pred.shape == (len(g["X_test"]), len(classes)) and pred.dtype == np.float64
        for j, cls in enumerate(classes):
            m = est._model[cls]
            lim_rtol = 1e-4 if (t2 in ("perc", "chi2pom")) else 1e-5
            np.testing.assert_allclose(m["T2_limit"], g["T2_limit"][ci][j], rtol=lim_rtol, err_msg=f"{combo}")
            np.testing.assert_allclose(m["Q_limit"], g["Q_limit"][ci][j], rtol=1e-4, err_msg=f"{combo}")
            np.testing.assert_allclose(m["D_limit"], g["D_limit"][ci][j], rtol=1e-4, err_msg=f"{combo}")
        if ty == "dd":
            assert est._t2dof == g["t2dof"][ci][0] and est._qdof == g["qdof"][ci][0]
        m0 = est._model[classes[0]]
        np.testing.assert_allclose(m0["T2red"][0], g["t2red0"][ci], rtol=1e-4)
        np.testing.assert_allclose(m0["Qred"][0], g["qred0"][ci], rtol=1e-4)
        # decisions: identical to the reference outside the tolerance band
        orc = O.OracleSIMCA(n_components=est.n_components if len(classes) > 1 else est.n_components[0],
                            model_class=None if len(classes) > 1 else int(classes[0]), type=ty, t2lim=t2, qlim=ql)
        with contextlib.redirect_stdout(io.StringIO()):
            orc.fit(g["X_fit"], g["y_fit"])
        ref = g["pred"][ci].astype(np.float64)
        for j, cls in enumerate(classes):
            d = orc.dred(g["X_test"], cls)
            dl = orc._model[cls]["D_limit"]
            clear = np.abs(d - dl) > BAND * abs(dl)
            np.testing.assert_array_equal(pred[clear, j], ref[clear, j], err_msg=f"{combo} class {cls}")
            n_checked += int(clear.sum())
    assert n_checked > 0


@pytest.mark.parametrize("name", ["simca_a.npz", "simca_b.npz"])
def test_fit_and_limits_with_bf16x3_gram(golden_dir, name):
    """The same reference parity with the Gram on the exact bf16×3 split."""
    from ocm import engine

    prev = engine.set_gram_mode("bf16x3")
    try:
        test_fit_arrays_vs_reference(golden_dir, name)
        test_limits_and_decisions_all_combos(golden_dir, name)
    finally:
        engine.set_gram_mode(prev)


@pytest.mark.parametrize("name", ["simca_a.npz", "simca_b.npz", "simca_multi.npz"])
def test_transform_vs_reference(golden_dir, name):
    g = _load(golden_dir, name)
    est, classes, ks = _est(g)
    est.fit(g["X_fit"], g["y_fit"])
    T2, T2red, Q, Qred = est.transform(g["X_test"])
    close(T2, g["tr_T2"], rtol=2e-4)
    close(Q, g["tr_Q"], rtol=2e-4)
    m = est._model[classes[-1]]
    np.testing.assert_allclose(T2red, T2 / m["T2_limit"], rtol=1e-12)
    np.testing.assert_allclose(Qred, Q / m["Q_limit"], rtol=1e-6)


def test_metrics_and_score(golden_dir):
    g = _load(golden_dir, "simca_a.npz")
    est, classes, ks = _est(g)
    est.fit(g["X_fit"], g["y_fit"])
    est.predict(g["X_test"], y_true=g["y_test"])
    ref = json.loads(str(g["metrics_json"]))["0"]
    for key in ("TP", "TN", "FP", "FN"):
        assert int(est.metrics[0][key]) == ref[key]
    s = est.score(g["X_test"], g["y_test"])
    assert np.isfinite(s)


def test_score_pinned_to_reference(golden_dir):
    """SIMCA.score (utils/SIMCA.py:268-278) returns the reference's value: the
    2-D prediction matrix and the list model_class broadcast (one class → an
    m×m comparison, specificity 5.5 on simca_a; three classes → ValueError)."""
    pins = _load(golden_dir, "score.npz")
    g = _load(golden_dir, "simca_a.npz")
    est, _, _ = _est(g)
    est.fit(g["X_fit"], g["y_fit"])
    with contextlib.redirect_stdout(io.StringIO()):
        np.testing.assert_allclose(est.score(g["X_test"], g["y_test"]), pins["a_score"], rtol=1e-12)
    gm = _load(golden_dir, "simca_multi.npz")
    est, _, _ = _est(gm)
    est.fit(gm["X_fit"], gm["y_fit"])
    assert str(pins["multi_error"]) == "ValueError"
    with contextlib.redirect_stdout(io.StringIO()), pytest.raises(ValueError):
        est.score(gm["X_test"], gm["y_test"])


def test_device_resident_inputs(golden_dir):
    import torch

    g = _load(golden_dir, "simca_b.npz")
    est, classes, ks = _est(g)
    X = torch.from_numpy(g["X_fit"]).cuda()
    y = torch.from_numpy(g["y_fit"]).cuda()
    est.fit(X, y)
    pred = est.predict(torch.from_numpy(g["X_test"]).cuda())
    assert isinstance(pred, torch.Tensor) and pred.is_cuda
    est2, _, _ = _est(g)
    est2.fit(g["X_fit"], g["y_fit"])
    np.testing.assert_array_equal(pred.cpu().numpy(), est2.predict(g["X_test"]))


def test_sklearn_protocol_clone():
    from sklearn.base import clone
    from utils import SIMCA

    est = SIMCA(n_components=3, type="ci", qlim="chi2box", verbose=False)
    c = clone(est)
    assert c.get_params() == est.get_params()


def test_errors_mirror_reference():
    from utils import SIMCA

    X = np.random.default_rng(0).standard_normal((50, 8)).astype(np.float32)
    y = np.repeat([0, 1], 25)
    with pytest.raises(ValueError):
        SIMCA(n_components=[2, 3, 4], verbose=False).fit(X, y)
    with pytest.raises(UnboundLocalError):
        SIMCA(n_components=2, model_class=0, t2lim="nope", verbose=False).fit(X, y)


def test_device_resident_full_api(golden_dir):
    """Every public entry point of the drop-in with device tensors (the
    reference only sees NumPy; the drop-in keeps device inputs on the device):
    predict with y_true (metrics), transform, score, the _model keys and the
    pca_model facade — against the same calls on NumPy inputs."""
    import contextlib
    import io

    import torch

    g = _load(golden_dir, "simca_multi.npz")
    Xf, yf, Xt = g["X_fit"], g["y_fit"], g["X_test"]
    yt = g["y_test"]
    a = _est(g)[0].fit(torch.from_numpy(Xf).cuda(), torch.from_numpy(yf).cuda())
    b = _est(g)[0].fit(Xf, yf)
    Xd, yd = torch.from_numpy(Xt).cuda(), torch.from_numpy(yt).cuda()
    with contextlib.redirect_stdout(io.StringIO()):
        pa = a.predict(Xd, y_true=yd)
        pb = b.predict(Xt, y_true=yt)
    np.testing.assert_array_equal(pa.cpu().numpy(), pb)
    for cls in b.model_class:
        for key in ("TP", "TN", "FP", "FN"):
            assert a.metrics[cls][key] == b.metrics[cls][key]
    ta, tb = a.transform(Xd), b.transform(Xt)
    for u, v in zip(ta, tb):
        np.testing.assert_allclose(u.cpu().numpy() if hasattr(u, "cpu") else u, v, rtol=1e-6)
    # the reference's score() raises on three classes (list model_class broadcast, score.npz)
    with contextlib.redirect_stdout(io.StringIO()), pytest.raises(ValueError):
        a.score(Xd, yd)
    ga = _load(golden_dir, "simca_a.npz")
    sa = _est(ga)[0].fit(torch.from_numpy(ga["X_fit"]).cuda(), torch.from_numpy(ga["y_fit"]).cuda())
    sb = _est(ga)[0].fit(ga["X_fit"], ga["y_fit"])
    with contextlib.redirect_stdout(io.StringIO()):
        np.testing.assert_allclose(sa.score(torch.from_numpy(ga["X_test"]).cuda(), torch.from_numpy(ga["y_test"]).cuda()),
                                   sb.score(ga["X_test"], ga["y_test"]), rtol=1e-12)
    for cls in b.model_class:
        ma, mb = a._model[cls], b._model[cls]
        for key in ("T2_limit", "Q_limit", "D_limit", "n_samples", "n_components"):
            np.testing.assert_allclose(ma[key], mb[key], rtol=1e-12)
        for key in ("xmean", "P", "T", "T2", "Q", "invcovT"):
            u = ma[key]
            np.testing.assert_allclose(u.cpu().numpy() if hasattr(u, "cpu") else u, mb[key], rtol=1e-5, atol=1e-7)
        Ta = ma["pca_model"].transform(Xd)
        np.testing.assert_allclose(Ta.cpu().numpy(), mb["pca_model"].transform(Xt), rtol=1e-5, atol=1e-6)
