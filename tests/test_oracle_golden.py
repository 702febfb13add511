"""Pin the CPU oracle against the reference's own outputs (tests/golden/*.npz,
made by tests/golden/make_golden.py from /root/reference).  CPU only."""
import json
import os

import numpy as np
import pytest

from oracle import simca_oracle as O

RT_LIM = 1e-5      # limits: scalar F/χ²/JM formulas on eigenvalues
RT_Q = 1e-4        # Q, T² (SURVEY.md §8c proposed tolerances)
BAND = 1e-4        # decisions compared outside |dred-Dlim|/Dlim < BAND
FLOOR = 1e-5       # absolute noise floor for per-row distances, × median(|ref|):
                   # the reference's float32 scores carry an absolute error ∝ row norm


def close(a, b, rtol=RT_Q, floor=FLOOR, **kw):
    b = np.asarray(b)
    np.testing.assert_allclose(a, b, rtol=rtol, atol=floor * float(np.median(np.abs(b))), **kw)


def _load(golden_dir, name):
    path = os.path.join(golden_dir, name)
    if not os.path.exists(path):
        pytest.skip(f"missing fixture {name}")
    return dict(np.load(path, allow_pickle=False))


@pytest.mark.parametrize("name", ["simca_a.npz", "simca_b.npz", "simca_multi.npz"])
def test_oracle_fit_arrays(golden_dir, name):
    g = _load(golden_dir, name)
    classes = list(g["classes"])
    ks = [int(g[f"c{i}_k"]) for i in range(len(classes))]
    nc = ks if len(classes) > 1 else ks[0]
    est = O.OracleSIMCA(n_components=nc, model_class=None if len(classes) > 1 else int(classes[0]))
    est.fit(g["X_fit"], g["y_fit"])
    for i, cls in enumerate(classes):
        m = est._model[cls]
        k = ks[i]
        np.testing.assert_allclose(m["xmean"], g[f"c{i}_xmean"], rtol=1e-5, atol=1e-6)
        ev = g[f"c{i}_eigs_all"]
        np.testing.assert_allclose(m["eigs_all"][:k], ev[:k], rtol=1e-5)
        th_ref = O.tail_thetas(ev, k)
        np.testing.assert_allclose(m["thetas"], th_ref, rtol=1e-4)
        # loadings: same sign convention (svd_flip u_based_decision=False)
        np.testing.assert_allclose(m["P"], g[f"c{i}_P"], atol=2e-4)
        np.testing.assert_allclose(m["T"], g[f"c{i}_T"], rtol=1e-4, atol=1e-3)
        ic = g[f"c{i}_invcovT"]  # off-diagonals are float32-SVD noise in the reference
        np.testing.assert_allclose(m["invcovT"], ic, rtol=1e-4, atol=1e-5 * np.abs(np.diag(ic)).max())
        close(m["T2"], g[f"c{i}_T2"])
        close(m["Q"], g[f"c{i}_Q"])
        assert m["Q"].dtype == g[f"c{i}_Q"].dtype == np.float32
        assert m["T2"].dtype == np.float64


@pytest.mark.parametrize("name", ["simca_a.npz", "simca_b.npz", "simca_multi.npz"])
def test_oracle_limits_and_decisions(golden_dir, name):
    g = _load(golden_dir, name)
    classes = list(g["classes"])
    ks = [int(g[f"c{i}_k"]) for i in range(len(classes))]
    nc = ks if len(classes) > 1 else ks[0]
    mc = None if len(classes) > 1 else int(classes[0])
    n_checked = 0
    for ci, combo in enumerate(g["combos"]):
        ty, t2, ql = str(combo).split("|")
        est = O.OracleSIMCA(n_components=nc, model_class=mc, type=ty, t2lim=t2, qlim=ql)
        est.fit(g["X_fit"], g["y_fit"])
        for j, cls in enumerate(classes):
            m = est._model[cls]
            np.testing.assert_allclose(m["T2_limit"], g["T2_limit"][ci][j], rtol=RT_LIM if t2 != "perc" else 1e-4,
                                       err_msg=f"{combo} T2_limit")
            np.testing.assert_allclose(m["Q_limit"], g["Q_limit"][ci][j], rtol=1e-4, err_msg=f"{combo} Q_limit")
            np.testing.assert_allclose(m["D_limit"], g["D_limit"][ci][j], rtol=1e-4, err_msg=f"{combo} D_limit")
        if ty == "dd":
            assert est.st.t2dof == g["t2dof"][ci][0] and est.st.qdof == g["qdof"][ci][0]
        m0 = est._model[classes[0]]
        np.testing.assert_allclose(m0["T2red"][0], g["t2red0"][ci], rtol=1e-4)
        np.testing.assert_allclose(m0["Qred"][0], g["qred0"][ci], rtol=1e-4)
        pred = est.predict(g["X_test"])
        ref = g["pred"][ci].astype(np.float64)
        for j, cls in enumerate(classes):
            d = est.dred(g["X_test"], cls)
            dl = est._model[cls]["D_limit"]
            clear = np.abs(d - dl) > BAND * abs(dl)
            np.testing.assert_array_equal(pred[clear, j], ref[clear, j], err_msg=f"{combo} class {cls}")
            n_checked += int(clear.sum())
    assert n_checked > 0


@pytest.mark.parametrize("name", ["simca_a.npz", "simca_b.npz", "simca_multi.npz"])
def test_oracle_transform(golden_dir, name):
    g = _load(golden_dir, name)
    classes = list(g["classes"])
    ks = [int(g[f"c{i}_k"]) for i in range(len(classes))]
    est = O.OracleSIMCA(n_components=ks if len(classes) > 1 else ks[0],
                        model_class=None if len(classes) > 1 else int(classes[0]))
    est.fit(g["X_fit"], g["y_fit"])
    T2, _, Q, _ = est.transform(g["X_test"])
    # reference transform() predicts with the randomized PCA(k) loadings (P2);
    # the oracle with the full-SVD loadings — the same subspace on gapped data.
    close(T2, g["tr_T2"], rtol=2e-4)
    close(Q, g["tr_Q"], rtol=2e-4)


def test_oracle_metrics(golden_dir):
    g = _load(golden_dir, "simca_a.npz")
    est = O.OracleSIMCA(n_components=int(g["c0_k"]), model_class=0)
    est.fit(g["X_fit"], g["y_fit"])
    est.predict(g["X_test"], y_true=g["y_test"])
    ref = json.loads(str(g["metrics_json"]))["0"]
    got = est.metrics[0]
    for key in ("TP", "TN", "FP", "FN"):
        assert got[key] == ref[key]
    for key in ("sensitivity", "specificity", "accuracy", "efficiency"):
        np.testing.assert_allclose(got[key], ref[key])


@pytest.mark.parametrize("name", ["cv_a.npz", "cv_grid.npz"])
def test_oracle_cv(golden_dir, name):
    g = _load(golden_dir, name)
    grid = json.loads(str(g["param_grid_json"]))
    from itertools import product

    keys = sorted(grid)
    combos = [dict(zip(keys, v)) for v in product(*[grid[k] for k in keys])] if grid else [{}]
    res = O.cross_validate_simca_grid(g["X"], g["y"], 0, int(g["n_splits"]), int(g["LV_min"]), int(g["LV_max"]),
                                      cfg_grid=combos)
    assert [r["params"] for r in res["results"]] == json.loads(str(g["params_json"]))
    np.testing.assert_array_equal([r["LV"] for r in res["results"]], g["LV"])
    np.testing.assert_allclose([r["spec"] for r in res["results"]], g["spec"], atol=0.5)
    np.testing.assert_allclose([r["sens"] for r in res["results"]], g["sens"], atol=0.5)
    assert res["best_LV"] == int(g["best_LV"])


def test_oracle_kfold_layout(golden_dir):
    g = _load(golden_dir, "cv_a.npz")
    y = g["y"]
    splits = list(O.classwise_kfold(len(y), np.flatnonzero(y == 0), int(g["n_splits"])))
    np.testing.assert_array_equal([len(a) for a, _ in splits], g["split_train"])
    np.testing.assert_array_equal([b[0] for _, b in splits], g["split_test_first"])


def test_oracle_qhf(golden_dir):
    g = _load(golden_dir, "qhf.npz")
    q, h, f, qc, hc, fc = O.compute_q_h_f(g["x"], g["x_rec"], g["z"])
    np.testing.assert_allclose(q, g["q"], rtol=1e-4)
    np.testing.assert_allclose(h, g["h"], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(f, g["f"], rtol=1e-4)
    np.testing.assert_allclose([qc, hc, fc], g["crit"], rtol=1e-4)


# ---------------------------------------------------------------------------
# round 2 fixtures: north-star shape, float64 input, score(), VAESIMCA and the
# final_vaesimca inline blocks (all produced by the reference itself)
# ---------------------------------------------------------------------------

def ns_data(g):
    """Regenerate the stored-by-seed inputs of simca_ns.npz / simca_f64.npz."""
    cfg = json.loads(str(g["config_json"]))
    if "n_test" in cfg:  # north star
        X = O.synth_spectra(cfg["n_fit"] + cfg["n_test"], cfg["p"], cfg["k"], rank=cfg["rank"], seed=cfg["seed"],
                            outlier_frac=cfg["outlier_frac"])
        return X[:cfg["n_fit"]], X[cfg["n_fit"]:], cfg["k"]
    X = O.synth_spectra(cfg["n"], cfg["p"], cfg["k"], rank=cfg["rank"], seed=cfg["seed"],
                        outlier_frac=cfg["outlier_frac"], dtype=np.float64)
    return X[:cfg["n_fit"]], X[cfg["n_fit"]:], cfg["k"]


def _oracle_combo_check(g, X_fit, X_test, k, lim_rtol):
    y = np.zeros(len(X_fit), dtype=np.int64)
    n_checked = 0
    for ci, combo in enumerate(g["combos"]):
        ty, t2, ql = str(combo).split("|")
        est = O.OracleSIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql)
        est.fit(X_fit, y)
        m = est._model[0]
        if ci == 0:
            np.testing.assert_allclose(m["xmean"], g["xmean"], rtol=1e-5, atol=1e-6)
            np.testing.assert_allclose(m["eigs_all"][:k], g["eigs_all"][:k], rtol=1e-5)
            np.testing.assert_allclose(m["thetas"], g["thetas"], rtol=1e-4)
            close(m["T2"], g["fit_T2"])
            close(m["Q"], g["fit_Q"])
            T2, _, Q, _ = est.transform(X_test)
            close(T2, g["test_T2"], rtol=2e-4)
            close(Q, g["test_Q"], rtol=2e-4)
        rt = lim_rtol if t2 not in ("perc", "chi2pom") else 1e-4
        np.testing.assert_allclose(m["T2_limit"], g["T2_limit"][ci], rtol=rt, err_msg=f"{combo} T2_limit")
        np.testing.assert_allclose(m["Q_limit"], g["Q_limit"][ci], rtol=1e-4, err_msg=f"{combo} Q_limit")
        np.testing.assert_allclose(m["D_limit"], g["D_limit"][ci], rtol=1e-4, err_msg=f"{combo} D_limit")
        pred = est.predict(X_test)[:, 0]
        d = est.dred(X_test, 0)
        clear = np.abs(d - m["D_limit"]) > BAND * abs(m["D_limit"])
        np.testing.assert_array_equal(pred[clear], g["pred"][ci][clear].astype(np.float64), err_msg=str(combo))
        n_checked += int(clear.sum())
    assert n_checked > 0


def test_oracle_north_star_shape(golden_dir):
    """p = 2048, k = 20 (SURVEY.md §8 north star) against the reference run."""
    g = _load(golden_dir, "simca_ns.npz")
    X_fit, X_test, k = ns_data(g)
    _oracle_combo_check(g, X_fit, X_test, k, RT_LIM)


def test_oracle_float64_input(golden_dir):
    g = _load(golden_dir, "simca_f64.npz")
    X_fit, X_test, k = ns_data(g)
    _oracle_combo_check(g, X_fit, X_test, k, RT_LIM)


def test_oracle_score_pins(golden_dir):
    """utils/SIMCA.py:268-278: predict(X, y_true) then the conformity metrics of
    the 2-D prediction matrix against the LIST model_class (NumPy broadcasting:
    one class → an m×m comparison; three classes → a broadcast error)."""
    pins = _load(golden_dir, "score.npz")
    g = _load(golden_dir, "simca_a.npz")
    est = O.OracleSIMCA(n_components=int(g["c0_k"]), model_class=0)
    est.fit(g["X_fit"], g["y_fit"])
    pred = est.predict(g["X_test"])
    got = O.metrics_conformity(g["y_test"], pred, est.model_class)["specificity"]
    np.testing.assert_allclose(got, pins["a_score"])
    assert str(pins["multi_error"]) == "ValueError"
    gm = _load(golden_dir, "simca_multi.npz")
    est = O.OracleSIMCA(n_components=[2, 3, 4], model_class=None)
    est.fit(gm["X_fit"], gm["y_fit"])
    with pytest.raises(ValueError):
        O.metrics_conformity(gm["y_test"], est.predict(gm["X_test"]), est.model_class)


def test_oracle_vaesimca_pinned(golden_dir):
    """VAESIMCA (VAE_SIMCA.py:215-382) restatement vs the reference class run
    on the vae_a network (same latents μ, ẑ as vae_a.npz)."""
    pins = _load(golden_dir, "vaesimca.npz")
    v = _load(golden_dir, "vae_a.npz")
    first = True
    for ci, combo in enumerate(pins["combos"]):
        ty, t2, ql = str(combo).split("|")
        err = str(pins["errors"][ci])
        if err:
            with pytest.raises(Exception):
                O.vaesimca_fit(v["mu_cal"], v["zhat_cal"], type=ty, t2lim=t2, qlim=ql)
            continue
        mdl = O.vaesimca_fit(v["mu_cal"], v["zhat_cal"], type=ty, t2lim=t2, qlim=ql)
        if first:
            np.testing.assert_allclose(mdl["T2"], pins["fit_T2"], rtol=1e-9)
            np.testing.assert_allclose(mdl["Q"], pins["fit_Q"], rtol=1e-6)
            first = False
        for key in ("T2_limit", "Q_limit", "D_limit"):
            # Q is a float32 torch sum in the script (±1 ulp here): Q-derived limits to 1e-6
            np.testing.assert_allclose(mdl[key], pins[key][ci], rtol=1e-6, err_msg=f"{combo} {key}")
        for key in ("T2dof", "Qdof"):
            ref = pins[key][ci]
            assert (mdl[key] is None and np.isnan(ref)) or mdl[key] == ref, (combo, key)
        acc, T2, Q, _ = O.vaesimca_predict(mdl, v["mu_test"], v["zhat_test"])
        np.testing.assert_array_equal(acc.astype(np.uint8), pins["pred"][ci], err_msg=str(combo))


def test_oracle_final_vaesimca_pinned(golden_dir):
    """utils/final_vaesimca.py:428-436 and :511-533 (extracted statements of the
    reference run on the vae_a latents) vs the restatement."""
    pins = _load(golden_dir, "final_vaesimca.npz")
    v = _load(golden_dir, "vae_a.npz")
    mu, inv, thr, qthr = O.latent_stats(v["mu_cal"], pins["rec_cal"])
    np.testing.assert_allclose(mu, pins["mu_train_mean"], rtol=1e-6)
    np.testing.assert_allclose(inv, pins["cov_inv"], rtol=1e-6, atol=1e-9 * np.abs(pins["cov_inv"]).max())
    np.testing.assert_allclose([thr, qthr], [pins["threshold"], pins["q_threshold"]], rtol=1e-6)
    acc, f, fcrit = O.full_distance_decision(v["mu_test"], pins["mu_train_mean"].astype(np.float32), pins["q_test"])
    np.testing.assert_allclose(f, pins["f"], rtol=1e-6)
    np.testing.assert_allclose(fcrit, pins["fcrit"], rtol=1e-6)  # the script works in float32
    np.testing.assert_array_equal(acc.astype(np.uint8), pins["pred_class0"])
