"""Generate golden vectors by running the REFERENCE implementation.

Run in the build container only (it imports /root/reference, which does not
exist on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 MPLBACKEND=Agg python tests/golden/make_golden.py

Outputs small .npz fixtures next to this script: inputs plus the reference's
outputs.  They are data (inputs and expected outputs), not reference source.

* simca_<name>.npz  — SIMCA fit on X_fit (one class, or three classes for
  'multi') for every type × t2lim × qlim combination: per-fit arrays once
  (xmean, eigs_all, P, invcovT, T, T2, Q, the second-PCA loadings P2 that the
  reference predicts with) and per-combination limits, T2red/Qred on the fit
  set, predictions and transform() outputs on X_test.
* cv_<name>.npz      — cross_validate_simca_grid records (spec/sens/eff per LV).
* qhf.npz            — vae_model.compute_q_h_f on a fixed batch.
* splits.npz         — utils.data_utils.object_aware_splits on synthetic objects.
* vae_<name>.npz     — vae_model.ConvVAE1D (seeded init → state_dict), eval /
  train forward on a fixed batch with seeded ε, both losses, and the latent
  inputs of VAESIMCA (encoder μ, round trip ẑ) on a calibration / test set.

* simca_ns.npz       — north-star shape: p = 2048, k = 20 on 8000 fit rows and
  2000 test rows (the synth_spectra seed and sizes are stored, not X), five
  type × t2lim × qlim combinations: xmean, eigs_all, θ1..θ3 of the tail,
  fit / test T2 and Q, limits, predictions.
* simca_f64.npz      — SIMCA on float64 input (the reference then runs its PCA
  in float64): limits, T2/Q, predictions for three combinations.
* score.npz          — SIMCA.score(X_test, y_test) of the simca_a / simca_multi
  configurations (utils/SIMCA.py:268-278, 2-D y_pred and list class quirk).
* vaesimca.npz       — VAESIMCA (VAE_SIMCA.py:215-382) run on the vae_a network:
  the class is taken from the script's syntax tree (ast) and executed alone —
  the script itself loads private data at import.  Limits, dofs, T2 / Q and
  decisions for every type × t2lim × qlim combination (or the error it raises).
* final_vaesimca.npz — the inline latent-statistics (utils/final_vaesimca.py:
  428-436) and full-distance decision (:511-533) statements, extracted the same
  way and executed on the vae_a latents.
* final_losses.npz   — the script's three losses (:198-224), its reconstruction
  error Q in the X_bce (min-max scaled) and plain branches (:417-425), and the
  seeded state_dict of its ConvVAE1D copy (:72-193).

np.random.seed is set before every fit: the reference's second PCA(k) draws
from NumPy's global RNG (SURVEY.md §8c caveat 1).

    python tests/golden/make_golden.py [ns f64 score vaesimca final final_losses]   # a subset
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("OCM_REFERENCE", "/root/reference")

sys.path.insert(0, REF)
sys.path.insert(0, REPO)  # for oracle.synth_spectra (data generator only)

from oracle.simca_oracle import synth_spectra  # noqa: E402

TYPES = ["sim", "alt", "ci", "dd"]
T2LIMS = ["Fdist", "Fdistrig", "chi2", "perc", "chi2pom"]
QLIMS = ["jm", "chi2box", "perc", "chi2pom"]


def _combos():
    for ty in TYPES:
        if ty == "dd":  # 'dd' forces chi2pom for both limits (utils/SIMCA.py:42-48)
            yield ty, "chi2pom", "chi2pom"
            continue
        for t2 in T2LIMS:
            for ql in QLIMS:
                yield ty, t2, ql


def make_simca(name, X_fit, y_fit, X_test, y_test, n_components, model_class):
    from utils import SIMCA  # reference

    out = {"X_fit": X_fit, "y_fit": y_fit, "X_test": X_test, "y_test": y_test}
    combos = list(_combos())
    out["combos"] = np.array(["|".join(c) for c in combos])
    per_fit_done = False
    lim = {"T2_limit": [], "Q_limit": [], "D_limit": [], "t2dof": [], "t2scfact": [], "qdof": [], "qscfact": []}
    preds = []
    classes = None
    for ty, t2, ql in combos:
        np.random.seed(7)
        est = SIMCA(n_components=n_components, model_class=model_class, type=ty, t2lim=t2, qlim=ql,
                    verbose=False)
        with contextlib.redirect_stdout(io.StringIO()):
            est.fit(X_fit, y_fit)
            pr = est.predict(X_test)
            trans = est.transform(X_test)
        classes = list(est.model_class)
        if not per_fit_done:
            for ci, cls in enumerate(classes):
                m = est._model[cls]
                for key in ("xmean", "eigs_all", "P", "invcovT", "T", "T2", "Q"):
                    out[f"c{ci}_{key}"] = np.asarray(m[key])
                out[f"c{ci}_P2"] = np.asarray(m["pca_model"].components_)
                out[f"c{ci}_mean2"] = np.asarray(m["pca_model"].mean_)
                out[f"c{ci}_k"] = np.int64(m["n_components"])
                out[f"c{ci}_n"] = np.int64(m["n_samples"])
            out["classes"] = np.array(classes)
            per_fit_done = True
        for key in lim:
            vals = []
            for cls in classes:
                m = est._model[cls]
                if key in ("T2_limit", "Q_limit", "D_limit"):
                    vals.append(float(m[key]))
            if key == "t2dof":
                vals = [float(getattr(est, "_t2dof", np.nan))]
            elif key == "t2scfact":
                vals = [float(getattr(est, "_t2scfact", np.nan))]
            elif key == "qdof":
                vals = [float(getattr(est, "_qdof", np.nan))]
            elif key == "qscfact":
                vals = [float(getattr(est, "_qscfact", np.nan))]
            lim[key].append(vals)
        preds.append(pr.astype(np.uint8))
        if "tr_T2" not in out:  # transform() output: the LAST class, loadings P2
            out["tr_T2"] = np.asarray(trans[0], np.float64)
            out["tr_Q"] = np.asarray(trans[2])
        # T2red/Qred are T2/limit (or dof-scaled for dd): keep one class-0 row per combo as a check
        out.setdefault("_t2red0", []).append(float(np.asarray(est._model[classes[0]]["T2red"])[0]))
        out.setdefault("_qred0", []).append(float(np.asarray(est._model[classes[0]]["Qred"])[0]))
    for key, vals in lim.items():
        out[key] = np.array(vals, dtype=np.float64)
    out["pred"] = np.stack(preds)
    out["t2red0"] = np.array(out.pop("_t2red0"))
    out["qred0"] = np.array(out.pop("_qred0"))
    # metrics of the default combo against y_test for the first class
    est = SIMCA(n_components=n_components, model_class=model_class, verbose=False)
    np.random.seed(7)
    with contextlib.redirect_stdout(io.StringIO()):
        est.fit(X_fit, y_fit)
        est.predict(X_test, y_true=y_test)
    out["metrics_json"] = np.array(json.dumps(
        {str(c): {k: float(v) for k, v in est.metrics[c].items()} for c in est.metrics}))
    np.savez_compressed(os.path.join(HERE, f"simca_{name}.npz"), **out)
    print(name, "combos", len(combos), "classes", classes)


def make_cv(name, X, y, n_splits, LV_min, LV_max, param_grid):
    from utils import SIMCA, cross_validate_simca_grid, ClasswiseKFoldWithExternalVal

    np.random.seed(11)
    cv = ClasswiseKFoldWithExternalVal(n_splits=n_splits, cls_label=0)
    with contextlib.redirect_stdout(io.StringIO()):
        res = cross_validate_simca_grid(SIMCA(verbose=False), X, y, cv, LV_min=LV_min, LV_max=LV_max,
                                        param_grid=param_grid, print_summary=False, store_predictions=True)
    recs = res["results"]
    out = {
        "X": X, "y": y, "n_splits": np.int64(n_splits), "LV_min": np.int64(LV_min), "LV_max": np.int64(LV_max),
        "param_grid_json": np.array(json.dumps(param_grid)),
        "params_json": np.array(json.dumps([r["params"] for r in recs])),
        "LV": np.array([r["LV"] for r in recs], dtype=np.int64),
        "spec": np.array([r["spec"] for r in recs]),
        "sens": np.array([r["sens"] for r in recs]),
        "eff": np.array([r["eff"] for r in recs]),
        "pred": np.stack([b["prediction"] for b in res["by_combo"]]).astype(np.uint8),
        "best_LV": np.int64(res["best_LV"]),
        "best_score": np.float64(res["best_score"]),
    }
    splits = list(cv.split(X, y))
    out["split_train"] = np.array([len(a) for a, _ in splits])
    out["split_test_first"] = np.array([b[0] for _, b in splits])
    np.savez_compressed(os.path.join(HERE, f"cv_{name}.npz"), **out)
    print("cv", name, "records", len(recs), "best LV", res["best_LV"])


def make_qhf():
    import torch
    from vae_model import compute_q_h_f

    g = torch.Generator().manual_seed(3)
    x = torch.randn(256, 96, generator=g) + 2.0
    x_rec = x + 0.1 * torch.randn(256, 96, generator=g)
    z = torch.randn(256, 8, generator=g) @ torch.randn(8, 8, generator=g)
    q, h, f, qc, hc, fc = compute_q_h_f(x, x_rec, z)
    np.savez_compressed(os.path.join(HERE, "qhf.npz"), x=x.numpy(), x_rec=x_rec.numpy(), z=z.numpy(),
                        q=q.numpy(), h=h.numpy(), f=f.numpy(), crit=np.array([qc, hc, fc], dtype=np.float64))
    print("qhf done")


VAE_CONFIGS = {
    # name: (input_length, latent_dim, kwargs)
    "a": (96, 8, dict(conv_blocks=2, n_filters=3, kernel_size=7, stride=2, hidden_fc=32)),
    "b": (101, 6, dict(conv_blocks=3, n_filters=2, kernel_size=5, stride=2, hidden_fc=24, activation="gelu",
                       use_batchnorm=False)),
}


def make_vae():
    """vae_model.ConvVAE1D / losses on fixed seeds, plus the latent inputs of
    VAESIMCA (encoder μ and the latent round trip ẑ = enc(dec(μ)))."""
    import torch
    from vae_model import ConvVAE1D, beta_vae_bce_loss, beta_vae_cosine_loss

    for name, (L, d, kw) in VAE_CONFIGS.items():
        g = np.random.default_rng(21)
        wl = np.linspace(0, 1, L)
        base = (1.0 + 0.5 * np.sin(6 * wl)).astype(np.float32)
        x = (base + 0.2 * g.standard_normal((64, L))).astype(np.float32)
        x_cal = (base + 0.2 * g.standard_normal((300, L))).astype(np.float32)
        x_test = (base + 0.2 * g.standard_normal((100, L))).astype(np.float32)
        x_test[60:] += 0.8 * np.exp(-0.5 * ((wl - 0.4) / 0.05) ** 2).astype(np.float32)
        mean, std = x_cal.mean(0), x_cal.std(0) + 1e-3
        torch.manual_seed(0)
        m = ConvVAE1D(L, d, mean, std, **kw)
        out = {"x": x, "x_cal": x_cal, "x_test": x_test, "mean": mean, "std": std,
               "config_json": np.array(json.dumps({"input_length": L, "latent_dim": d, **kw}))}
        sd0 = {k: v.detach().clone() for k, v in m.state_dict().items()}
        for k, v in sd0.items():
            out["sd/" + k] = v.numpy().copy()
        xt = torch.from_numpy(x)
        with torch.no_grad():
            m.eval()
            torch.manual_seed(1)
            x_rec, mu, logvar = m(xt)
            out["eval_x_rec"], out["eval_mu"], out["eval_logvar"] = x_rec.numpy(), mu.numpy(), logvar.numpy()
            out["eval_x_dec"] = (m.decode(mu) * m.spec_std + m.spec_mean).numpy()
            m.train()
            torch.manual_seed(2)
            x_rec_t, mu_t, lv_t = m(xt)
            out["train_x_rec"], out["train_mu"], out["train_logvar"] = x_rec_t.numpy(), mu_t.numpy(), lv_t.numpy()
            l1 = beta_vae_bce_loss(xt, x_rec_t, mu_t, lv_t, beta=0.5)
            l2 = beta_vae_cosine_loss(xt, x_rec_t, mu_t, lv_t, beta=0.5)
            out["bce_loss"] = np.array([float(l1[0]), l1[1], l1[2]])
            out["cos_loss"] = np.array([float(l2[0]), l2[1], l2[2]])
            m.load_state_dict(sd0)  # the train-mode forward above moved the BN running stats
            m.eval()
            for tag, xs in (("cal", x_cal), ("test", x_test)):
                xs_t = torch.from_numpy(xs)
                mu_s, _ = m.encode((xs_t - m.spec_mean) / m.spec_std)
                z_hat, _ = m.encode((m.decode(mu_s) - m.spec_mean) / m.spec_std)
                out[f"mu_{tag}"] = mu_s.numpy()
                out[f"zhat_{tag}"] = z_hat.numpy()
        np.savez_compressed(os.path.join(HERE, f"vae_{name}.npz"), **out)
        print("vae", name, sum(v.numel() for v in m.parameters()), "params")


def make_splits():
    """utils.data_utils.object_aware_splits on a synthetic 3-type object set
    (with NaN rows and shifted outlier pixels)."""
    from utils.data_utils import object_aware_splits

    rng = np.random.default_rng(31)
    p = 40
    wl = np.linspace(0, 1, p)
    data, inputs = {}, {}
    for t, nut in enumerate(["almond", "hazelnut", "peanut"]):
        objs = []
        for o in range(7 + t):
            n_o = int(rng.integers(30, 90))
            base = 1.0 + 0.3 * np.sin((3 + t) * wl) + 0.05 * o
            X = (base + 0.02 * rng.standard_normal((n_o, p))).astype(np.float32)
            X[rng.random(n_o) < 0.05] += 0.3 * np.exp(-0.5 * ((wl - 0.6) / 0.05) ** 2).astype(np.float32)
            if o == 1:
                X[3, 5] = np.nan
            objs.append({"spectral_data": X})
            inputs[f"in/{nut}/{o}"] = X
        data[nut] = objs
    with contextlib.redirect_stdout(io.StringIO()):
        splits, Xts, yts, Xc, Xv, Xti, Xto = object_aware_splits(data, list(data), "peanut", p)
    out = dict(inputs)
    out.update({"Xts": Xts, "yts": yts, "Xc": Xc, "Xv": Xv, "Xti": Xti, "Xto": Xto})
    for nut, d in splits.items():
        for k, v in d.items():
            out[f"split/{nut}/{k}"] = v
    np.savez_compressed(os.path.join(HERE, "splits.npz"), **out)
    print("splits", Xc.shape, Xv.shape, Xti.shape, Xto.shape)


NS = dict(n_fit=8000, n_test=2000, p=2048, k=20, rank=40, seed=2026, outlier_frac=0.1)
NS_COMBOS = [("alt", "Fdist", "jm"), ("sim", "perc", "perc"), ("ci", "chi2", "chi2box"),
             ("dd", "chi2pom", "chi2pom"), ("alt", "Fdistrig", "chi2pom")]


def _tails(eigs, k):
    tail = np.asarray(eigs, dtype=np.float64)[k:]
    return np.array([tail.sum(), (tail ** 2).sum(), (tail ** 3).sum()])


def _simca_combo_run(X_fit, y_fit, X_test, k, combos, seed=7):
    """Per combo: fit + predict + transform with the reference; per-fit arrays once."""
    from utils import SIMCA

    out, per = {}, {"T2_limit": [], "Q_limit": [], "D_limit": []}
    preds, first = [], True
    for ty, t2, ql in combos:
        np.random.seed(seed)
        est = SIMCA(n_components=k, model_class=0, type=ty, t2lim=t2, qlim=ql, verbose=False)
        with contextlib.redirect_stdout(io.StringIO()):
            est.fit(X_fit, y_fit)
            pr = est.predict(X_test)
            tr = est.transform(X_test)
        m = est._model[0]
        if first:
            out["xmean"] = np.asarray(m["xmean"])
            out["eigs_all"] = np.asarray(m["eigs_all"], dtype=np.float64)
            out["thetas"] = _tails(m["eigs_all"], k)
            out["fit_T2"] = np.asarray(m["T2"], dtype=np.float64)
            out["fit_Q"] = np.asarray(m["Q"])
            out["test_T2"] = np.asarray(tr[0], dtype=np.float64)
            out["test_Q"] = np.asarray(tr[2])
            first = False
        for key in per:
            per[key].append(float(m[key]))
        preds.append(np.asarray(pr)[:, 0].astype(np.uint8))
    out["combos"] = np.array(["|".join(c) for c in combos])
    for key, v in per.items():
        out[key] = np.array(v)
    out["pred"] = np.stack(preds)
    return out


def make_northstar():
    """SURVEY.md §8 north-star shape (p = 2048, k = 20) from the reference."""
    from oracle.simca_oracle import synth_spectra

    c = NS
    X = synth_spectra(c["n_fit"] + c["n_test"], c["p"], c["k"], rank=c["rank"], seed=c["seed"],
                      outlier_frac=c["outlier_frac"])
    X_fit, X_test = X[:c["n_fit"]], X[c["n_fit"]:]
    y_fit = np.zeros(c["n_fit"], dtype=np.int64)
    out = _simca_combo_run(X_fit, y_fit, X_test, c["k"], NS_COMBOS)
    out["config_json"] = np.array(json.dumps(c))
    out["fit_T2"] = out["fit_T2"].astype(np.float64)
    np.savez_compressed(os.path.join(HERE, "simca_ns.npz"), **out)
    print("ns", {k: out[k] for k in ("T2_limit", "Q_limit")})


def make_f64():
    """Float64 input: the reference's PCA then runs in float64."""
    from oracle.simca_oracle import synth_spectra

    cfg = dict(n=2600, n_fit=2000, p=256, k=10, rank=24, seed=404, outlier_frac=600 / 2600)
    X = synth_spectra(cfg["n"], cfg["p"], cfg["k"], rank=cfg["rank"], seed=cfg["seed"],
                      outlier_frac=cfg["outlier_frac"], dtype=np.float64)
    X_fit, X_test = X[:cfg["n_fit"]], X[cfg["n_fit"]:]
    y_fit = np.zeros(2000, dtype=np.int64)
    out = _simca_combo_run(X_fit, y_fit, X_test, 10, [("alt", "Fdist", "jm"), ("sim", "chi2", "chi2box"),
                                                      ("dd", "chi2pom", "chi2pom")])
    out["config_json"] = np.array(json.dumps(cfg))  # X regenerates from the seed (float64 synth_spectra)
    np.savez_compressed(os.path.join(HERE, "simca_f64.npz"), **out)
    print("f64", out["Q_limit"])


def make_score_pins():
    """SIMCA.score on the simca_a / simca_multi fixtures (their stored inputs)."""
    from utils import SIMCA

    out = {}
    for name, k, mc in (("a", 4, 0), ("multi", [2, 3, 4], None)):
        g = np.load(os.path.join(HERE, f"simca_{name}.npz"), allow_pickle=False)
        np.random.seed(7)
        est = SIMCA(n_components=k, model_class=mc, verbose=False)
        with contextlib.redirect_stdout(io.StringIO()):
            est.fit(g["X_fit"], g["y_fit"])
            try:
                out[f"{name}_score"] = np.float64(est.score(g["X_test"], g["y_test"]))
                out[f"{name}_error"] = np.array("")
            except Exception as e:  # the reference's list-class quirk can raise
                out[f"{name}_score"] = np.float64(np.nan)
                out[f"{name}_error"] = np.array(type(e).__name__)
    np.savez_compressed(os.path.join(HERE, "score.npz"), **out)
    print("score", {k: v for k, v in out.items()})


def _extract(path, first, last, names=None):
    """Compile the statements of a reference script whose first line lies in
    [first, last] (any nesting depth), or the top-level class ``names``."""
    import ast

    src = open(path).read()
    tree = ast.parse(src)
    if names:
        body = [n for n in tree.body if isinstance(n, ast.ClassDef) and n.name in names]
    else:
        body, seen = [], set()
        for node in ast.walk(tree):
            if isinstance(node, ast.stmt) and first <= node.lineno <= last and node.lineno not in seen:
                if any(first <= a.lineno <= last and a is not node and node in ast.walk(a) for a in body):
                    continue
                body.append(node)
                seen.add(node.lineno)
        body.sort(key=lambda n: n.lineno)
        # drop statements nested inside another extracted statement
        outer = []
        for n in body:
            if not any(n is not o and n in list(ast.walk(o)) for o in body):
                outer.append(n)
        body = outer
    mod = ast.Module(body=body, type_ignores=[])
    return compile(mod, path, "exec")


def _vae_a_model():
    import torch
    from vae_model import ConvVAE1D

    L, d, kw = VAE_CONFIGS["a"]
    g = np.load(os.path.join(HERE, "vae_a.npz"), allow_pickle=False)
    m = ConvVAE1D(L, d, g["mean"], g["std"], **kw)
    m.load_state_dict({k[3:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("sd/")})
    return m.eval(), g


def make_vaesimca():
    """VAESIMCA of VAE_SIMCA.py:215-382, executed alone on the vae_a network."""
    import torch
    from scipy import special

    ns = {"np": np, "torch": torch, "special": special}
    exec(_extract(os.path.join(REF, "VAE_SIMCA.py"), 0, 0, names={"VAESIMCA"}), ns)
    VAESIMCA = ns["VAESIMCA"]
    m, g = _vae_a_model()
    cal = [(torch.from_numpy(g["x_cal"]),)]   # one batch: bit-identical to mu_cal / zhat_cal
    test = [(torch.from_numpy(g["x_test"]),)]
    out = {}
    combos = []
    for ty in ("sim", "alt", "ci", "dd"):
        for t2 in ("perc", "Fdist", "chi2", "chi2pom"):
            for ql in ("perc", "jm", "chi2pom"):
                combos.append((ty, t2, ql))
    lim = {k: [] for k in ("T2_limit", "Q_limit", "D_limit", "T2dof", "Qdof", "T2scfact", "Qscfact")}
    preds, errs = [], []
    for ty, t2, ql in combos:
        vs = VAESIMCA(m, type=ty, t2lim=t2, qlim=ql, verbose=False)
        try:
            vs.fit_thresholds(cal, class_label=0)
            y_pred, T2, Q = vs.predict(test)
            info = vs._model[0]
            for k in lim:
                v = info[k]
                lim[k].append(np.nan if v is None else float(v))
            preds.append(np.asarray(y_pred, dtype=np.uint8))
            errs.append("")
            if "fit_T2" not in out:
                out["fit_T2"], out["fit_Q"] = np.asarray(info["T2"]), np.asarray(info["Q"])
                out["test_T2"], out["test_Q"] = np.asarray(T2), np.asarray(Q)
                out["latent_mean"], out["invcovT"] = np.asarray(info["latent_mean"]), np.asarray(info["invcovT"])
        except Exception as e:
            for k in lim:
                lim[k].append(np.nan)
            preds.append(np.zeros(len(g["x_test"]), np.uint8))
            errs.append(type(e).__name__)
    out["combos"] = np.array(["|".join(c) for c in combos])
    out["errors"] = np.array(errs)
    for k, v in lim.items():
        out[k] = np.array(v)
    out["pred"] = np.stack(preds)
    np.savez_compressed(os.path.join(HERE, "vaesimca.npz"), **out)
    print("vaesimca", len(combos), "combos,", sum(1 for e in errs if e), "raise")


class _Buffers:
    """Stand-in for the loaded network whose buffers the f-distance block reads."""

    def __init__(self, latent_mean):
        import torch

        self.latent_mean = torch.from_numpy(np.asarray(latent_mean, dtype=np.float32))


def make_final_vaesimca():
    """utils/final_vaesimca.py:428-436 (latent stats) and :511-533 (full-distance
    decision), extracted statement by statement and executed on vae_a latents
    and synthetic reconstruction errors."""
    import scipy as sp
    import scipy.stats  # noqa: F401

    g = np.load(os.path.join(HERE, "vae_a.npz"), allow_pickle=False)
    path = os.path.join(REF, "utils", "final_vaesimca.py")
    rng = np.random.default_rng(55)
    rec_cal = rng.gamma(4.0, 0.5, size=len(g["mu_cal"])).astype(np.float32)
    q_test = rng.gamma(4.0, 0.5, size=len(g["mu_test"])).astype(np.float32)
    q_test[60:] *= 3.0
    ns = {"np": np, "sp": sp, "mus_train_list": [g["mu_cal"][:150], g["mu_cal"][150:]],
          "rec_errors_list": [rec_cal[:150], rec_cal[150:]]}
    exec(_extract(path, 428, 436), ns)
    out = {"rec_cal": rec_cal, "q_test": q_test, "mu_train_mean": ns["mu_train_mean"], "cov_inv": ns["cov_inv"],
           "threshold": np.float64(ns["threshold"]), "q_threshold": np.float64(ns["q_threshold"])}
    ns2 = {"np": np, "sp": sp, "mus_test": g["mu_test"], "q_errors": q_test,
           "vae_best": _Buffers(ns["mu_train_mean"])}
    exec(_extract(path, 511, 533), ns2)
    for key in ("h", "h0", "sh", "Nh", "q0", "sq", "Nq", "f", "Nf", "fcrit"):
        out[key] = np.asarray(ns2[key])
    out["pred_class0"] = np.asarray(ns2["pred_class0"], dtype=np.uint8)
    np.savez_compressed(os.path.join(HERE, "final_vaesimca.npz"), **out)
    print("final_vaesimca fcrit", float(out["fcrit"]), "accept", int(out["pred_class0"].sum()))


def make_final_losses():
    """utils/final_vaesimca.py: the three losses (:198-224), the calibration /
    test reconstruction error Q in both branches (:417-425), and the state_dict
    of the script's own ConvVAE1D copy (:72-193, seeded), each taken from the
    script's syntax tree and executed alone."""
    import torch
    import torch.nn as nn
    import torch.nn.functional as F

    path = os.path.join(REF, "utils", "final_vaesimca.py")
    ns = {"torch": torch, "F": F, "nn": nn, "np": np}
    exec(_extract(path, 198, 224), ns)
    rng = np.random.default_rng(77)
    B, L, d = 48, 300, 8
    wl = np.linspace(0, 1, L)
    x = (1.0 + 0.5 * wl + 0.2 * rng.standard_normal((B, 1)) * np.sin(7 * wl) +
         0.02 * rng.standard_normal((B, L))).astype(np.float32)
    x_recon = (x + 0.08 * rng.standard_normal((B, L))).astype(np.float32)  # partly outside [min, max]
    mu = rng.standard_normal((B, d)).astype(np.float32)
    logvar = (0.3 * rng.standard_normal((B, d))).astype(np.float32)
    out = {"x": x, "x_recon": x_recon, "mu": mu, "logvar": logvar}
    t = [torch.from_numpy(a) for a in (x, x_recon, mu, logvar)]
    for name in ("cosine", "euclidean", "bce"):
        total, recon, kl = ns[f"beta_vae_{name}_loss"](*t, beta=0.7)
        out[f"{name}_total"] = np.float64(total.item())
        out[f"{name}_recon"] = np.float64(recon)
        out[f"{name}_kl"] = np.float64(kl)
    for loss_type in ("X_bce", "X_euclidean"):
        ns_q = {"torch": torch, "np": np, "x": t[0], "x_rec": t[1], "loss_type": loss_type}
        exec(_extract(path, 417, 425), ns_q)
        out[f"rec_err_{loss_type}"] = np.asarray(ns_q["rec_err"])
    # the script's ConvVAE1D copy: seeded init → state_dict (keys, order, values)
    ns_m = {"torch": torch, "nn": nn, "F": F, "np": np}
    exec(_extract(path, 0, 0, names={"ConvVAE1D"}), ns_m)
    torch.manual_seed(5)
    mean, std = x.mean(0), x.std(0) + 1e-3
    m = ns_m["ConvVAE1D"](L, d, mean, std, conv_blocks=2, n_filters=3, kernel_size=5, hidden_fc=16)
    sd = m.state_dict()
    out["sd_keys"] = np.array(list(sd.keys()))
    for k, v in sd.items():
        out["sd/" + k] = v.detach().numpy()
    out["model_cfg"] = np.array(json.dumps({"L": L, "d": d, "conv_blocks": 2, "n_filters": 3, "kernel_size": 5,
                                            "hidden_fc": 16}))
    np.savez_compressed(os.path.join(HERE, "final_losses.npz"), **out)
    print("final_losses", {k: float(v) for k, v in out.items() if np.ndim(v) == 0 and k.endswith(("_total", "_recon", "_kl"))})


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    extra = {"ns": make_northstar, "f64": make_f64, "score": make_score_pins, "vaesimca": make_vaesimca,
             "final": make_final_vaesimca, "final_losses": make_final_losses}
    if argv:
        for name in argv:
            extra[name]()
        return
    # A: one class, spectral gap at k, wavelength-correlated bands.
    # The last 100 rows carry the out-of-class band; fit on the first 1200.
    Xa_all = synth_spectra(1600, 96, 4, rank=12, seed=1234, outlier_frac=100 / 1600)
    Xa, Xa_t = Xa_all[:1200], Xa_all[1200:]
    ya = np.zeros(1200, dtype=np.int64)
    ya_t = np.concatenate([np.zeros(300, np.int64), np.ones(100, np.int64)])
    make_simca("a", Xa, ya, Xa_t, ya_t, 4, 0)

    # B: nuts-like plumbing stand-in (p=256, k=10).
    Xb_all = synth_spectra(1700, 256, 10, rank=24, seed=99, outlier_frac=100 / 1700)
    Xb, Xb_t = Xb_all[:1500], Xb_all[1500:]
    yb = np.zeros(1500, dtype=np.int64)
    yb_t = np.concatenate([np.zeros(100, np.int64), np.ones(100, np.int64)])
    make_simca("b", Xb, yb, Xb_t, yb_t, 10, 0)

    # M: three classes, per-class n_components, model_class=None.
    parts, labels = [], []
    for c in range(3):
        parts.append(synth_spectra(300, 64, 3, rank=8, seed=500 + c) + 0.5 * c)
        labels.append(np.full(300, c, dtype=np.int64))
    Xm = np.concatenate(parts)
    ym = np.concatenate(labels)
    perm = np.random.default_rng(5).permutation(len(ym))
    Xm, ym = Xm[perm], ym[perm]
    make_simca("multi", Xm[:750], ym[:750], Xm[750:], ym[750:], [2, 3, 4], None)

    # CV: target class 0 (500 rows) + 100 other-class rows.
    Xc_all = synth_spectra(600, 64, 4, rank=10, seed=77, outlier_frac=100 / 600)
    yc = np.concatenate([np.zeros(500, np.int64), np.ones(100, np.int64)])
    make_cv("a", Xc_all, yc, 5, 2, 6, {})
    make_cv("grid", Xc_all, yc, 4, 2, 4, {"type": ["alt", "sim"], "qlim": ["jm", "chi2box"]})

    make_qhf()
    make_vae()
    make_splits()
    for fn in extra.values():
        fn()


if __name__ == "__main__":
    main()
