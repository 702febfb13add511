"""Drop-in class-wise cross-validation for SIMCA (utils/CVSIMCA.py:39-331).

``ClasswiseKFoldWithExternalVal`` and ``cross_validate_simca_grid`` keep the
reference's signatures, fold layout, aggregation (spec = mean over folds,
sens from the pooled predictions, eff = √(sens·spec)), refit and return
dict.  When the estimator is this package's SIMCA and the CV object is a
ClasswiseKFoldWithExternalVal, the grid runs on the fold engine
(``ocm.cv``): one Gram pass over the target-class rows produces every fold's
Gram (training Gram = total − fold, fp64 downdating), the LV sweep reuses
one eigensolve per fold (prefix sums of the scores), and the test rows are
scored in HBM by index — instead of K × #LV full refits.  Any other
estimator / splitter goes through the generic loop below.
"""
from __future__ import annotations

import numpy as np
from sklearn.base import clone
from sklearn.model_selection import BaseCrossValidator, KFold, ParameterGrid
from sklearn.pipeline import Pipeline

__all__ = ["ClasswiseKFoldWithExternalVal", "cross_validate_simca_grid", "plot_cv"]


class ClasswiseKFoldWithExternalVal(BaseCrossValidator):
    """KFold over the target class only; every split's test set = the held-out
    target fold + ALL other samples (utils/CVSIMCA.py:39-80)."""

    def __init__(self, n_splits=5, cls_idx=None, cls_label=None, shuffle=False, random_state=None):
        self.kf = KFold(n_splits=n_splits, shuffle=shuffle, random_state=random_state)
        self.cls_idx = None if cls_idx is None else np.asarray(cls_idx)
        self.cls_label = cls_label

    def get_n_splits(self, X=None, y=None, groups=None):
        return self.kf.get_n_splits()

    def target_indices(self, X, y=None):
        if y is None and self.cls_idx is None and self.cls_label is not None:
            raise ValueError("Per usare cls_label serve y in split(X, y).")
        cls_idx = self.cls_idx
        if cls_idx is None and self.cls_label is not None:
            cls_idx = np.flatnonzero(np.asarray(y) == self.cls_label)
        if cls_idx is not None and np.ndim(cls_idx) == 0:
            if y is None:
                raise ValueError("Hai passato uno scalare a cls_idx; serve y per ricavarne gli indici.")
            cls_idx = np.flatnonzero(np.asarray(y) == int(cls_idx))
        if cls_idx is None or cls_idx.size == 0:
            raise ValueError("cls_idx è vuoto: nessun campione della classe target trovato.")
        if cls_idx.size < self.kf.n_splits:
            raise ValueError(f"Troppi split ({self.kf.n_splits}) rispetto ai campioni della classe target "
                             f"({cls_idx.size}).")
        return cls_idx

    def split(self, X, y=None, groups=None):
        cls_idx = self.target_indices(X, y)
        others = np.setdiff1d(np.arange(X.shape[0]), cls_idx)
        for train_rel, test_rel in self.kf.split(cls_idx):
            yield cls_idx[train_rel], np.concatenate([cls_idx[test_rel], others])


def _get_simca(estimator):
    if hasattr(estimator, "_metrics_simca_conformity"):
        return estimator
    if isinstance(estimator, Pipeline):
        for _, step in reversed(list(estimator.named_steps.items())):
            if hasattr(step, "_metrics_simca_conformity"):
                return step
    raise AttributeError("Non trovo un oggetto SIMCA nell'estimator.")


def _find_ncomp_param_name(estimator):
    if isinstance(estimator, Pipeline):
        for name, step in estimator.named_steps.items():
            if hasattr(step, "_metrics_simca_conformity"):
                return f"{name}__n_components"
        raise AttributeError("Pipeline senza step SIMCA per determinare n_components.")
    return "n_components"


def cross_validate_simca_grid(estimator, X, y, cv, LV_min=2, LV_max=10, param_grid=None, refit_metric="eff",
                              class_index=None, print_summary=True, store_predictions=False):
    """utils/CVSIMCA.py:103-269 (same records, best selection, refit and output keys)."""
    if param_grid is None:
        param_grid = {}
    base_est = clone(estimator)
    ncomp_key = _find_ncomp_param_name(base_est)
    grid_includes_ncomp = any(k.endswith("n_components") for k in param_grid.keys())
    lv_values = None if grid_includes_ncomp else list(range(LV_min, LV_max + 1))

    records, by_combo = _fast_grid(base_est, X, y, cv, lv_values, param_grid, class_index, store_predictions)
    if records is None:
        records, by_combo = _generic_grid(base_est, X, y, cv, lv_values, param_grid, ncomp_key, class_index,
                                          store_predictions, grid_includes_ncomp)

    metric_key = {"eff": "eff", "spec": "spec", "sens": "sens"}[refit_metric]
    best_idx = int(np.argmax([r[metric_key] for r in records]))
    best_score = records[best_idx][metric_key]
    best_params = records[best_idx]["params"].copy()
    best_LV = records[best_idx]["LV"]

    if print_summary:
        def params_to_str(p):
            return ", ".join(f"{k}={v}" for k, v in sorted(p.items()))

        rows = sorted(records, key=lambda r: (params_to_str(r["params"]), r["LV"]))
        curr = None
        for r in rows:
            pstr = params_to_str(r["params"])
            if pstr != curr:
                print("\nPARAMS:", pstr)
                curr = pstr
            print(f"  LV={r['LV']:>2} | SPEC={r['spec']:.4f} | SENS={r['sens']:.4f} | EFF={r['eff']:.4f}")
        print(f"\n[best @ {refit_metric}] LV={best_LV} | score={best_score:.4f} | params={best_params}")

    best_estimator = clone(estimator)
    best_estimator.set_params(**best_params)
    if not grid_includes_ncomp:
        best_estimator.set_params(**{_find_ncomp_param_name(best_estimator): best_LV})
    best_estimator.fit(X, y)

    out = {"results": records, "best_params": best_params, "best_LV": best_LV, "best_score": best_score,
           "best_estimator": best_estimator}
    if store_predictions:
        out["by_combo"] = by_combo
    return out


def _generic_grid(base_est, X, y, cv, lv_values, param_grid, ncomp_key, class_index, store_predictions,
                  grid_includes_ncomp):
    """The reference's clone/fit/predict loop, for estimators/splitters the fold engine does not cover."""
    records, by_combo = [], []
    for combo in ParameterGrid(param_grid):
        for lv in ([None] if grid_includes_ncomp else lv_values):
            est_lv = clone(base_est)
            est_lv.set_params(**combo)
            if not grid_includes_ncomp:
                est_lv.set_params(**{ncomp_key: lv})
            n_samples = X.shape[0]
            n_folds = cv.get_n_splits(X, y)
            pred_vec = np.zeros(n_samples, dtype=float)
            step_spec = np.zeros(n_folds, dtype=float)
            last = None
            for i, (train_idx, test_idx) in enumerate(list(cv.split(X, y)), start=1):
                est_fold = clone(est_lv)
                est_fold.fit(X[train_idx, :], y[train_idx])
                try:
                    y_pred = est_fold.predict(X[test_idx, :])
                except TypeError:
                    y_pred = est_fold.predict(X[test_idx, :], y[test_idx])
                y_pred = np.ravel(np.asarray(y_pred))
                pred_vec[test_idx] = y_pred
                simca = _get_simca(est_fold)
                ci = class_index if class_index is not None else getattr(simca, "model_class", 1)
                m = simca._metrics_simca_conformity(y_true=y[test_idx], y_pred=y_pred, class_index=ci)
                step_spec[i - 1] = m["specificity"]
                last = simca
            spec = float(np.mean(step_spec))
            ci = class_index if class_index is not None else getattr(last, "model_class", 1)
            sens = float(last._metrics_simca_conformity(y_true=y, y_pred=pred_vec, class_index=ci)["sensitivity"])
            rec = {"params": combo.copy(), "LV": (combo.get(ncomp_key) if grid_includes_ncomp else lv),
                   "spec": spec, "sens": sens, "eff": float(np.sqrt(sens * spec))}
            records.append(rec)
            if store_predictions:
                by_combo.append({"params": combo.copy(), "LV": rec["LV"], "prediction": pred_vec.copy()})
    return records, by_combo


def _fast_grid(base_est, X, y, cv, lv_values, param_grid, class_index, store_predictions):
    """Fold engine path (ocm.cv); returns (None, None) when not applicable."""
    from . import SIMCA as _SIMCA_mod  # noqa: F401

    try:
        from ocm import cv as fold_engine
    except Exception:
        return None, None
    return fold_engine.grid(base_est, X, y, cv, lv_values, param_grid, class_index, store_predictions)


def plot_cv(res, metric="eff", params=None, show_best=True, title=None):
    """CV metric against LV (utils/CVSIMCA.py:274-331); host plotting glue."""
    import matplotlib.pyplot as plt

    results = res["results"]
    best_params = res.get("best_params", None)
    if params is None and best_params is not None:
        params = best_params

    def match_params(r, p):
        return all(k in r["params"] and r["params"][k] == v for k, v in p.items())

    selected = [r for r in results if match_params(r, params)]
    if not selected:
        raise ValueError("Nessun record trovato con i parametri specificati.")
    selected = sorted(selected, key=lambda r: r["LV"])
    LV = np.array([r["LV"] for r in selected])
    values = np.array([r[metric] for r in selected])
    plt.figure(figsize=(8, 5))
    plt.plot(LV, values, marker="o", color="C0", label=f"Mean CV {metric.upper()}")
    if show_best and "best_LV" in res:
        plt.axvline(res["best_LV"], color="r", linestyle="--",
                    label=f"Best LV = {res['best_LV']} ({metric} = {res['best_score']:.3f})")
    plt.xlabel("Number of latent variables (LVs)")
    plt.ylabel(metric.upper())
    plt.title(title or f"Cross-validation {metric.upper()} vs LV")
    plt.grid(True, linestyle="--", alpha=0.5)
    plt.legend()
    plt.show()
