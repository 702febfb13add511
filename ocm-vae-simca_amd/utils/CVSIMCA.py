"""Class-wise cross-validation for SIMCA — the drop-in for the reference's
utils/CVSIMCA.py (public names, signatures, record layout, printed summary,
error messages and return keys are the reference's contract; the bodies are
written here from that contract).

Contract (reference file:line):
* ``ClasswiseKFoldWithExternalVal(n_splits, cls_idx, cls_label, shuffle,
  random_state)`` (:39-80): KFold over the target-class rows only; the test
  set of every split is the held-out target fold followed by every
  non-target row.
* ``cross_validate_simca_grid(...)`` (:103-269): for every parameter combo
  and LV, class-wise CV; spec = mean of the per-fold specificities, sens =
  sensitivity of the pooled prediction vector (each row keeps the prediction
  of the LAST split that tested it), eff = √(sens·spec); best record by
  ``refit_metric`` (first maximum), refit on all rows; returns
  {results, best_params, best_LV, best_score, best_estimator[, by_combo]}.
* ``plot_cv`` (:274-331): the CV metric against LV for one parameter set.

Execution: when the estimator is this package's SIMCA under a
``ClasswiseKFoldWithExternalVal`` split, ``ocm.cv`` evaluates the whole grid
on the GPU in one Gram pass (fold Grams by downdating, one eigensolve per
fold, every LV a prefix of it).  Anything else (pipelines, other splitters,
foreign estimators) goes through ``_crossval_loop``: per setting, a clone is
fitted per split and scored with the estimator's own conformity metric.
"""
from __future__ import annotations

import numpy as np
from sklearn.base import clone
from sklearn.model_selection import BaseCrossValidator, KFold, ParameterGrid
from sklearn.pipeline import Pipeline

__all__ = ["ClasswiseKFoldWithExternalVal", "cross_validate_simca_grid", "plot_cv"]

# user-facing messages of the reference (behavioural output, kept verbatim)
_MSG_LABEL_NEEDS_Y = "Per usare cls_label serve y in split(X, y)."
_MSG_SCALAR_NEEDS_Y = "Hai passato uno scalare a cls_idx; serve y per ricavarne gli indici."
_MSG_EMPTY_TARGET = "cls_idx è vuoto: nessun campione della classe target trovato."
_MSG_TOO_MANY_SPLITS = "Troppi split ({k}) rispetto ai campioni della classe target ({n})."
_MSG_NO_SIMCA = "Non trovo un oggetto SIMCA nell'estimator."
_MSG_PIPE_NO_SIMCA = "Pipeline senza step SIMCA per determinare n_components."
_MSG_NO_RECORD = "Nessun record trovato con i parametri specificati."

_REFIT_KEYS = {"eff": "eff", "spec": "spec", "sens": "sens"}


def _is_simca(obj) -> bool:
    # the reference recognises a SIMCA step by duck typing on this method
    return hasattr(obj, "_metrics_simca_conformity")


class ClasswiseKFoldWithExternalVal(BaseCrossValidator):
    """KFold on the target class; every test set = held-out target fold +
    all other samples.  The target rows come from ``cls_idx`` (indices, or a
    scalar label) or from ``cls_label`` looked up in ``y``."""

    def __init__(self, n_splits=5, cls_idx=None, cls_label=None, shuffle=False, random_state=None):
        self.kf = KFold(n_splits=n_splits, shuffle=shuffle, random_state=random_state)
        self.cls_idx = None if cls_idx is None else np.asarray(cls_idx)
        self.cls_label = cls_label

    def get_n_splits(self, X=None, y=None, groups=None):
        return self.kf.get_n_splits()

    def _rows_of_label(self, y, label, missing_y_msg):
        if y is None:
            raise ValueError(missing_y_msg)
        return np.flatnonzero(np.asarray(y) == label)

    def target_indices(self, X, y=None):
        """Indices of the target-class rows, validated against n_splits."""
        given = self.cls_idx
        if given is None:
            target = None if self.cls_label is None else self._rows_of_label(y, self.cls_label, _MSG_LABEL_NEEDS_Y)
        elif np.ndim(given) == 0:  # a label passed where indices were expected
            target = self._rows_of_label(y, int(given), _MSG_SCALAR_NEEDS_Y)
        else:
            target = given
        if target is None or target.size == 0:
            raise ValueError(_MSG_EMPTY_TARGET)
        if target.size < self.kf.n_splits:
            raise ValueError(_MSG_TOO_MANY_SPLITS.format(k=self.kf.n_splits, n=target.size))
        return target

    def split(self, X, y=None, groups=None):
        target = self.target_indices(X, y)
        external = np.setdiff1d(np.arange(X.shape[0]), target)
        for fit_pos, held_pos in self.kf.split(target):
            yield target[fit_pos], np.concatenate([target[held_pos], external])


# --------------------------------------------------------------------------
# estimator introspection (Pipeline-aware)
# --------------------------------------------------------------------------

def _simca_steps(estimator):
    """(name, step) pairs of the SIMCA-like steps, in pipeline order."""
    if isinstance(estimator, Pipeline):
        return [(name, step) for name, step in estimator.named_steps.items() if _is_simca(step)]
    return []


def _get_simca(estimator):
    """The estimator itself if it is SIMCA-like, else the LAST SIMCA step of a Pipeline."""
    if _is_simca(estimator):
        return estimator
    steps = _simca_steps(estimator)
    if not steps:
        raise AttributeError(_MSG_NO_SIMCA)
    return steps[-1][1]


def _find_ncomp_param_name(estimator):
    """``set_params`` key of n_components: the FIRST SIMCA step of a Pipeline, else the estimator's own."""
    if not isinstance(estimator, Pipeline):
        return "n_components"
    steps = _simca_steps(estimator)
    if not steps:
        raise AttributeError(_MSG_PIPE_NO_SIMCA)
    return steps[0][0] + "__n_components"


# --------------------------------------------------------------------------
# the grid
# --------------------------------------------------------------------------

def _settings(param_grid, lv_values):
    """(combo, lv) in the reference's order: combos outer (ParameterGrid
    order), LV inner; lv is None when n_components lives in the grid."""
    for combo in ParameterGrid(param_grid):
        for lv in (lv_values if lv_values is not None else [None]):
            yield combo, lv


def _configured(template, combo, ncomp_key, lv):
    est = clone(template)
    est.set_params(**combo)
    if lv is not None:
        est.set_params(**{ncomp_key: lv})
    return est


def _fold_predictions(est, X_test, y_test):
    try:
        pred = est.predict(X_test)
    except TypeError:  # estimators whose predict needs the labels
        pred = est.predict(X_test, y_test)
    if hasattr(pred, "detach"):  # the drop-in returns device tensors for device inputs
        pred = pred.detach().cpu().numpy()
    return np.ravel(np.asarray(pred))


def _crossval_one(est, X, y, cv, class_index):
    """Class-wise CV of one configured estimator → (spec, sens, pooled predictions)."""
    pooled = np.zeros(X.shape[0], dtype=float)
    spec_per_fold = np.zeros(cv.get_n_splits(X, y), dtype=float)
    simca = None
    for f, (fit_rows, test_rows) in enumerate(list(cv.split(X, y))):
        model = clone(est)
        model.fit(X[fit_rows, :], y[fit_rows])
        pred = _fold_predictions(model, X[test_rows, :], y[test_rows])
        pooled[test_rows] = pred
        simca = _get_simca(model)
        ci = class_index if class_index is not None else getattr(simca, "model_class", 1)
        spec_per_fold[f] = simca._metrics_simca_conformity(y_true=y[test_rows], y_pred=pred,
                                                           class_index=ci)["specificity"]
    ci = class_index if class_index is not None else getattr(simca, "model_class", 1)
    sens = simca._metrics_simca_conformity(y_true=y, y_pred=pooled, class_index=ci)["sensitivity"]
    return float(np.mean(spec_per_fold)), float(sens), pooled


def _crossval_loop(template, X, y, cv, lv_values, param_grid, ncomp_key, class_index, store_predictions):
    """Generic path: refit per (setting, split) — any estimator / splitter."""
    records, by_combo = [], []
    for combo, lv in _settings(param_grid, lv_values):
        est = _configured(template, combo, ncomp_key, lv)
        spec, sens, pooled = _crossval_one(est, X, y, cv, class_index)
        record = {"params": combo.copy(), "LV": combo.get(ncomp_key) if lv is None else lv,
                  "spec": spec, "sens": sens, "eff": float(np.sqrt(sens * spec))}
        records.append(record)
        if store_predictions:
            by_combo.append({"params": combo.copy(), "LV": record["LV"], "prediction": pooled.copy()})
    return records, by_combo


def _fold_engine(template, X, y, cv, lv_values, param_grid, class_index, store_predictions):
    """GPU fold engine (ocm.cv); (None, None) when it does not cover the setup."""
    from ocm import cv as engine_cv

    return engine_cv.grid(template, X, y, cv, lv_values, param_grid, class_index, store_predictions)


# kept under the round-1 name: tests switch the engine off through it
_fast_grid = _fold_engine


def _summary_lines(records, refit_metric, best):
    def key_of(params):
        return ", ".join(f"{k}={v}" for k, v in sorted(params.items()))

    shown = None
    for r in sorted(records, key=lambda r: (key_of(r["params"]), r["LV"])):
        if key_of(r["params"]) != shown:
            shown = key_of(r["params"])
            yield "\nPARAMS: " + shown
        yield f"  LV={r['LV']:>2} | SPEC={r['spec']:.4f} | SENS={r['sens']:.4f} | EFF={r['eff']:.4f}"
    yield (f"\n[best @ {refit_metric}] LV={best['LV']} | score={best[_REFIT_KEYS[refit_metric]]:.4f} | "
           f"params={best['params']}")


def cross_validate_simca_grid(estimator, X, y, cv, LV_min=2, LV_max=10, param_grid=None, refit_metric="eff",
                              class_index=None, print_summary=True, store_predictions=False):
    """Grid × LV class-wise CV with refit (contract: utils/CVSIMCA.py:103-269)."""
    param_grid = {} if param_grid is None else param_grid
    template = clone(estimator)
    ncomp_key = _find_ncomp_param_name(template)
    lv_in_grid = any(name.endswith("n_components") for name in param_grid)
    lv_values = None if lv_in_grid else list(range(LV_min, LV_max + 1))

    records, by_combo = _fast_grid(template, X, y, cv, lv_values, param_grid, class_index, store_predictions)
    if records is None:
        records, by_combo = _crossval_loop(template, X, y, cv, lv_values, param_grid, ncomp_key, class_index,
                                           store_predictions)

    metric = _REFIT_KEYS[refit_metric]
    best = records[int(np.argmax([r[metric] for r in records]))]  # first maximum, NaN-aware like np.argmax
    if print_summary:
        for line in _summary_lines(records, refit_metric, best):
            print(line)

    refit = clone(estimator)
    refit.set_params(**best["params"])
    if not lv_in_grid:
        refit.set_params(**{_find_ncomp_param_name(refit): best["LV"]})
    refit.fit(X, y)

    result = {"results": records, "best_params": best["params"].copy(), "best_LV": best["LV"],
              "best_score": best[metric], "best_estimator": refit}
    if store_predictions:
        result["by_combo"] = by_combo
    return result


def plot_cv(res, metric="eff", params=None, show_best=True, title=None):
    """CV ``metric`` against LV for the records whose params include ``params``
    (default: the best params), with the best LV marked.  Host plotting glue
    (matplotlib object API); returns the Figure."""
    import matplotlib.pyplot as plt

    wanted = res.get("best_params") if params is None else params
    wanted = wanted or {}
    chosen = [r for r in res["results"] if all(r["params"].get(k, _Missing) == v for k, v in wanted.items())]
    if not chosen:
        raise ValueError(_MSG_NO_RECORD)
    chosen.sort(key=lambda r: r["LV"])
    lv = np.array([r["LV"] for r in chosen])
    val = np.array([r[metric] for r in chosen])
    fig, ax = plt.subplots(figsize=(8, 5))
    ax.plot(lv, val, marker="o", color="C0", label=f"Mean CV {metric.upper()}")
    if show_best and "best_LV" in res:
        ax.axvline(res["best_LV"], color="r", linestyle="--",
                   label=f"Best LV = {res['best_LV']} ({metric} = {res['best_score']:.3f})")
    ax.set_xlabel("Number of latent variables (LVs)")
    ax.set_ylabel(metric.upper())
    ax.set_title(title or f"Cross-validation {metric.upper()} vs LV")
    ax.grid(True, linestyle="--", alpha=0.5)
    ax.legend()
    plt.show()
    return fig


class _Missing:
    """Sentinel: a params key absent from a record never matches."""
