"""CPU oracle for the SIMCA hot path — TEST INFRASTRUCTURE ONLY.

This module is a plain NumPy/SciPy restatement of the reference's SIMCA
algorithm (TEAM-AIOLY/OCM-VAE-SIMCA ``utils/SIMCA.py``) and of the pieces of
scikit-learn 1.7.2 it calls (``sklearn/decomposition/_pca.py`` ``_fit_full``,
``sklearn/utils/extmath.py`` ``svd_flip`` / ``_randomized_svd``).  It exists
only to check the HIP engine:

* ``tests/`` compare the HIP path against it on the same seeded inputs;
* ``__graft_entry__.smoke()`` checks one small HIP invocation against it;
* ``bench.py``'s ``cpu_baseline`` leg times it ("port") on the host cores.

Nothing under ``ocm-vae-simca_amd/`` may import it: the product path runs on
the GPU through ``libocm.so`` or fails loudly.

Pinning: ``tests/golden/*.npz`` hold outputs of the reference itself
(imported from /root/reference in the build container by
``tests/golden/make_golden.py``); ``tests/test_oracle_golden.py`` checks this
restatement against every vector there.

Precision: the oracle works in float64 internally ("exact" arithmetic for the
sizes tests use) and casts its outputs to the dtypes the reference produces
for float32 input (``Q`` float32, ``T2`` float64, ``T`` float32).  The
reference's own float32 SVD is what bounds agreement with the goldens
(SURVEY.md §8c).  ``precision='reference'`` instead runs the float32 LAPACK
path the reference runs; bench.py times that mode as the CPU baseline.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np
import scipy.linalg
from scipy import stats
from scipy import special
from scipy.special import erfinv

# ---------------------------------------------------------------------------
# PCA pieces (sklearn 1.7.2 restated)
# ---------------------------------------------------------------------------


def svd_flip_rows(Vt: np.ndarray, U: np.ndarray | None = None):
    """Sign convention of sklearn ``svd_flip(u_based_decision=False)``
    (sklearn/utils/extmath.py:895-953): every row of Vt gets its largest
    |entry| positive; U's columns flip with it."""
    idx = np.argmax(np.abs(Vt), axis=1)
    signs = np.sign(Vt[np.arange(Vt.shape[0]), idx])
    signs[signs == 0] = 1.0
    Vt = Vt * signs[:, None]
    if U is not None:
        U = U * signs[None, :]
    return Vt, U


def pca_full(X: np.ndarray, precision: str = "exact", ncomp: int | None = None):
    """Full PCA as ``PCA(n_components=None, svd_solver='full').fit_transform``
    (utils/SIMCA.py:64-65 -> sklearn/decomposition/_pca.py:544-702).

    Returns mean (p,), explained_variance (min(n,p),), components Vt, scores
    U*S.  ``precision='exact'`` does the SVD in float64; ``'reference'`` in
    the input dtype like sklearn (float32 gesdd for float32 X); ``'gram'`` is
    the same float64 result through the covariance (Xcᵀ Xc, ``eigh``) for the
    large parity cases (100k × 2048), with scores for the leading ``ncomp``
    components only.
    """
    n = X.shape[0]
    if precision == "gram":
        Xc = np.asarray(X, dtype=np.float64)
        mean = Xc.mean(axis=0)
        Xc = Xc - mean
        w, V = np.linalg.eigh(Xc.T @ Xc)
        order = np.argsort(w)[::-1][: min(n, X.shape[1])]
        Vt, _ = svd_flip_rows(V[:, order].T)
        ev = np.maximum(w[order], 0.0) / (n - 1)
        kk = Vt.shape[0] if ncomp is None else ncomp
        return mean, ev, Vt, Xc @ Vt[:kk].T
    work = np.float64 if precision == "exact" else X.dtype
    Xw = np.asarray(X, dtype=work)
    mean = Xw.mean(axis=0)
    Xc = Xw - mean
    U, S, Vt = scipy.linalg.svd(Xc, full_matrices=False, check_finite=False)
    Vt, U = svd_flip_rows(Vt, U)
    ev = (S.astype(np.float64) ** 2) / (n - 1)
    scores = U * S
    return mean, ev, Vt, scores


def covariance_chunked(X: np.ndarray, chunk: int = 32768):
    """fp64 mean and covariance (ddof 1) of a large float32 X without an fp64
    copy of it: Σ over row chunks of the shifted Gram YᵀY (one host dsyrk per
    chunk, y = x − s with s the mean of the first chunk), then
    C = (G − n·d·dᵀ)/(n − 1), μ = s + d — the covariance whose eigenpairs the
    reference's full SVD returns (utils/SIMCA.py:64-66 → sklearn/decomposition/
    _pca.py:569-584, explained_variance_ = S²/(n − 1)).  For the headline-size
    (1M × 2048) parity test."""
    n, p = X.shape
    s = np.asarray(X[: min(n, chunk)], dtype=np.float64).mean(axis=0)
    G = np.zeros((p, p))
    cs = np.zeros(p)
    for a in range(0, n, chunk):
        Y = np.asarray(X[a:a + chunk], dtype=np.float64) - s
        G += Y.T @ Y
        cs += Y.sum(axis=0)
    d = cs / n
    return s + d, (G - n * np.outer(d, d)) / (n - 1)


def eig_desc(C: np.ndarray):
    """Eigenvalues (descending) and loadings rows with the svd_flip sign."""
    w, V = np.linalg.eigh(C)
    order = np.argsort(w)[::-1]
    Vt, _ = svd_flip_rows(V[:, order].T)
    return w[order], Vt


def randomized_pca(X: np.ndarray, k: int, rng: np.random.RandomState,
                   n_oversamples: int = 10, n_iter: int | str = "auto"):
    """Restatement of the solver ``PCA(k).fit`` picks for p > 1000
    (utils/SIMCA.py:75 -> sklearn/decomposition/_pca.py:524-536,704-796 ->
    sklearn/utils/extmath.py:_randomized_svd / randomized_range_finder):
    Gaussian test matrix, ``n_iter`` LU-normalised power iterations, QR, a
    small SVD and ``svd_flip(u_based_decision=False)``.  Used only by the
    CPU-baseline timing (it is what the reference spends 21% of fit on)."""
    Xw = np.asarray(X)
    mean = Xw.mean(axis=0)
    Xc = Xw - mean
    n, p = Xc.shape
    size = k + n_oversamples
    if n_iter == "auto":
        n_iter = 7 if k < 0.1 * min(n, p) else 4
    Q = rng.normal(size=(p, size)).astype(Xc.dtype, copy=False)
    for _ in range(n_iter):
        Q, _ = scipy.linalg.lu(Xc @ Q, permute_l=True)
        Q, _ = scipy.linalg.lu(Xc.T @ Q, permute_l=True)
    Q, _ = scipy.linalg.qr(Xc @ Q, mode="economic")
    B = Q.T @ Xc
    _, S, Vt = scipy.linalg.svd(B, full_matrices=False)
    Vt, _ = svd_flip_rows(Vt)
    return mean, Vt[:k], (S[:k].astype(np.float64) ** 2) / (n - 1)


# ---------------------------------------------------------------------------
# Limits (utils/SIMCA.py:156-236)
# ---------------------------------------------------------------------------


@dataclass
class DDState:
    """The reference keeps the chi2pom dof/scale factors on ``self`` and
    overwrites them per class (utils/SIMCA.py:179-180, 215-216); predict uses
    the last class's values for every class (:142-143)."""
    t2dof: float | None = None
    t2scfact: float | None = None
    qdof: float | None = None
    qscfact: float | None = None


def t2_limit(T2: np.ndarray, k: int, t2lim: str, t2cl: float, st: DDState):
    """utils/SIMCA.py:156-182."""
    n = len(T2)
    if t2lim == "perc":
        return float(np.percentile(T2, t2cl * 100))
    if t2lim == "Fdistrig":
        F = stats.f.ppf(t2cl, k, n - k)
        return (k / n) * (n ** 2 - 1) / (n - k) * F
    if t2lim == "Fdist":
        F = stats.f.ppf(t2cl, k, n - k)
        return k * (n - 1) / (n - k) * F
    if t2lim == "chi2":
        return stats.chi2.ppf(t2cl, k)
    if t2lim == "chi2pom":
        h0 = float(np.mean(T2))
        v = float(np.var(T2, ddof=1)) if n > 1 else 0.0
        Nh = max(int(np.round(2 * h0 * h0 / v)) if v > 0 else 1, 1)
        st.t2dof, st.t2scfact = Nh, h0
        return h0 * stats.chi2.ppf(t2cl, Nh) / Nh
    raise UnboundLocalError(f"unknown t2lim {t2lim!r}")


def tail_thetas(ev: np.ndarray, k: int):
    """θ_m = Σ_{i>k} λ_i^m over the discarded eigenvalues (utils/SIMCA.py:189-191)."""
    tail = np.asarray(ev[k:], dtype=np.float64)
    return float(tail.sum()), float((tail ** 2).sum()), float((tail ** 3).sum())


def q_limit(Q: np.ndarray, thetas, qlim: str, qcl: float, st: DDState):
    """utils/SIMCA.py:184-217.  ``thetas`` = (θ1, θ2, θ3) of the tail."""
    th1, th2, th3 = thetas
    if qlim == "perc":
        return float(np.percentile(Q, qcl * 100))
    if qlim == "jm":
        if th1 == 0:
            raise UnboundLocalError("jm Q limit: theta1 == 0 leaves h0 unbound (utils/SIMCA.py:192-200)")
        h0 = max(1 - (2 * th1 * th3) / (3 * th2 ** 2), 0.001)
        ca = math.sqrt(2) * erfinv(2 * qcl - 1)
        h1 = ca * math.sqrt(2 * th2 * h0 ** 2) / th1
        h2 = th2 * h0 * (h0 - 1) / th1 ** 2
        return th1 * (h1 + 1 + h2) ** (1 / h0)
    if qlim == "chi2box":
        g = th2 / th1
        Ng = th1 ** 2 / th2
        return g * stats.chi2.ppf(qcl, Ng)
    if qlim == "chi2pom":
        Qd = np.asarray(Q, dtype=np.float64)
        v0 = float(np.mean(Q))
        Nv = max(round(2 * v0 * v0 / float(np.var(Qd, ddof=1))), 1)
        st.qdof, st.qscfact = Nv, v0
        return v0 * stats.chi2.ppf(qcl, Nv) / Nv
    raise UnboundLocalError(f"unknown qlim {qlim!r}")


def critic_distance(kind: str, T2lim, Qlim, thetas, k: int, dcl: float, st: DDState):
    """utils/SIMCA.py:219-236."""
    if kind == "sim":
        return 1
    if kind == "alt":
        return math.sqrt(2)
    if kind == "ci":
        th1, th2, _ = thetas
        tr1 = k / T2lim + th1 / Qlim
        tr2 = k / T2lim ** 2 + th2 / Qlim ** 2
        return (tr2 / tr1) * stats.chi2.ppf(dcl, tr1 ** 2 / tr2)
    if kind == "dd":
        return stats.chi2.ppf(dcl, st.t2dof + st.qdof)
    raise UnboundLocalError(f"unknown type {kind!r}")


# ---------------------------------------------------------------------------
# Scores
# ---------------------------------------------------------------------------


def project_scores(X: np.ndarray, P: np.ndarray, mean: np.ndarray, invcovT: np.ndarray):
    """T = (X-μ)Pᵀ, X̂ = T P + μ, Q = Σ(X-X̂)², T² = tᵀ·invcovT·t
    (utils/SIMCA.py:65-71 fit; 104-107 transform; 127-130 predict), done in
    float64; returned as the reference's dtypes for float32 X."""
    Xd = np.asarray(X, dtype=np.float64)
    Pd = np.asarray(P, dtype=np.float64)
    D = Xd - np.asarray(mean, dtype=np.float64)
    T = D @ Pd.T
    R = D - T @ Pd
    Q = np.einsum("ij,ij->i", R, R)
    T2 = np.einsum("ij,jk,ik->i", T, np.asarray(invcovT, dtype=np.float64), T)
    out_dt = np.float32 if X.dtype == np.float32 else np.float64
    return T.astype(out_dt), T2, Q.astype(out_dt)


def reduce_distances(kind: str, T2, Q, T2lim, Qlim, st: DDState):
    """T2red/Qred and dred by type (utils/SIMCA.py:76-81, 109-114, 131-144)."""
    T2 = np.asarray(T2, dtype=np.float64)
    Q = np.asarray(Q)
    if kind == "dd":
        t = st.t2dof * T2 / st.t2scfact
        q = st.qdof * Q / st.qscfact
        return t, q, t + q
    t = T2 / T2lim
    q = Q / Qlim
    if kind == "sim":
        d = np.maximum(t, q)
    elif kind == "alt":
        d = np.sqrt(t ** 2 + q ** 2)
    elif kind == "ci":
        d = t + q
    else:
        raise UnboundLocalError(f"unknown type {kind!r}")
    return t, q, d


# ---------------------------------------------------------------------------
# SIMCA estimator restated (utils/SIMCA.py:12-278)
# ---------------------------------------------------------------------------


@dataclass
class SimcaConfig:
    type: str = "alt"
    t2lim: str = "Fdist"
    t2cl: float = 0.95
    qlim: str = "jm"
    qcl: float = 0.95
    dcl: float = 0.95


def fit_one_class(X: np.ndarray, k: int, cfg: SimcaConfig, st: DDState,
                  precision: str = "exact", predict_loadings: str = "full",
                  rng: np.random.RandomState | None = None):
    """utils/SIMCA.py:62-99.  ``predict_loadings='full'`` uses the full-SVD
    loadings for predict/transform (the subspace the reference's second
    ``PCA(k)`` estimates, SURVEY.md §8c caveat 1); ``'randomized'`` reruns the
    randomized estimate like the reference (CPU-baseline timing)."""
    mean, ev, Vt, scores = pca_full(X, precision, ncomp=k)
    T = scores[:, :k]
    P = Vt[:k]
    if precision in ("exact", "gram"):
        T_, T2, Q = project_scores(X, P, mean, np.eye(k))
        Tf = np.asarray(T, dtype=np.float64)
        invcovT = np.linalg.pinv(np.atleast_2d(np.cov(Tf, rowvar=False)))
        T2 = np.einsum("ij,jk,ik->i", Tf, invcovT, Tf)
    else:
        Xhat = T @ P + mean
        Q = np.sum((X - Xhat) ** 2, axis=1)
        invcovT = np.linalg.pinv(np.atleast_2d(np.cov(T, rowvar=False)))
        T2 = np.einsum("ij,jk,ik->i", T, invcovT, T)
    thetas = tail_thetas(ev, k)
    T2lim = t2_limit(T2, k, cfg.t2lim, cfg.t2cl, st)
    Qlim = q_limit(Q, thetas, cfg.qlim, cfg.qcl, st)
    Dlim = critic_distance(cfg.type, T2lim, Qlim, thetas, k, cfg.dcl, st)
    if predict_loadings == "randomized":
        mean_p, P_p, _ = randomized_pca(X, k, rng or np.random.RandomState(0))
    else:
        mean_p, P_p = mean, P
    T2red, Qred, _ = reduce_distances(cfg.type, T2, Q, T2lim, Qlim, st)
    Tout = np.asarray(T, dtype=np.float32 if X.dtype == np.float32 else np.float64)
    return {
        "n_components": k,
        "xmean": np.asarray(mean),
        "invcovT": invcovT,
        "eigs_all": ev,
        "T": Tout,
        "P": P,
        "T2": T2,
        "Q": Q,
        "T2red": T2red,
        "Qred": Qred,
        "T2_limit": T2lim,
        "Q_limit": Qlim,
        "D_limit": Dlim,
        "n_samples": X.shape[0],
        "thetas": thetas,
        "P_pred": P_p,
        "mean_pred": mean_p,
    }


class OracleSIMCA:
    """Restatement of ``utils.SIMCA.SIMCA`` with the same fit/predict/
    transform/score semantics (list mutation of n_components/model_class,
    'dd' forcing chi2pom, last-class dd state)."""

    def __init__(self, n_components=2, model_class=None, type="alt", t2lim="Fdist", t2cl=0.95,
                 qlim="jm", qcl=0.95, dcl=0.95, precision="exact", predict_loadings="full"):
        self.n_components = n_components
        self.model_class = model_class
        self.cfg = SimcaConfig(type, t2lim, t2cl, qlim, qcl, dcl)
        self.precision = precision
        self.predict_loadings = predict_loadings
        self.st = DDState()
        self.metrics = {}

    def fit(self, X, classes, rng=None):
        """utils/SIMCA.py:27-59."""
        if self.model_class is None:
            self.model_class = np.unique(classes)
        elif isinstance(self.model_class, (int, np.integer)):
            self.model_class = [self.model_class]
        if not isinstance(self.n_components, list):
            self.n_components = [self.n_components]
        if len(self.n_components) == 1:
            self.n_components = [self.n_components[0]] * len(self.model_class)
        elif len(self.n_components) != len(self.model_class):
            raise ValueError("n_components length must match number of classes")
        if self.cfg.type == "dd":
            self.cfg.t2lim = "chi2pom"
            self.cfg.qlim = "chi2pom"
        self._model = {}
        for i, cls in enumerate(self.model_class):
            Xc = X[classes == cls]
            self._model[cls] = fit_one_class(Xc, self.n_components[i], self.cfg, self.st,
                                             self.precision, self.predict_loadings, rng)
        self.n_features_in_ = X.shape[1]
        return self

    def _scores(self, X, m):
        k = m["n_components"]
        return project_scores(X, m["P_pred"], m["mean_pred"], m["invcovT"][:k, :k])

    def transform(self, X):
        """utils/SIMCA.py:101-117 — returns the LAST class's (T2, T2red, Q, Qred)."""
        out = None
        for cls in self.model_class:
            m = self._model[cls]
            _, T2, Q = self._scores(X, m)
            t, q, _ = reduce_distances(self.cfg.type, T2, Q, m["T2_limit"], m["Q_limit"], self.st)
            out = (T2, t, Q, q)
        return out

    def predict(self, X, y_true=None):
        """utils/SIMCA.py:120-154 — (m, C) float64 of 0/1."""
        pred = np.zeros((X.shape[0], len(self.model_class)))
        for i, cls in enumerate(self.model_class):
            m = self._model[cls]
            _, T2, Q = self._scores(X, m)
            _, _, d = reduce_distances(self.cfg.type, T2, Q, m["T2_limit"], m["Q_limit"], self.st)
            pred[:, i] = d < m["D_limit"]
            if y_true is not None:
                self.metrics[cls] = metrics_conformity(y_true, pred[:, i], cls)
        return pred

    def dred(self, X, cls):
        m = self._model[cls]
        _, T2, Q = self._scores(X, m)
        return reduce_distances(self.cfg.type, T2, Q, m["T2_limit"], m["Q_limit"], self.st)[2]


def metrics_conformity(y_true, y_pred, class_index):
    """utils/SIMCA.py:238-266 (NaN where a denominator is zero)."""
    true_class = (np.asarray(y_true) == class_index).astype(int)
    y_pred = np.asarray(y_pred)
    TP = int(np.sum((y_pred == 1) & (true_class == 1)))
    TN = int(np.sum((y_pred == 0) & (true_class == 0)))
    FP = int(np.sum((y_pred == 1) & (true_class == 0)))
    FN = int(np.sum((y_pred == 0) & (true_class == 1)))
    with np.errstate(divide="ignore", invalid="ignore"):
        sens = np.float64(TP) / np.float64(TP + FN) * 100
        spec = np.float64(TN) / np.float64(TN + FP) * 100
        acc = np.float64(TP + TN) / np.float64(TP + TN + FP + FN) * 100
        eff = np.sqrt(sens * spec)
    return {"sensitivity": sens, "specificity": spec, "accuracy": acc, "efficiency": eff,
            "TP": TP, "TN": TN, "FP": FP, "FN": FN}


# ---------------------------------------------------------------------------
# Cross-validation restated (utils/CVSIMCA.py:39-269)
# ---------------------------------------------------------------------------


def classwise_kfold(n_total: int, cls_idx: np.ndarray, n_splits: int):
    """ClasswiseKFoldWithExternalVal.split with shuffle=False
    (utils/CVSIMCA.py:54-80 -> sklearn KFold): contiguous folds over the
    target-class indices, first n % K folds one longer; test = fold ∪ every
    non-target row (sorted, via setdiff1d)."""
    cls_idx = np.asarray(cls_idx)
    m = cls_idx.size
    sizes = np.full(n_splits, m // n_splits, dtype=int)
    sizes[: m % n_splits] += 1
    others = np.setdiff1d(np.arange(n_total), cls_idx)
    start = 0
    for s in sizes:
        test_rel = np.arange(start, start + s)
        train_rel = np.concatenate([np.arange(0, start), np.arange(start + s, m)])
        yield cls_idx[train_rel], np.concatenate([cls_idx[test_rel], others])
        start += s


def cross_validate_simca_grid(X, y, cls_label, n_splits, LV_min=2, LV_max=10, cfg_grid=None,
                              refit_metric="eff", class_index=None, simca_kwargs=None):
    """Restatement of cross_validate_simca_grid for a bare SIMCA estimator and
    ClasswiseKFoldWithExternalVal(cls_label=...) (utils/CVSIMCA.py:103-269).
    ``cfg_grid`` is a list of param dicts (ParameterGrid order)."""
    simca_kwargs = dict(simca_kwargs or {})
    cfg_grid = cfg_grid or [{}]
    grid_has_nc = any(k.endswith("n_components") for c in cfg_grid for k in c)
    cls_idx = np.flatnonzero(y == cls_label)
    splits = list(classwise_kfold(X.shape[0], cls_idx, n_splits))
    records = []
    for combo in cfg_grid:
        lvs = [None] if grid_has_nc else list(range(LV_min, LV_max + 1))
        for lv in lvs:
            kw = dict(simca_kwargs)
            kw.update(combo)
            if lv is not None:
                kw["n_components"] = lv
            pred_vec = np.zeros(X.shape[0])
            margin = np.full(X.shape[0], np.nan)  # |dred − D_lim| / D_lim of the fold that set pred_vec
            specs, senses = [], []
            last_mc = None
            for tr, te in splits:
                est = OracleSIMCA(**kw)
                est.fit(X[tr], y[tr])
                yp = np.ravel(est.predict(X[te]))
                pred_vec[te] = yp
                mc = np.atleast_1d(est.model_class)
                if mc.size == 1:
                    dlim = est._model[mc[0]]["D_limit"]
                    margin[te] = np.abs(est.dred(X[te], mc[0]) - dlim) / abs(dlim)
                ci = class_index if class_index is not None else est.model_class
                m = metrics_conformity(y[te], yp, _ci_scalar(ci))
                specs.append(m["specificity"])
                senses.append(m["sensitivity"])
                last_mc = est.model_class
            spec = float(np.mean(specs))
            ci = class_index if class_index is not None else last_mc
            sens = float(metrics_conformity(y, pred_vec, _ci_scalar(ci))["sensitivity"])
            records.append({"params": dict(combo), "LV": combo.get("n_components") if grid_has_nc else lv,
                            "spec": spec, "sens": sens, "eff": float(np.sqrt(sens * spec)),
                            "prediction": pred_vec,  # pooled fold predictions (store_predictions)
                            "margin": margin})  # not in the reference: the decision band of each pooled row
    key = {"eff": "eff", "spec": "spec", "sens": "sens"}[refit_metric]
    best = int(np.argmax([r[key] for r in records]))
    return {"results": records, "best_LV": records[best]["LV"], "best_score": records[best][key],
            "best_params": records[best]["params"]}


def _ci_scalar(ci):
    arr = np.atleast_1d(np.asarray(ci))
    return arr[0] if arr.size == 1 else arr


# ---------------------------------------------------------------------------
# VAE latent statistics (vae_model.py:162-182; utils/final_vaesimca.py:428-442,510-533)
# ---------------------------------------------------------------------------


def compute_q_h_f(x: np.ndarray, x_rec: np.ndarray, z: np.ndarray):
    """vae_model.py:162-182 in float64: q = Σ(x-x̂)², χ² moment-matched dof
    (unbiased std), leverage h = Σ U² of the thin SVD of the column-
    standardised z, f = h/h0·Nh + q/q0·Nq and the three χ²₀.₉₅ criticals."""
    x = np.asarray(x, np.float64)
    xr = np.asarray(x_rec, np.float64)
    z = np.asarray(z, np.float64)
    q = np.sum((x - xr) ** 2, axis=1)
    q0, sq = q.mean(), q.std(ddof=1)
    Nq = 2 * (q0 / sq) ** 2
    zs = (z - z.mean(axis=0)) / (z.std(axis=0, ddof=1) + 1e-12)
    U, _, _ = np.linalg.svd(zs, full_matrices=False)
    h = np.sum(U ** 2, axis=1)
    h0, sh = h.mean(), h.std(ddof=1)
    Nh = 2 * (h0 / sh) ** 2
    f = h / h0 * Nh + q / q0 * Nq
    return q, h, f, stats.chi2.ppf(0.95, Nq), stats.chi2.ppf(0.95, Nh), stats.chi2.ppf(0.95, Nh + Nq)


def latent_stats(mus: np.ndarray, q_cal: np.ndarray, ridge: float = 1e-6):
    """utils/final_vaesimca.py:428-442: latent mean, inverse of cov+ridge·I,
    95th-percentile Mahalanobis threshold and 95th-percentile Q threshold."""
    mus = np.asarray(mus, np.float64)
    mu = mus.mean(axis=0)
    cov = np.cov(mus, rowvar=False) + np.eye(mus.shape[1]) * ridge
    try:
        inv = np.linalg.inv(cov)
    except np.linalg.LinAlgError:
        inv = np.linalg.pinv(cov)
    d = mus - mu
    t2 = np.einsum("ij,jk,ik->i", d, inv, d)
    return mu, inv, float(np.percentile(t2, 95)), float(np.percentile(np.asarray(q_cal), 95))


def full_distance_decision(mus_test: np.ndarray, latent_mean: np.ndarray, q: np.ndarray, alpha=0.05):
    """utils/final_vaesimca.py:510-533: Euclidean h about the stored latent
    mean, test-set moments (ddof 0), f = h/h0·Nh + q/q0·Nq ≤ χ²₁₋α(Nh+Nq)."""
    h = np.sum((np.asarray(mus_test, np.float64) - latent_mean) ** 2, axis=1)
    q = np.asarray(q, np.float64)
    h0, sh = h.mean(), h.std()
    q0, sq = q.mean(), q.std()
    Nh = 2 * (h0 / sh) ** 2
    Nq = 2 * (q0 / sq) ** 2
    f = h / h0 * Nh + q / q0 * Nq
    fcrit = stats.chi2.ppf(1 - alpha, Nh + Nq)
    return f <= fcrit, f, fcrit


def vaesimca_fit(Z: np.ndarray, Zhat: np.ndarray, type="alt", t2lim="Fdist", t2cl=0.95, qlim="jm", qcl=0.95,
                 dcl=0.95):
    """VAE_SIMCA.py:230-346 restated (not importable: the script loads data at
    import, :388-389).  Z: calibration latents μ (float32 as produced by the
    encoder), Zhat: enc(dec(μ)).  Returns the class-model dict the script
    stores (latent_mean, invcovT, T2, Q, limits, dofs)."""
    Z = np.asarray(Z, np.float32)
    nc = Z.shape[1]
    n = Z.shape[0]
    x_mean = np.mean(Z, axis=0)  # float32, as the script (:246): the centring happens in float32
    cov = np.cov(Z, rowvar=False) + np.eye(nc) * 1e-12
    invcovT = np.linalg.pinv(cov)
    diff = Z - x_mean[None, :]
    T2 = np.einsum("ij,jk,ik->i", diff, invcovT, diff)
    Q = np.sum((Z - np.asarray(Zhat, np.float32)) ** 2, axis=1, dtype=np.float64).astype(np.float32)
    t2dof = t2sc = qdof = qsc = None
    # _compute_T2_limit (:281-300): percentile surrogates
    if t2lim in ("perc", "chi2"):
        T2lim = np.percentile(T2, t2cl * 100)
    elif t2lim == "Fdist":
        T2lim = nc * (n - 1) / (n - nc) * np.percentile(T2, t2cl * 100)
    elif t2lim == "chi2pom":
        h0 = float(np.mean(T2))
        v = float(np.var(T2, ddof=1)) if n > 1 else 0.0
        Nh = max(int(np.round(2 * h0 ** 2 / v)) if v > 0 else 1, 1)
        T2lim, t2dof, t2sc = h0 * np.percentile(T2, t2cl * 100) / Nh, Nh, h0
    else:
        raise ValueError(t2lim)
    # _compute_Q_limit (:302-327): jm from Q moments (not eigenvalues)
    Qd = Q.astype(np.float64)
    if qlim == "perc":
        Qlim = np.percentile(Q, qcl * 100)
    elif qlim == "jm":
        th1, th2, th3 = Qd.sum(), (Qd ** 2).sum(), (Qd ** 3).sum()
        if th1 == 0:
            Qlim = 0
        else:
            h0 = max(1 - (2 * th1 * th3) / (3 * th2 ** 2), 1e-3)
            ca = np.sqrt(2) * special.erfinv(2 * qcl - 1)
            Qlim = th1 * (1 + ca * np.sqrt(2 * th2 * h0 ** 2) / th1 + th2 * h0 * (h0 - 1) / th1 ** 2) ** (1 / h0)
    elif qlim == "chi2pom":
        v0 = Qd.mean()
        Nv = max(round(2 * v0 ** 2 / np.var(Qd, ddof=1)), 1)
        Qlim, qdof, qsc = v0 * np.percentile(Q, qcl * 100) / Nv, Nv, v0
    else:
        raise ValueError(qlim)
    # _compute_D_limit (:329-346)
    if type == "sim":
        Dlim = 1
    elif type == "alt":
        Dlim = np.sqrt(2)
    elif type == "ci":
        tr1 = nc / T2lim + Qd.sum() / Qlim
        tr2 = nc / T2lim ** 2 + (Qd ** 2).sum() / Qlim ** 2
        Dlim = tr2 / tr1 * np.percentile(Q, dcl * 100)
    elif type == "dd":
        Dlim = t2dof + qdof
    else:
        raise ValueError(type)
    return {"latent_mean": x_mean, "invcovT": invcovT, "T2": T2, "Q": Q, "T2_limit": float(T2lim),
            "Q_limit": float(Qlim), "D_limit": float(Dlim), "T2dof": t2dof, "T2scfact": t2sc, "Qdof": qdof,
            "Qscfact": qsc, "n_components": nc, "type": type}


def vaesimca_predict(model: dict, Z: np.ndarray, Zhat: np.ndarray):
    """VAE_SIMCA.py:348-382: T², latent Q and the decision (sim and ci take the max rule)."""
    Z = np.asarray(Z, np.float32)
    diff = Z - model["latent_mean"][None, :]
    T2 = np.einsum("ij,jk,ik->i", diff, model["invcovT"], diff)
    Q = np.sum((Z - np.asarray(Zhat, np.float32)) ** 2, axis=1, dtype=np.float64).astype(np.float32)
    with np.errstate(divide="ignore"):
        if model["type"] == "alt":
            D = np.sqrt((T2 / model["T2_limit"]) ** 2 + (Q / model["Q_limit"]) ** 2)
        elif model["type"] == "dd":
            D = T2 * model["T2dof"] / model["T2scfact"] + Q * model["Qdof"] / model["Qscfact"]
        else:
            D = np.maximum(T2 / model["T2_limit"], Q / model["Q_limit"])
    return D < model["D_limit"], T2, Q, D


# ---------------------------------------------------------------------------
# Synthetic spectra
# ---------------------------------------------------------------------------


def synth_spectra(n: int, p: int, k: int, rank: int = 40, seed: int = 1234, noise: float = 0.05,
                  outlier_frac: float = 0.0, dtype=np.float32, loadings: str = "bands"):
    """Rank-``rank`` spectra with a spectral gap at k plus a sloped baseline:
    scores ~ N(0, diag(s²)), s = linspace(20,8,k) ++ linspace(2,0.5,rank-k);
    Gaussian-band loadings (``loadings='bands'``; overlapping bands leave
    fewer than ~70 independent directions at p = 2048) or orthonormal
    N(0, 1) rows (``'random'``: full rank, the gap at any k — SURVEY.md §8d);
    σ = ``noise``.  ``outlier_frac`` of the rows get an extra absorption band
    (≈3σ shift) so both decisions occur."""
    rng = np.random.default_rng(seed)
    rank = min(rank, p)
    k = min(k, rank)
    s = np.concatenate([np.linspace(20, 8, k), np.linspace(2, 0.5, rank - k)])
    wl = np.linspace(0.0, 1.0, p)
    if loadings == "random":
        L = np.linalg.qr(rng.standard_normal((p, rank)))[0].T
    else:
        centers = rng.uniform(0.05, 0.95, size=rank)
        widths = rng.uniform(0.01, 0.08, size=rank)
        L = np.exp(-0.5 * ((wl[None, :] - centers[:, None]) / widths[:, None]) ** 2)
        L /= np.linalg.norm(L, axis=1, keepdims=True)
    S = rng.standard_normal((n, rank)) * s
    X = S @ L + noise * rng.standard_normal((n, p)) + (1.0 + 0.3 * wl)[None, :]
    if outlier_frac > 0:
        n_out = int(round(outlier_frac * n))
        band = np.exp(-0.5 * ((wl - 0.5) / 0.03) ** 2)
        band /= np.linalg.norm(band)
        X[n - n_out:] += 3.0 * band[None, :] * rng.uniform(0.8, 1.2, size=(n_out, 1))
    return X.astype(dtype)


# ---------------------------------------------------------------------------
# Spectral preprocessing
# ---------------------------------------------------------------------------


def preprocess_reference(X: np.ndarray, window: int | None, polyorder: int = 2, deriv: int = 0,
                         delta: float = 1.0, snv: bool = True) -> np.ndarray:
    """The drivers' preprocessing as they run it: NumPy SNV in the array dtype
    (simca_nuts.py:47-49, utils/data_utils.py:57) then
    scipy.signal.savgol_filter(..., axis=1, mode='interp') (simca_nuts.py:51,
    simca_new_cheese.py:37-38)."""
    from scipy.signal import savgol_filter

    Y = X
    if snv:
        Y = (Y - np.mean(Y, axis=1, keepdims=True)) / (np.std(Y, axis=1, keepdims=True) + 1e-8)
    if window:
        Y = savgol_filter(Y, window, polyorder, deriv=deriv, delta=delta, axis=1)
    return Y


def _fma32(c, d, a):
    # fmaf: the product of two float32 is exact in float64
    return (c.astype(np.float64) * d.astype(np.float64) + a.astype(np.float64)).astype(np.float32)


def prep_fused_f32(X: np.ndarray, window: int, taps: np.ndarray, deriv: int, snv: bool) -> np.ndarray:
    """NumPy restatement of the lazy view's float32 formula (include/ocm.h,
    ``ocm_prep``): differences of neighbouring raw samples with antisymmetric
    taps (odd deriv), symmetric pair sums (deriv 0), edge rows about u_j
    (deriv >= 1), times 1/(std + 1e-8).  Used by the CPU tests to check that
    the formula the kernels share is SG(SNV(x)) to float32 rounding."""
    X = np.asarray(X, dtype=np.float32)
    m, p = X.shape
    w = int(window or 0)
    h = w // 2
    t32 = np.asarray(taps, dtype=np.float32) if w else None
    mean = X.astype(np.float64).mean(1)
    sd = np.sqrt(((X.astype(np.float64) - mean[:, None]) ** 2).mean(1)).astype(np.float32)
    s = (np.float32(1.0) / (sd + np.float32(1e-8))).astype(np.float32)
    mr = mean.astype(np.float32)
    U = (X - mr[:, None]).astype(np.float32) if (snv and (not w or deriv == 0)) else X
    if not w:
        A = U
    else:
        A = np.zeros((m, p), dtype=np.float32)
        c = t32[:w]
        J = np.arange(h, p - h)
        if deriv % 2 == 1:
            for t in range(1, h + 1):
                A[:, J] = _fma32(c[h + t], (U[:, J + t] - U[:, J - t]).astype(np.float32), A[:, J])
        elif deriv == 0:
            A[:, J] = (c[h] * U[:, J]).astype(np.float32)
            for t in range(1, h + 1):
                A[:, J] = _fma32(c[h + t], (U[:, J + t] + U[:, J - t]).astype(np.float32), A[:, J])
        else:
            for t in range(1, h + 1):
                d = ((U[:, J + t] - U[:, J]).astype(np.float32) + (U[:, J - t] - U[:, J]).astype(np.float32))
                A[:, J] = _fma32(c[h + t], d.astype(np.float32), A[:, J])
        L = t32[w:w + h * w].reshape(h, w)
        R = t32[w + h * w:].reshape(h, w)
        for i in range(h):
            for j, row, s0 in ((i, L[i], 0), (p - h + i, R[i], p - w)):
                ref = U[:, j] if deriv >= 1 else np.zeros(m, np.float32)
                a = np.zeros(m, np.float32)
                for t in range(w):
                    a = _fma32(row[t], (U[:, s0 + t] - ref).astype(np.float32), a)
                A[:, j] = a
    return (A * s[:, None]).astype(np.float32) if snv else A
