"""Drop-in ``SIMCA`` estimator backed by the MI355X engine (libocm.so).

Same class name, constructor keywords, attributes, ``_model`` keys, return
types and quirks as the reference estimator (TEAM-AIOLY/OCM-VAE-SIMCA
``utils/SIMCA.py:12-381``), so drivers such as ``simca_nuts.py``
(``from utils import SIMCA`` … ``.fit`` / ``.predict`` / ``.transform`` /
``._model[cls]['D_limit']``) run unchanged.  The arithmetic runs on the GPU
through ``ocm.engine`` (Gram on int8-digit MFMA — three base-254 digits per
value, fp32-grade, outlier rows added back exactly —, fp64 eigensolver,
single-pass projection/Q/T² scoring); only the scalar limits are evaluated
on the host.

Inputs may be NumPy arrays (copied to HBM; results come back as NumPy, like
the reference), CUDA torch tensors (device-resident; ``predict`` then
returns a device tensor and ``_model`` arrays are materialised lazily), or a
lazy preprocessed view (``ocm.preprocess.snv_savgol(X, ..., lazy=True)``:
the drivers' SNV / Savitzky–Golay step, applied inside the Gram quantiser and
the scoring kernel instead of as a pass of its own; results as for tensors).

Multi-GPU: under ``torchrun`` (a process group of W > 1
ranks) ``fit`` / ``predict`` / ``transform`` first exchange a fingerprint of
their arguments (``ocm.replica``).  When every rank passed the same X and
labels — an unchanged driver — the rows are sharded: rank r fits and scores
its contiguous block, the class moments meet in one all-reduce, and the
per-row results (``_model`` T / T2 / Q, predict's (m, C) matrix, transform's
arrays) are all-gathered, so every rank returns the single-process result.
When the ranks' data differ, each rank runs the reference's per-process
computation.  Every rank must make the call (``ocm.replica.per_process()``
for calls on a subset of the ranks).

Documented deviations:
* predict/transform use the exact top-k loadings of the covariance; the
  reference re-estimates them with a randomized ``PCA(k)`` (utils/SIMCA.py:75)
  which agrees on the same subspace to its own randomised tolerance;
* ``_model[cls]['pca_model']`` is an engine-backed facade with the sklearn
  PCA attributes drivers read (``components_``, ``mean_``, ``transform``,
  ``inverse_transform``);
* ``eigs_all`` holds the leading k eigenvalues from the HIP eigensolver and,
  on first access only, the rest of the spectrum from libocm's dense
  eigensolver (a diagnostic no limit uses; the θ moments come from device
  traces);
* float64 inputs are computed in float64 as the reference's PCA then is
  (fp64-MFMA Gram, fp64 scoring; T, Q and ``_model`` arrays float64);
* ``n_components`` may be any k ≤ p as in the reference; beyond 64 the
  eigensolver's block steps run on the host in fp64 and scoring takes one
  launch per 64 components, and a CV sweep with ``LV_max`` > 64 runs the
  generic refit loop instead of the fold engine;
* a fit whose leading k eigenpairs do not converge (no spectral gap after
  component k within the iteration budget) takes the dense eigensolver
  (``ocm_eigh_f64``) with a RuntimeWarning instead of returning loadings of
  an unconverged subspace.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist
from sklearn.base import BaseEstimator, ClassifierMixin

from ocm import engine, limits
from ocm.dist import make_allreduce
from ocm.prepview import PrepView
from ocm.replica import gather_rows, replicated_group
from ocm.synth import shard_bounds

__all__ = ["SIMCA"]


class _Lazy:
    __slots__ = ("fn",)

    def __init__(self, fn):
        self.fn = fn


class ModelDict(dict):
    """``_model[cls]`` — a dict whose large arrays are copied out of HBM on
    first access (the timed path never pays for host copies)."""

    def __getitem__(self, key):
        v = dict.__getitem__(self, key)
        if isinstance(v, _Lazy):
            v = v.fn()
            dict.__setitem__(self, key, v)
        return v

    def get(self, key, default=None):
        return self[key] if key in self else default

    def values(self):
        return [self[k] for k in self]

    def items(self):
        return [(k, self[k]) for k in self]

    def __repr__(self):
        return "{" + ", ".join(f"{k!r}: {self[k]!r}" for k in self) + "}"


class EnginePCA:
    """sklearn-PCA-shaped view of one class model (what ``pca_model`` exposes)."""

    def __init__(self, fit: engine.ClassFit, out_dtype):
        self._fit = fit
        self._dt = out_dtype
        self.n_components = fit.k
        self.n_components_ = fit.k
        self.n_features_in_ = fit.p

    @property
    def components_(self):
        return self._fit.P64.cpu().numpy().astype(self._dt)

    @property
    def mean_(self):
        return self._fit.mean64.cpu().numpy().astype(self._dt)

    @property
    def explained_variance_(self):
        return self._fit.evals_host.astype(self._dt)

    def transform(self, X):
        Xd = engine.as_device_x(X)
        out = engine.score(Xd, None, Xd.shape[0], self._fit.P64, self._fit.mean64, self._fit.inv_diag,
                           want_T=True, want_T2=False, want_Q=False)
        T = out["T"]
        return T if _is_dev(X) else T.cpu().numpy().astype(self._dt)

    def inverse_transform(self, T):
        # T·P + μ (sklearn/decomposition/_base.py:197); facade utility, not on the hot path
        Td = T if isinstance(T, torch.Tensor) else torch.from_numpy(np.asarray(T))
        Td = Td.to(self._fit.P64.device, torch.float64)
        Xr = Td @ self._fit.P64 + self._fit.mean64
        return Xr if isinstance(T, torch.Tensor) else Xr.cpu().numpy().astype(self._dt)


def _np(t, dtype=None):
    a = t.detach().cpu().numpy()
    return a.astype(dtype) if dtype is not None and a.dtype != dtype else a



def _rates(TP, TN, FP, FN):
    """Sensitivity / specificity / accuracy / efficiency in percent from the
    confusion counts (utils/SIMCA.py:247-266; NumPy division semantics)."""
    with np.errstate(divide="ignore", invalid="ignore"):
        sensitivity = TP / (TP + FN) * 100
        specificity = TN / (TN + FP) * 100
        accuracy = (TP + TN) / (TP + TN + FP + FN) * 100
        efficiency = np.sqrt(sensitivity * specificity)
    return {"sensitivity": sensitivity, "specificity": specificity, "accuracy": accuracy,
            "efficiency": efficiency, "TP": TP, "TN": TN, "FP": FP, "FN": FN}

def check_components(k: int, n: int, p: int):
    """The reference fits PCA(n_components=k) on each class (utils/SIMCA.py:73), so
    k > min(n, p) raises sklearn's ValueError (sklearn/decomposition/_pca.py,
    ``_fit``); the same message here, before any device work.  The solver it
    names is the one svd_solver='auto' picks for an n×p class matrix when k
    cannot fit (a tall, narrow matrix takes 'covariance_eigh', any other 'full')."""
    if k > min(n, p):
        solver = "covariance_eigh" if p <= 1000 and n >= 10 * p else "full"
        raise ValueError(f"n_components={k} must be between 0 and min(n_samples, n_features)={min(n, p)} "
                         f"with svd_solver='{solver}'")


_check_components = check_components


class SIMCA(BaseEstimator, ClassifierMixin):
    def __init__(self, n_components=2, model_class=None, type: str = "alt", t2lim="Fdist", t2cl=0.95, qlim="jm",
                 qcl=0.95, dcl=0.95, maxPC=20, criteria="compl", verbose=True):
        self.n_components = n_components
        self.model_class = model_class
        self.type = type
        self.t2lim = t2lim
        self.t2cl = t2cl
        self.qlim = qlim
        self.qcl = qcl
        self.criteria = criteria
        self.dcl = dcl
        self.maxPC = maxPC
        self.metrics = {}
        self.verbose = verbose

    # ------------------------------------------------------------------ fit
    def fit(self, X, classes):
        """utils/SIMCA.py:27-59 (same parameter normalisation and quirks)."""
        if self.model_class is None:
            self.model_class = np.unique(_host_labels(classes))
        elif isinstance(self.model_class, (int, np.integer)):
            self.model_class = [self.model_class]
        if not isinstance(self.n_components, list):
            self.n_components = [self.n_components]
        if len(self.n_components) == 1:
            self.n_components = [self.n_components[0]] * len(self.model_class)
        elif len(self.n_components) != len(self.model_class):
            raise ValueError("n_components length must match number of classes")
        if self.type == "dd" and self.t2lim != "chi2pom":
            print("t2lim set as chi2pom")
            self.t2lim = "chi2pom"
        if self.type == "dd" and self.qlim != "chi2pom":
            print("qlim set as chi2pom")
            self.qlim = "chi2pom"

        self._out_dtype = _out_dtype(X)
        # Under torchrun with the same X and y on every rank (an unchanged
        # driver, simca_nuts.py:186-189) the fit is row-sharded: rank r fits
        # its contiguous block with one packed all-reduce of the moments and
        # the per-row arrays of _model are all-gathered, so every rank holds
        # the single-process model.  Otherwise the reference's per-process fit.
        group = replicated_group(X, classes, eligible=_n_rows(classes) == X.shape[0])
        self._sharded = group is not None
        self._model = {}
        self._fits = {}
        if self._sharded:
            lab_h = _host_labels(classes)
            bounds = _bounds(X.shape[0])
            rank = dist.get_rank()
            lo, hi = bounds[rank]
            Xd = engine.as_device_x(X[lo:hi])
            ar = make_allreduce(group)
            for i, cls in enumerate(self.model_class):
                mask = lab_h == cls
                counts = [int(mask[a:b].sum()) for a, b in bounds]
                _check_components(int(self.n_components[i]), sum(counts), X.shape[1])
                rows = None if counts[rank] == hi - lo else \
                    torch.from_numpy(np.flatnonzero(mask[lo:hi])).to(Xd.device)
                self._model[cls] = self._fit_one_class(Xd, rows, counts[rank], int(self.n_components[i]),
                                                       (counts, ar))
                self._fits[cls] = self._model[cls]._fit
        else:
            Xd = engine.as_device_x(X)
            lab = _device_labels(classes, Xd.device)
            for i, cls in enumerate(self.model_class):
                mask = lab == int(cls)
                n = int(mask.sum().item())
                _check_components(int(self.n_components[i]), n, Xd.shape[1])
                rows = None if n == Xd.shape[0] else torch.nonzero(mask).flatten()
                self._model[cls] = self._fit_one_class(Xd, rows, n, int(self.n_components[i]))
                self._fits[cls] = self._model[cls]._fit
        self.n_features_in_ = X.shape[1]
        self.is_fitted_ = True
        return self

    def _fit_one_class(self, Xd, rows, n, k, shard=None):
        """utils/SIMCA.py:62-99 on the device.  ``shard`` = (class rows of each
        rank, all-reduce) marks a row-sharded fit of this rank's block Xd."""
        if shard is None:
            fit = engine.fit_class(Xd, rows, n, k, limits.theta_mode_for(self), want_T=True, keep_C=True)
        else:
            counts, ar = shard
            fit = engine.fit_class(Xd, rows, n, k, limits.theta_mode_for(self), want_T=True, keep_C=True,
                                   allreduce=ar)
            # every rank holds the single-process per-row arrays (utils/SIMCA.py:65-71, 89-95)
            fit.T, fit.T2, fit.Q = (gather_rows(t, counts) for t in (fit.T, fit.T2, fit.Q))
            n = fit.n
        T2m = limits.Moments(n, lambda: fit.T2_stats, None, lambda pct: engine.percentile(fit.T2, pct))
        Qm = limits.Moments(n, lambda: fit.Q_stats, None, lambda pct: engine.percentile(fit.Q, pct))
        T2_limit = limits.t2_limit(self, T2m, k)
        Q_limit = limits.q_limit(self, Qm, fit.thetas)
        D_limit = limits.critic_distance(self, T2_limit, Q_limit, fit.thetas, k)
        engine._mark("limits")
        dec = self._decision(T2_limit, Q_limit, D_limit)
        dt = self._out_dtype
        red = {}

        def reds():
            if not red:
                t2r, qr, _ = engine.decide(fit.T2, fit.Q, dec)
                red["t2"], red["q"] = _np(t2r), _np(qr)
            return red

        md = ModelDict()
        md._fit = fit
        md.update({
            "pca_model": EnginePCA(fit, dt),
            "n_components": k,
            "xmean": _Lazy(lambda: _np(fit.mean64, dt)),
            "invcovT": _Lazy(lambda: _np(fit.invcov_mat())),
            "eigs_all": _Lazy(lambda: _all_eigs(fit, n)),
            "T": _Lazy(lambda: _np(fit.T, dt)),
            "P": _Lazy(lambda: _np(fit.P64, dt)),
            "T2": _Lazy(lambda: _np(fit.T2)),
            "Q": _Lazy(lambda: _np(fit.Q, dt)),
            "T2red": _Lazy(lambda: reds()["t2"]),
            "Qred": _Lazy(lambda: reds()["q"]),
            "T2_limit": T2_limit,
            "Q_limit": Q_limit,
            "D_limit": D_limit,
            "n_samples": n,
        })
        return md

    def _score_shard(self, X):
        """(lo, hi, rows of each rank) when the model was fitted row-sharded and
        every rank scores the same X (ocm/replica.py): this rank scores rows
        [lo, hi) and the results are all-gathered.  None: score all rows here."""
        if not getattr(self, "_sharded", False) or replicated_group(X) is None:
            return None
        bounds = _bounds(X.shape[0])
        lo, hi = bounds[dist.get_rank()]
        return lo, hi, [b - a for a, b in bounds]

    def _decision(self, T2_limit, Q_limit, D_limit):
        if self.type == "dd":
            return engine.make_decision("dd", self._t2dof / self._t2scfact, self._qdof / self._qscfact, D_limit)
        if self.type not in ("sim", "alt", "ci"):
            raise UnboundLocalError(f"local variable 'dred' referenced before assignment (type={self.type!r})")
        return engine.make_decision(self.type, 1.0 / T2_limit, 1.0 / Q_limit, D_limit)

    # ------------------------------------------------------------ transform
    def transform(self, X):
        """utils/SIMCA.py:101-117 — (T2, T2red, Q, Qred) of the LAST class."""
        cls = self.model_class[-1]
        fit = self._fits[cls]
        m = self._model[cls]
        shard = self._score_shard(X)
        Xd = engine.as_device_x(X if shard is None else X[shard[0]:shard[1]])
        if Xd.shape[0]:
            out = engine.score(Xd, None, Xd.shape[0], fit.P64, fit.mean64, fit.inv_diag)
        else:  # a rank without rows of a sharded transform
            vdt = torch.float64 if Xd.dtype == torch.float64 else torch.float32
            out = {"T2": torch.empty(0, dtype=torch.float64, device=Xd.device),
                   "Q": torch.empty(0, dtype=vdt, device=Xd.device)}
        if shard is not None:
            out = {key: gather_rows(out[key], shard[2]) for key in ("T2", "Q")}
        dec = self._decision(m["T2_limit"], m["Q_limit"], m["D_limit"])
        t2r, qr, _ = engine.decide(out["T2"], out["Q"], dec)
        if _is_dev(X):
            return out["T2"], t2r, out["Q"], qr
        return _np(out["T2"]), _np(t2r), _np(out["Q"], self._out_dtype), _np(qr)

    # -------------------------------------------------------------- predict
    def predict(self, X, y_true=None):
        """utils/SIMCA.py:120-154 — (m, C) float64 of 0/1, decision fused in the scoring kernel."""
        shard = self._score_shard(X)
        Xd = engine.as_device_x(X if shard is None else X[shard[0]:shard[1]])
        m = Xd.shape[0]
        C = len(self.model_class)
        pred = torch.zeros((m, C), dtype=torch.float64, device=Xd.device)
        for i, cls in enumerate(self.model_class):
            fit = self._fits[cls]
            info = self._model[cls]
            dec = self._decision(info["T2_limit"], info["Q_limit"], info["D_limit"])
            if m == 0:  # a rank without rows of a sharded predict
                continue
            acc = pred[:, i:] if C > 1 else pred
            engine.score(Xd, None, m, fit.P64, fit.mean64, fit.inv_diag, want_T2=False, want_Q=False,
                         decision=dec, accept_out=acc, accept_stride=C)
        if shard is not None:  # every rank returns the (m, C) matrix of all rows
            pred = gather_rows(pred, shard[2])
            m = pred.shape[0]
        out = pred if _is_dev(X) else pred.cpu().numpy()
        if y_true is not None:
            yt = _host_labels(y_true)
            for i, cls in enumerate(self.model_class):
                if yt.shape == (m,):
                    # counts on the device from the prediction column (ocm_confusion_counts)
                    pos = torch.from_numpy(np.ascontiguousarray(yt == cls).astype(np.uint8)).to(Xd.device)
                    cnt = engine.confusion_counts(pred[:, i:], pos, stride=C).cpu().numpy()
                    self.metrics[cls] = _rates(*(np.int64(v) for v in cnt))
                else:  # the reference's NumPy broadcasting semantics for odd label shapes
                    ph = pred.cpu().numpy()
                    self.metrics[cls] = self._metrics_simca_conformity(yt, ph[:, i], cls)
                if self.verbose:
                    mt = self.metrics[cls]
                    print(f"Sample class {cls} = {np.sum(yt == cls)}")
                    print(f"Confusion Matrix for class {cls}:\nTP: {mt['TP']}, TN: {mt['TN']}, FP: {mt['FP']}, FN: {mt['FN']}")
                    print(f"Class {cls} - Sensitivity: {mt['sensitivity']}, Specificity: {mt['specificity']:.4f}, "
                          f"Accuracy: {mt['accuracy']:.4f}, Efficiency: {mt['efficiency']:.4f}")
        return out

    # -------------------------------------------------------------- metrics
    def _metrics_simca_conformity(self, y_true, y_pred, class_index):
        """utils/SIMCA.py:238-266 (NumPy broadcasting semantics kept)."""
        y_true = _host_labels(y_true)
        y_pred = y_pred.cpu().numpy() if isinstance(y_pred, torch.Tensor) else np.asarray(y_pred)
        true_class = (y_true == class_index).astype(int)
        return _rates(np.sum((y_pred == 1) & (true_class == 1)), np.sum((y_pred == 0) & (true_class == 0)),
                      np.sum((y_pred == 1) & (true_class == 0)), np.sum((y_pred == 0) & (true_class == 1)))

    def score(self, X, y):
        """utils/SIMCA.py:268-278 — returns specificity (2-D y_pred, list class index, as the reference)."""
        y_pred = self.predict(X, y_true=y)
        metrics = self._metrics_simca_conformity(y, y_pred, self.model_class)
        return metrics["specificity"]

    # ------------------------------------------------------------ plotting
    # Host glue (out of the hot path): the T²red/Qred plane of
    # transform() with the acceptance boundary of the decision rule.  Method
    # names and return values follow utils/SIMCA.py:280-381; like there, the
    # points are transform(X) (the LAST class) on every panel.

    def _t2q_panels(self, X):
        """(class, T2red, Qred, D_limit, boundary x, boundary y) per class."""
        _, t2red, _, qred = self.transform(X)
        t2red = t2red.cpu().numpy() if isinstance(t2red, torch.Tensor) else np.asarray(t2red)
        qred = qred.cpu().numpy() if isinstance(qred, torch.Tensor) else np.asarray(qred)
        for cls in self._model:
            dlim = float(self._model[cls]["D_limit"])
            bx, by = _boundary(self.type, dlim)
            yield cls, t2red, qred, dlim, bx, by

    def toplotT2Q(self, X, y_test):
        """matplotlib scatter of the first class panel; returns the pyplot module (as the reference)."""
        import matplotlib.pyplot as plt

        for cls, t2red, qred, _, bx, by in self._t2q_panels(X):
            fig, ax = plt.subplots(figsize=(6, 6))
            pts = ax.scatter(t2red, qred, c=np.asarray(y_test), cmap="viridis", s=40, edgecolor="k",
                             linewidth=0.5, alpha=0.7)
            ax.plot(bx, by, "b-", lw=2)
            ax.legend(*pts.legend_elements(), title="Class")
            ax.set_xlabel(r"$T^2_{red}$")
            ax.set_ylabel(r"$Q_{red}$")
            ax.set_title(rf"$T^2$ vs $Q$  class {cls}")
            ax.grid(True, alpha=0.3)
            ax.set_xlim(left=0)
            ax.set_ylim(bottom=0)
            fig.tight_layout()
            plt.show()
            return plt  # the reference stops after the first class

    def toplotT2Q_iterative(self, X, y_test):
        """plotly figure per class (one trace per label + the boundary); one figure or a list."""
        import plotly.graph_objects as go

        labels = np.asarray(y_test).astype(str)
        figs = []
        for cls, t2red, qred, dlim, bx, by in self._t2q_panels(X):
            fig = go.Figure()
            for lab in np.unique(labels):
                sel = labels == lab
                fig.add_trace(go.Scatter(x=t2red[sel], y=qred[sel], mode="markers", name=f"Class {lab}",
                                         marker=dict(size=7, line=dict(width=0.7, color="black"))))
            fig.add_trace(go.Scatter(x=bx, y=by, mode="lines", name="Decision Limit",
                                     line=dict(color="blue", width=3)))
            top_x = 1.05 * max(float(t2red.max()) if t2red.size else 0.0, dlim)
            top_y = 1.05 * max(float(qred.max()) if qred.size else 0.0, dlim)
            fig.update_layout(width=600, height=600, title=f"T2 vs Q, class {cls}",
                              xaxis=dict(title="T<sup>2</sup><sub>red</sub>", range=[0, top_x]),
                              yaxis=dict(title="Q<sub>red</sub>", range=[0, top_y]))
            figs.append(fig)
        return figs[0] if len(figs) == 1 else figs


def _boundary(type_name, dlim, npts=1201):
    """Acceptance boundary dred(t, q) = D_limit in the (T2red, Qred) plane:
    a quarter circle for 'alt', a square corner for 'sim', a line for 'ci'
    (SURVEY.md §8a predict row); 'dd' is a line in dof-scaled units."""
    t = np.linspace(0.0, dlim, npts)
    if type_name == "sim":
        return np.array([0.0, dlim, dlim]), np.array([dlim, dlim, 0.0])
    if type_name in ("ci", "dd"):
        return t, dlim - t
    return t, np.sqrt(np.maximum(dlim * dlim - t * t, 0.0))


def _is_dev(X):
    """Device-resident input (tensor or lazy view): results stay on the device."""
    return isinstance(X, (torch.Tensor, PrepView))


def _out_dtype(X):
    if isinstance(X, (torch.Tensor, PrepView)):
        return np.float64 if X.dtype == torch.float64 else np.float32
    return np.float64 if np.asarray(X).dtype == np.float64 else np.float32


def _n_rows(y) -> int:
    return int(y.shape[0]) if hasattr(y, "shape") and len(y.shape) else len(y)


def _bounds(n: int):
    """Every rank's contiguous row block of an n-row matrix."""
    W = dist.get_world_size()
    return [shard_bounds(n, r, W) for r in range(W)]


def _host_labels(y):
    if isinstance(y, torch.Tensor):
        return y.detach().cpu().numpy()
    return np.asarray(y)


def _device_labels(y, device):
    if isinstance(y, torch.Tensor):
        return y.to(device=device, dtype=torch.int64)
    return torch.from_numpy(np.asarray(y).astype(np.int64)).to(device)


def _all_eigs(fit: engine.ClassFit, n: int):
    """Full explained-variance spectrum (min(n, p) values, descending,
    utils/SIMCA.py:88): the leading k from the fit's eigensolver, the rest from
    the dense libocm eigensolver on the HBM-resident covariance on first
    access (``ocm_eigh_f64``; diagnostic only, no limit uses it)."""
    r = min(n, fit.p)
    if fit.C is None:
        return fit.evals_host.copy()
    lam, _ = engine.eigh_dense(fit.C, 0)
    full = lam[:r].cpu().numpy()
    full[: fit.k] = fit.evals_host
    return full
