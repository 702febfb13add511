"""Fold engine for class-wise SIMCA cross-validation (C3).

Replaces the per-(combo, LV, fold) refit loop of utils/CVSIMCA.py:145-222
for this package's SIMCA under a ``ClasswiseKFoldWithExternalVal`` split:

* one segmented Gram pass over the target-class rows, segments = folds
  (``ocm_gram_f32``); fold f trains on Gram(total) − Gram(f) (fp64
  downdating, ``ocm_cov_from_gram`` with coefficients +1/−1);
* one eigensolve per fold at LV_max; every LV in the sweep is a prefix of it
  (the LV-component PCA of the same class matrix is the leading LV of the
  same decomposition, utils/SIMCA.py:64-70); the tail moments θ for LV are
  θ(LV_max) plus the eigenvalues LV..LV_max−1;
* each fold's test rows (held-out fold ∪ all other-class rows,
  utils/CVSIMCA.py:77-80) are scored ONCE at LV_max by row index
  (``ocm_score_f32``); ``ocm_cv_counts`` turns those scores into confusion
  counts for every (param combo, LV) decision at once;
* training-row statistics (``perc`` / ``chi2pom`` limits) come from one more
  scoring of the fold's training rows and ``ocm_cv_prefix``.

Aggregation is the reference's: spec = mean over folds of TN/(TN+FP)·100
(:195-203), sens from the pooled prediction vector, where target rows carry
their own fold's prediction and other-class rows the LAST fold's
(:190, 205-207), eff = √(sens·spec) (:208).

Multi-GPU (``group`` given; the drop-in ``grid`` passes dist.group.WORLD
when the process runs as one of W > 1 ranks and every rank passed the same X
and y, ``ocm.replica.replicated_group``): each rank holds a contiguous row block of X
(``row_offset``) and the full label vector.  Fold f's eigensolve runs on
its owner rank f mod W: every rank forms its local TRAIN Gram of fold f
(Σ_g G_g − G_f, fp64 downdating on the device) and one RCCL reduce brings
the sum to the owner only (K reduces of the packed upper triangle, p(p+1)/2
+ p + 1 doubles with the fold's column sums and row count, instead of K
all-reduces).  All K reduces are issued before any eigensolve, so the owners
solve their folds concurrently (⌈K/W⌉ eigensolves deep).  The owners
broadcast the fold model (P, μ, λ, θ ≈ 0.3 MB), every rank scores its own
rows, the confusion counts and training moments are all-reduced, and the
pooled prediction vectors travel as one device all-gather of each rank's
row block.  Same code path at W = 1 without collectives.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from . import engine, limits
from .replica import replicated_group

__all__ = ["grid", "cv_grid", "FoldModels"]


class _Spec:
    """The limit-relevant configuration of one param combo (SIMCA kwargs)."""

    def __init__(self, params: dict):
        self.type = params.get("type", "alt")
        self.t2lim = params.get("t2lim", "Fdist")
        self.t2cl = params.get("t2cl", 0.95)
        self.qlim = params.get("qlim", "jm")
        self.qcl = params.get("qcl", 0.95)
        self.dcl = params.get("dcl", 0.95)
        if self.type == "dd":  # utils/SIMCA.py:42-48
            self.t2lim = "chi2pom"
            self.qlim = "chi2pom"

    def needs_train_stats(self) -> bool:
        return self.t2lim in ("perc", "chi2pom") or self.qlim in ("perc", "chi2pom")

    def needs_percentile(self) -> bool:
        return self.t2lim == "perc" or self.qlim == "perc"


def _applicable(base_est, X, y, cv, lv_values, param_grid):
    """The fold engine covers this package's SIMCA (not wrapped in a Pipeline),
    a ClasswiseKFoldWithExternalVal split, an LV sweep, and a single target
    label whose model_class is that label (or None)."""
    from sklearn.model_selection import ParameterGrid
    from utils.CVSIMCA import ClasswiseKFoldWithExternalVal
    from utils.SIMCA import SIMCA

    if type(base_est) is not SIMCA or not isinstance(cv, ClasswiseKFoldWithExternalVal):
        return None
    if lv_values is None or len(lv_values) == 0 or y is None:
        return None
    y = np.asarray(y)
    cls_idx = cv.target_indices(X, y)
    labels = np.unique(y[cls_idx])
    if labels.size != 1:
        return None
    tl = labels[0]
    combos = list(ParameterGrid(param_grid))
    base = base_est.get_params()
    for combo in combos:
        params = dict(base, **combo)
        mc = params.get("model_class")
        if mc is not None and not np.array_equal(np.ravel(np.asarray(mc)), np.asarray([tl])):
            return None
    if max(lv_values) > 64 or min(lv_values) < 1:
        return None
    from .prepview import PrepView

    if isinstance(X, PrepView):
        return cls_idx, labels[0], combos, base
    if (X.dtype == torch.float64) if isinstance(X, torch.Tensor) else (np.asarray(X).dtype == np.float64):
        return None  # float64 spectra: the refit loop runs the fp64 fits (utils/SIMCA.py:64-66 dtype rule)
    return cls_idx, tl, combos, base


def grid(base_est, X, y, cv, lv_values, param_grid, class_index, store_predictions):
    """utils/CVSIMCA.py drop-in hook: (records, by_combo), or (None, None)
    when the fold engine does not cover the configuration."""
    try:
        app, err = _applicable(base_est, X, y, cv, lv_values, param_grid), None
    except Exception as e:  # raised after the exchange, so the other ranks are not left waiting in it
        app, err = None, e
    # Under torchrun (an initialised world of W > 1 ranks) the drop-in is
    # collective only when every rank passed the same X and y, as an unchanged
    # driver does (ocm/replica.py): rank r then keeps its contiguous row block
    # and the fold engine runs sharded (C3), and every rank
    # returns the same records and predictions.  Ranks holding different data
    # run the reference's per-process CV.  Every rank exchanges its
    # fingerprint before anything rank-dependent decides the path.
    eligible = app is not None and y is not None and int(X.shape[0]) == int(np.asarray(y).shape[0])
    group = replicated_group(X, y, eligible)
    if err is not None:
        raise err
    if app is None:
        return None, None
    cls_idx, tl, combos, base = app
    if class_index is None:
        # the reference reads simca.model_class after fit: the list [label]
        class_index = [tl]
    y = np.asarray(y)
    folds = [cls_idx[test_rel] for _, test_rel in cv.kf.split(cls_idx)]
    if group is None:
        return cv_grid(X, y, folds, cls_idx, lv_values, combos, base, class_index, store_predictions)
    from .synth import shard_bounds

    lo, hi = shard_bounds(int(y.shape[0]), dist.get_rank(group), dist.get_world_size(group))
    return cv_grid(X[lo:hi], y, folds, cls_idx, lv_values, combos, base, class_index, store_predictions,
                   row_offset=lo, group=group)


class FoldModels:
    """Per-fold eigen-models at LV_max (device tensors on every rank)."""

    def __init__(self):
        self.evals = []     # (LVmax,) f64 device
        self.evecs = []     # (LVmax, p) f64 device
        self.mean = []      # (p,) f64 device
        self.inv = []       # (LVmax,) f64 device: diag of invcovT
        self.evals_h = []   # host numpy
        self.theta_h = []   # host (3,) tail moments at LVmax
        self.n_train = []


def _inv_evals(evals: torch.Tensor, rcond=1e-15) -> torch.Tensor:
    cut = rcond * evals.abs().max()
    return torch.where(evals.abs() > cut, 1.0 / evals, torch.zeros_like(evals))


def _thetas_for(lv, lvmax, evals_h, theta_h):
    """θ_m(LV) = Σ_{i>LV} λ_i^m = θ_m(LVmax) + Σ_{LV≤i<LVmax} λ_i^m."""
    tail = evals_h[lv:lvmax]
    return (float(theta_h[0] + np.sum(tail)), float(theta_h[1] + np.sum(tail ** 2)),
            float(theta_h[2] + np.sum(tail ** 3)))


def _local(idx: np.ndarray, lo: int, hi: int) -> np.ndarray:
    """Global row indices in [lo, hi) → local indices."""
    sel = idx[(idx >= lo) & (idx < hi)]
    return (sel - lo).astype(np.int64)


def _rates(TP, TN, FP, FN):
    """utils/SIMCA.py:246-250 on int64 counts (NaN on an empty denominator)."""
    TP, TN, FP, FN = (np.int64(v) for v in (TP, TN, FP, FN))
    with np.errstate(divide="ignore", invalid="ignore"):
        sens = TP / (TP + FN) * 100
        spec = TN / (TN + FP) * 100
    return sens, spec


def cv_grid(X, y, folds, cls_idx, lv_values, combos, base_params, class_index, store_predictions,
            row_offset=0, group=None):
    """The fold engine.  X: this rank's rows (host array or device tensor) =
    global rows [row_offset, row_offset + len(X)); y, folds, cls_idx: global.
    Returns (records, by_combo) in the reference's record order."""
    Xd = engine.as_device_f32(X)
    dev = Xd.device
    n_loc, p = Xd.shape
    lo, hi = row_offset, row_offset + n_loc
    y = np.asarray(y)
    n_glob = y.shape[0]
    # cross-rank only when a group is passed explicitly (``grid`` passes WORLD
    # under torchrun); an initialised process group alone changes nothing
    distributed = group is not None
    W = dist.get_world_size(group) if distributed else 1
    R = dist.get_rank(group) if distributed else 0
    K = len(folds)
    lvs = sorted(set(int(v) for v in lv_values))
    lvmax = lvs[-1]
    n_target = int(cls_idx.size)
    # the reference fits each fold's SIMCA on its training rows of the class, LV
    # by LV in the grid's order, fold by fold (utils/CVSIMCA.py:158-185): the
    # first LV above min(n_train, p) raises sklearn's ValueError there
    from utils.SIMCA import check_components

    for lv in lv_values:
        for f_ in folds:
            n_tr = n_target - int(f_.size)
            check_components(int(lv), n_tr, p)
    specs = [_Spec(dict(base_params, **c)) for c in combos]
    theta_mode = max(limits.theta_mode_for(s) for s in specs)
    need_train = any(s.needs_train_stats() for s in specs)
    need_pct = any(s.needs_percentile() for s in specs)
    others = np.setdiff1d(np.arange(n_glob), cls_idx)
    positive_glob = (y == np.asarray(class_index)) if np.ndim(class_index) else (y == class_index)
    positive_glob = np.asarray(positive_glob, dtype=bool).reshape(n_glob)

    # ---- pass 1: per-fold Grams of the target rows (one HBM pass) ----
    loc_folds = [_local(f, lo, hi) for f in folds]
    order = np.concatenate(loc_folds) if loc_folds else np.zeros(0, np.int64)
    seg = np.concatenate([[0], np.cumsum([f.size for f in loc_folds])]).astype(np.int64)
    rows_t = torch.from_numpy(order).to(dev)
    if order.size:
        shift64 = engine.colmean(Xd, rows_t, min(int(order.size), engine.SHIFT_SAMPLE))
    else:
        shift64 = torch.zeros(p, dtype=torch.float64, device=dev)
    if distributed:
        has = torch.tensor([1.0 if order.size else 0.0], dtype=torch.float64, device=dev)
        shift64 = shift64 * has
        dist.all_reduce(shift64, group=group)
        dist.all_reduce(has, group=group)
        shift64 /= has
    shift32 = engine.cast_f32(shift64)
    if order.size:
        G, cs = engine.gram(Xd, rows_t, seg, shift32)
    else:
        G = torch.zeros((K, p, p), dtype=torch.float64, device=dev)
        cs = torch.zeros((K, p), dtype=torch.float64, device=dev)
    # local total Gram Σ_g G_g and column sums (distributed: this rank's rows
    # only; the packed train moments below carry them to the fold owners)
    Gt = torch.empty((p, p), dtype=torch.float64, device=dev)
    cst = torch.empty(p, dtype=torch.float64, device=dev)
    engine.gram_combine([(1.0, G[f], cs[f]) for f in range(K)], Gt, cst)

    # ---- per-fold eigen-models (fold f on rank f mod W, then broadcast) ----
    # Distributed: every fold's train-Gram reduce is issued before any
    # eigensolve, so the owners solve their folds at the same time (⌈K/W⌉
    # eigensolves deep instead of K), and the model broadcasts go out
    # together at the end.  The reduced operand is this rank's shifted train
    # Gram packed as its upper triangle (ocm_gram_pack about a zero shift:
    # p(p+1)/2 + p + 1 doubles, half of p²), so C and d = Σy/n come from
    # ocm_cov_from_packed and μ = shift + d, as ocm_cov_from_gram forms them.
    models = FoldModels()
    n_trs = [n_target - int(folds[f].size) for f in range(K)]
    if min(n_trs) < 2:
        raise ValueError("SIMCA needs at least 2 samples in a class")

    def gglobal(r):
        return dist.get_global_rank(group, r) if group is not None else r

    def solve(C, mean):
        evals, evecs, theta, _ = engine.eig_topk(C, lvmax, theta_mode)
        pack = torch.empty(lvmax + 3 + p + lvmax * p, dtype=torch.float64, device=dev)
        pack[:lvmax] = evals
        pack[lvmax:lvmax + 3] = theta
        pack[lvmax + 3:lvmax + 3 + p] = mean
        pack[lvmax + 3 + p:] = evecs.reshape(-1)
        return pack

    packs = [None] * K
    if distributed:
        zero32 = torch.zeros(p, dtype=torch.float32, device=dev)
        Gtr = torch.empty((p, p), dtype=torch.float64, device=dev)
        cs_tr = torch.empty(p, dtype=torch.float64, device=dev)
        n_loc_f = [int(f_.size) for f_ in loc_folds]
        n_loc_t = sum(n_loc_f)
        red, works = [], []
        for f in range(K):
            engine.gram_combine([(1.0, Gt, cst), (-1.0, G[f], cs[f])], Gtr, cs_tr)
            buf = engine.gram_pack(Gtr, cs_tr, zero32, n_loc_t - n_loc_f[f])
            red.append(buf)
            works.append(dist.reduce(buf, dst=gglobal(f % W), group=group, async_op=True))
        for w in works:
            w.wait()
        del Gtr, cs_tr
        shift64f = shift32.to(torch.float64)
        for f in range(R, K, W):
            C, d = engine.cov_from_packed(red[f], p)
            packs[f] = solve(C, d + shift64f)
            del C
        del red
        works = []
        for f in range(K):
            if packs[f] is None:
                packs[f] = torch.empty(lvmax + 3 + p + lvmax * p, dtype=torch.float64, device=dev)
            works.append(dist.broadcast(packs[f], src=gglobal(f % W), group=group, async_op=True))
        for w in works:
            w.wait()
    else:
        for f in range(K):
            C, mean = engine.cov_from_gram([(1.0, Gt, cst), (-1.0, G[f], cs[f])], shift32, n_trs[f])
            packs[f] = solve(C, mean)
            del C
    for f in range(K):
        n_tr = n_trs[f]
        pack = packs[f]
        evals = pack[:lvmax]
        models.evals.append(evals)
        models.mean.append(pack[lvmax + 3:lvmax + 3 + p])
        models.evecs.append(pack[lvmax + 3 + p:].view(lvmax, p))
        models.inv.append(_inv_evals(evals))
        host = pack[:lvmax + 3].cpu().numpy()
        models.evals_h.append(host[:lvmax])
        models.theta_h.append(host[lvmax:lvmax + 3])
        models.n_train.append(n_tr)
    del G, cs, Gt, packs

    # ---- per-fold scoring, limits, counts ----
    ncfg = len(combos) * len(lvs)
    counts = np.zeros((K, ncfg, 2, 4), dtype=np.int64)
    preds_fold = [] if store_predictions else None
    others_loc = _local(others, lo, hi)
    F_cache = {}
    for f in range(K):
        mean, evecs, inv = models.mean[f], models.evecs[f], models.inv[f]
        n_tr = models.n_train[f]
        # training-row statistics per LV (perc / chi2pom limits)
        tr_stats = None
        tr_arrays = None
        if need_train:
            tr_loc = np.concatenate([loc_folds[g] for g in range(K) if g != f]) if K > 1 else np.zeros(0, np.int64)
            if tr_loc.size:
                rows = torch.from_numpy(tr_loc).to(dev)
                sc = engine.score(Xd, rows, int(tr_loc.size), evecs, mean, inv, want_T=True, want_T2=False,
                                  want_Q=True)
                T2a, Qa, st = engine.cv_prefix(sc["T"], sc["Q"], inv, lvs, want_T2=need_pct, want_Q=need_pct,
                                               want_stats=True)
                del sc
            else:
                T2a = torch.zeros((len(lvs), 0), dtype=torch.float64, device=dev) if need_pct else None
                Qa = torch.zeros((len(lvs), 0), dtype=torch.float32, device=dev) if need_pct else None
                st = torch.zeros((len(lvs), 4), dtype=torch.float64, device=dev)
            if distributed:
                dist.all_reduce(st, group=group)
            tr_stats = st.cpu().numpy()
            tr_arrays = (T2a, Qa)

        # limits → decision configs (host fp64, utils/SIMCA.py:156-236)
        configs = []
        for s in specs:
            for li, lv in enumerate(lvs):
                th = _thetas_for(lv, lvmax, models.evals_h[f], models.theta_h[f])
                if tr_stats is not None:
                    T2a, Qa = tr_arrays
                    s1 = tr_stats[li]
                    T2m = limits.Moments(n_tr, s1[0], s1[1], _pct_fn(T2a, li, n_tr, group, distributed))
                    Qm = limits.Moments(n_tr, s1[2], s1[3], _pct_fn(Qa, li, n_tr, group, distributed))
                else:
                    T2m = Qm = limits.Moments(n_tr, 0.0, 0.0, None)
                key = (s.t2lim, s.t2cl, lv, n_tr)
                if s.t2lim in ("Fdist", "Fdistrig", "chi2") and key in F_cache:
                    t2l = F_cache[key]
                else:
                    t2l = limits.t2_limit(s, T2m, lv)
                    if s.t2lim in ("Fdist", "Fdistrig", "chi2"):
                        F_cache[key] = t2l
                ql = limits.q_limit(s, Qm, th)
                dl = limits.critic_distance(s, t2l, ql, th, lv)
                if s.type == "dd":
                    configs.append((lv, "dd", s._t2dof / s._t2scfact, s._qdof / s._qscfact, float(dl)))
                else:
                    configs.append((lv, s.type, 1.0 / t2l, 1.0 / ql, float(dl)))

        # held-out fold ∪ other-class rows, scored once at LV_max
        fold_loc = loc_folds[f]
        test_loc = np.concatenate([fold_loc, others_loc])
        m = int(test_loc.size)
        if m:
            rows = torch.from_numpy(test_loc).to(dev)
            pos = torch.from_numpy(positive_glob[test_loc + lo].astype(np.uint8)).to(dev)
            sc = engine.score(Xd, rows, m, evecs, mean, inv, want_T=True, want_T2=False, want_Q=True)
            cnt, acc = engine.cv_counts(sc["T"], sc["Q"], inv, pos, int(fold_loc.size), configs,
                                        want_accept=store_predictions)
            del sc
        else:
            cnt = torch.zeros((ncfg, 2, 4), dtype=torch.int64, device=dev)
            acc = torch.zeros((ncfg, 0), dtype=torch.float64, device=dev) if store_predictions else None
        if distributed:
            dist.all_reduce(cnt, group=group)
        counts[f] = cnt.cpu().numpy()
        if store_predictions:
            # the pooled vector (utils/CVSIMCA.py:190, 205-207): target rows
            # take their own fold's decision, other-class rows the last fold's
            keep = slice(0, int(fold_loc.size)) if f < K - 1 else slice(0, m)
            preds_fold.append((torch.from_numpy(test_loc[keep]).to(dev), acc[:, keep]))

    # ---- aggregation (utils/CVSIMCA.py:190-222) ----
    records, by_combo = [], []
    pred_all = None
    if store_predictions:
        pred_loc = torch.zeros((ncfg, n_loc), dtype=torch.float64, device=dev)
        for idx, acc in preds_fold:
            if idx.numel():
                pred_loc[:, idx] = acc
        if distributed:
            pred_all = _gather_blocks(pred_loc, lo, n_glob, group)
        elif lo == 0 and n_loc == n_glob:
            pred_all = pred_loc
        else:  # one process holding a row block: its columns of the (ncfg, n_glob) matrix
            pred_all = torch.zeros((ncfg, n_glob), dtype=torch.float64, device=dev)
            pred_all[:, lo:lo + n_loc] = pred_loc
        pred_all = pred_all.cpu().numpy()
    for ci_, combo in enumerate(combos):
        for li, lv in enumerate(lvs):
            c = ci_ * len(lvs) + li
            step_spec = np.zeros(K, dtype=float)
            for f in range(K):
                tot = counts[f, c, 0] + counts[f, c, 1]
                step_spec[f] = _rates(*tot)[1]
            pooled = counts[:, c, 0].sum(axis=0) + counts[K - 1, c, 1]
            sens = float(_rates(*pooled)[0])
            spec = float(np.mean(step_spec))
            records.append({"params": combo.copy(), "LV": lv, "spec": spec, "sens": sens,
                            "eff": float(np.sqrt(sens * spec))})
            if store_predictions:
                by_combo.append({"params": combo.copy(), "LV": lv, "prediction": pred_all[c].copy()})
    # keep the reference's record order: combos outer, LV in the given order
    if list(lv_values) != lvs:
        order = {lv: i for i, lv in enumerate(lvs)}
        per = len(lvs)
        recs, bys = [], []
        for ci_ in range(len(combos)):
            for lv in lv_values:
                recs.append(records[ci_ * per + order[int(lv)]])
                if store_predictions:
                    bys.append(by_combo[ci_ * per + order[int(lv)]])
        records, by_combo = recs, bys
    return records, by_combo


def _pct_fn(arr, li, n, group, distributed):
    if arr is None:
        return None

    def pct(q):
        v = arr[li]
        if distributed:
            from .dist import percentile_sharded

            return percentile_sharded(v, q, n, group)
        return engine.percentile(v, q)

    return pct


def _gather_blocks(block: torch.Tensor, lo: int, n_glob: int, group) -> torch.Tensor:
    """Every rank's (rows, n_loc) column block at global offset ``lo`` →
    the (rows, n_glob) matrix on every rank: one all-gather of the offsets and
    one of the blocks padded to the largest (device tensors; no host pickling)."""
    W = dist.get_world_size(group)
    dev = block.device
    meta = torch.tensor([lo, block.shape[1]], dtype=torch.int64, device=dev)
    metas = [torch.empty_like(meta) for _ in range(W)]
    dist.all_gather(metas, meta, group=group)
    metas = [m.cpu().tolist() for m in metas]
    width = max(n for _, n in metas)
    pad = torch.zeros((block.shape[0], width), dtype=block.dtype, device=dev)
    pad[:, :block.shape[1]] = block
    parts = [torch.empty_like(pad) for _ in range(W)]
    dist.all_gather(parts, pad, group=group)
    out = torch.zeros((block.shape[0], n_glob), dtype=block.dtype, device=dev)
    for (o, n), part in zip(metas, parts):
        out[:, o:o + n] = part[:, :n]
    return out
