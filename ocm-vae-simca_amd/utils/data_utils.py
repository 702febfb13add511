"""Drop-in for the reference's utils/data_utils.py (object-aware splits) plus
the drivers' data loaders.

``object_aware_splits`` keeps the reference's signature, returns and printed
messages (utils/data_utils.py:12-167).  Its arithmetic, the SNV +
Savitzky–Golay copy and the PCA-score Mahalanobis outlier screen
(:56-80), runs on the MI355X kernels (``ocm.preprocess``); the object
bookkeeping and sklearn ``train_test_split`` stay on the host, as in the
reference, so the object-level splits are the same.
"""
from __future__ import annotations

import numpy as np
from sklearn.model_selection import train_test_split

__all__ = ["object_aware_splits", "load_ir_ml_mat", "load_nut_objects_h5"]


def _outlier_keep(X_proc: np.ndarray, n_comp: int, outlier_percentile: float):
    """PCA(n_comp) score-space Mahalanobis screen (utils/data_utils.py:64-78) on
    the GPU: (keep mask, threshold)."""
    from ocm import preprocess

    mask, thr = preprocess.mahalanobis_outlier_mask(X_proc, n_comp, outlier_percentile)
    return mask.cpu().numpy(), thr


def _snv_savgol_copy(X: np.ndarray) -> np.ndarray:
    """SNV then savgol(5, 2, deriv 1) (utils/data_utils.py:57-61); when the
    filter cannot run (fewer than 5 wavelengths) the SNV copy is kept, as the
    reference's try/except does."""
    from ocm import preprocess

    try:
        out = preprocess.snv_savgol(X, 5, 2, 1)
    except ValueError:
        out = preprocess.snv(X)
    return out.cpu().numpy()


def object_aware_splits(data, nut_types, target_nut, n_wavelengths, cal_frac=0.7, val_frac=0.15, test_frac=0.15,
                        random_state=42, outlier_percentile=95, use_pca=True):
    """Split by objects so that spectra of one object never cross splits
    (utils/data_utils.py:12-167).  Returns (splits, Xts_data, Xts_label,
    X_cal, X_val, X_test_in, X_test_out)."""
    assert abs(cal_frac + val_frac + test_frac - 1.0) < 1e-6, "Fractions must sum to 1.0"

    def empty():
        return np.empty((0, n_wavelengths), dtype=np.float32)

    splits = {}
    for nut_type in nut_types:
        obj_spectra = [np.asarray(obj["spectral_data"], dtype=np.float32) for obj in data[nut_type]]
        if len(obj_spectra) == 0:
            print(f"  {nut_type}: no objects found, skipping")
            splits[nut_type] = {"cal": empty(), "val": empty(), "test": empty()}
            continue
        X_nut = np.vstack(obj_spectra)
        obj_ids = np.concatenate([np.full(s.shape[0], i, dtype=int) for i, s in enumerate(obj_spectra)])

        bad = np.isnan(X_nut).any(axis=1) | np.isinf(X_nut).any(axis=1)
        if np.any(bad):
            print(f"  WARNING: {nut_type}: Found {np.sum(bad)} NaN/inf samples. Removing them.")
            X_nut, obj_ids = X_nut[~bad], obj_ids[~bad]

        X_clean, obj_ids_clean = X_nut.copy(), obj_ids
        if use_pca and X_nut.shape[0] > 3 and X_nut.shape[0] > 1:
            n_comp = min(10, X_nut.shape[1], max(1, X_nut.shape[0] - 1))
            if X_nut.shape[0] > n_comp:
                keep, out_thr = _outlier_keep(_snv_savgol_copy(X_nut), n_comp, outlier_percentile)
                n_removed = int(np.sum(~keep))
                if n_removed > 0:
                    print(f"  {nut_type}: removed {n_removed} outliers (threshold {out_thr:.3f})")
                X_clean, obj_ids_clean = X_nut[keep], obj_ids[keep]
            else:
                print(f"  {nut_type}: not enough samples for PCA components, skipping outlier removal")

        objects_after = {}
        for idx in np.unique(obj_ids_clean):
            rows = X_clean[obj_ids_clean == idx]
            if rows.shape[0] > 0:
                objects_after[int(idx)] = rows
        if not objects_after:
            print(f"  {nut_type}: no objects remaining after cleaning, skipping")
            splits[nut_type] = {"cal": empty(), "val": empty(), "test": empty()}
            continue

        ids = list(objects_after.keys())
        if len(ids) >= 3:
            cal_objs, temp_objs = train_test_split(ids, test_size=1.0 - cal_frac, random_state=random_state)
            rel = test_frac / (val_frac + test_frac) if (val_frac + test_frac) > 0 else 0.5
            val_objs, test_objs = train_test_split(temp_objs, test_size=rel, random_state=random_state)
        elif len(ids) == 2:
            cal_objs, val_objs, test_objs = [ids[0]], [], [ids[1]]
        else:
            cal_objs, val_objs, test_objs = [ids[0]], [], []

        def stack(lst):
            return np.vstack([objects_after[i] for i in lst]) if lst else empty()

        Xc, Xv, Xt = stack(cal_objs), stack(val_objs), stack(test_objs)
        splits[nut_type] = {"cal": Xc, "val": Xv, "test": Xt}
        print(f"  {nut_type}: objects after cleaning={len(objects_after)}, raw samples after cleaning="
              f"{X_clean.shape[0]} -> cal={Xc.shape}, val={Xv.shape}, test={Xt.shape}")

    parts, labels = [], []
    for nut_type in nut_types:
        Xt = splits[nut_type]["test"]
        if Xt.shape[0] == 0:
            continue
        parts.append(Xt)
        labels.append(np.full(Xt.shape[0], 0 if nut_type == target_nut else 1, dtype=int))
    Xts_data = np.vstack(parts) if parts else empty()
    Xts_label = np.concatenate(labels) if labels else np.array([], dtype=int)
    others = [splits[n]["test"] for n in nut_types if n != target_nut and splits[n]["test"].shape[0] > 0]
    X_test_out = np.vstack(others) if others else empty()
    return (splits, Xts_data, Xts_label, splits[target_nut]["cal"], splits[target_nut]["val"],
            splits[target_nut]["test"], X_test_out)


def load_ir_ml_mat(path):
    """The cheese IR_ML.mat layout (simca_new_cheese.py:12-25): MATLAB structs
    Xtr / Xts with fields 'data' and 'class' (1-based).  Returns (Xtr_data,
    Xtr_label, Xts_data, Xts_label) with 0-based int labels."""
    from scipy.io import loadmat

    d = {k: v for k, v in loadmat(path).items() if not k.startswith("_")}

    def fields(s):
        return {key: s[0][0][i] for i, key in enumerate(s.dtype.names)}

    tr, ts = fields(d["Xtr"]), fields(d["Xts"])
    return (tr["data"], np.squeeze(tr["class"][0][0]).astype(int) - 1, ts["data"],
            np.squeeze(ts["class"][0][0]).astype(int) - 1)


def load_nut_objects_h5(path):
    """nut_objects.h5 (nut_data.py:147-185; read at vae_bce_nut.py:65-77):
    {nut}/img_{i}/obj_{j}/spectra float32 → {nut: [{'spectral_data', 'obj_idx',
    'img_idx'}]} in sorted key order.  Needs h5py."""
    try:
        import h5py
    except ImportError as e:  # not installed in every image
        raise ImportError("load_nut_objects_h5 needs h5py") from e
    data = {}
    with h5py.File(path, "r") as f:
        for nut in sorted(f.keys()):
            data[nut] = []
            for img in sorted(f[nut].keys()):
                for obj in sorted(f[nut][img].keys()):
                    g = f[nut][img][obj]
                    data[nut].append({"spectral_data": g["spectra"][()], "obj_idx": int(g.attrs.get("obj_idx", -1)),
                                      "img_idx": int(g.attrs.get("img_idx", -1))})
    return data
