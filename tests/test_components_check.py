"""n_components above min(n_samples, n_features): the reference fits
PCA(n_components) on every class (utils/SIMCA.py:73) and, in its CV, on every
fold's training rows LV by LV (utils/CVSIMCA.py:158-185), so sklearn raises
ValueError there.  The drop-ins raise the same message before any device work
(CPU: the device entry points are tests/fake_engine.py)."""
import sys

import numpy as np
import pytest
from sklearn.decomposition import PCA

import fake_engine


@pytest.fixture
def fake():
    import ocm.cv as ocv
    import ocm.engine as real
    import utils.SIMCA  # noqa: F401

    mod = sys.modules["utils.SIMCA"]
    mod.engine, ocv.engine = fake_engine, fake_engine
    yield
    mod.engine, ocv.engine = real, real


def _sklearn_msg(k, X):
    with pytest.raises(ValueError) as e:
        PCA(k).fit(X)
    return str(e.value)


def _data(n_cls, n_other, p=24, seed=0):
    rng = np.random.default_rng(seed)
    X = rng.standard_normal((n_cls + n_other, p)).astype(np.float32)
    y = np.r_[np.zeros(n_cls, np.int64), np.ones(n_other, np.int64)]
    return X, y


def test_simca_fit_k_above_class_rows(fake):
    from utils.SIMCA import SIMCA

    X, y = _data(5, 30)
    want = _sklearn_msg(8, X[y == 0])
    with pytest.raises(ValueError) as e:
        SIMCA(n_components=8, model_class=0, verbose=False).fit(X, y)
    assert str(e.value) == want


def test_simca_fit_k_above_features(fake):
    from utils.SIMCA import SIMCA

    X, y = _data(60, 10, p=6)
    want = _sklearn_msg(7, X[y == 0])
    with pytest.raises(ValueError) as e:
        SIMCA(n_components=7, model_class=0, verbose=False).fit(X, y)
    assert str(e.value) == want


def test_cv_lv_above_fold_training_rows(fake):
    """12 class rows in 3 folds: 8 training rows per fold, so LV 9 is the first
    of LV 2..10 the reference's fold fit rejects (its first fold, same message)."""
    from utils.CVSIMCA import ClasswiseKFoldWithExternalVal, cross_validate_simca_grid
    from utils.SIMCA import SIMCA

    X, y = _data(12, 10)
    cv = ClasswiseKFoldWithExternalVal(n_splits=3, cls_label=0)
    train0 = next(iter(cv.split(X, y)))[0]
    want = _sklearn_msg(9, X[train0][y[train0] == 0])
    with pytest.raises(ValueError) as e:
        cross_validate_simca_grid(SIMCA(model_class=0, verbose=False), X, y, cv, LV_min=2, LV_max=10,
                                  print_summary=False)
    assert str(e.value) == want


@pytest.mark.parametrize("n,p,k", [(5, 24, 8), (300, 24, 25), (40, 24, 30), (2000, 1500, 1600), (600, 2048, 700)])
def test_message_matches_sklearn_solver_choice(n, p, k):
    """The solver sklearn names (svd_solver='auto' → 'covariance_eigh' for tall,
    narrow matrices, else 'full') for shapes on both sides of its rule."""
    from utils.SIMCA import check_components

    X = np.random.default_rng(1).standard_normal((n, p)).astype(np.float32)
    want = _sklearn_msg(k, X)
    with pytest.raises(ValueError) as e:
        check_components(k, n, p)
    assert str(e.value) == want
