"""Host / multi-rank logic of the CV fold engine (ocm/cv.py) on the CPU.

The device entry points are replaced by tests/fake_engine.py (exact NumPy
arithmetic with the same contracts), so what is tested here is the fold
engine's own logic: fold layout, Gram downdating, LV prefixes, limit
evaluation per (combo, LV, fold), count aggregation and the reference's
spec / pooled-sens rules, and the row-sharded multi-rank path over
torch.distributed ``gloo`` (world size 2) against the single-process run.
"""
import json
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import fake_engine
from oracle import simca_oracle as O


def _load(golden_dir, name):
    return dict(np.load(os.path.join(golden_dir, name), allow_pickle=False))


def _combos(grid):
    from sklearn.model_selection import ParameterGrid

    return list(ParameterGrid(grid))


BASE = dict(n_components=2, model_class=None, type="alt", t2lim="Fdist", t2cl=0.95, qlim="jm", qcl=0.95, dcl=0.95,
            maxPC=20, criteria="compl", verbose=False)


def _folds(y, n_splits):
    from sklearn.model_selection import KFold

    cls_idx = np.flatnonzero(y == 0)
    return cls_idx, [cls_idx[te] for _, te in KFold(n_splits=n_splits).split(cls_idx)]


def _run_fold_engine(X, y, n_splits, lvs, grid, row_offset=0, group=None, Xlocal=None):
    import ocm.cv as fe

    fe.engine = fake_engine
    cls_idx, folds = _folds(y, n_splits)
    return fe.cv_grid(X if Xlocal is None else Xlocal, y, folds, cls_idx, lvs, _combos(grid), BASE, [0], True,
                      row_offset=row_offset, group=group)


@pytest.fixture
def restore_engine():
    import ocm.cv as fe
    import ocm.engine as real

    yield
    fe.engine = real


@pytest.mark.parametrize("name", ["cv_a.npz", "cv_grid.npz"])
def test_fold_engine_logic_vs_oracle_and_reference(golden_dir, name, restore_engine):
    g = _load(golden_dir, name)
    grid = json.loads(str(g["param_grid_json"]))
    lvs = list(range(int(g["LV_min"]), int(g["LV_max"]) + 1))
    recs, by = _run_fold_engine(g["X"], g["y"], int(g["n_splits"]), lvs, grid)
    # reference goldens (record order, LV, metrics within 0.5 pp)
    assert [r["params"] for r in recs] == json.loads(str(g["params_json"]))
    np.testing.assert_array_equal([r["LV"] for r in recs], g["LV"])
    np.testing.assert_allclose([r["spec"] for r in recs], g["spec"], atol=0.5)
    np.testing.assert_allclose([r["sens"] for r in recs], g["sens"], atol=0.5)
    pred = np.stack([b["prediction"] for b in by]).astype(np.uint8)
    assert np.mean(pred != g["pred"]) <= 5e-3
    # oracle restatement of the refit loop (exact fp64 PCA per fold)
    o = O.cross_validate_simca_grid(g["X"], g["y"], 0, int(g["n_splits"]), int(g["LV_min"]), int(g["LV_max"]),
                                    cfg_grid=_combos(grid))
    np.testing.assert_allclose([r["spec"] for r in recs], [r["spec"] for r in o["results"]], atol=0.5)
    np.testing.assert_allclose([r["sens"] for r in recs], [r["sens"] for r in o["results"]], atol=0.5)


@pytest.mark.parametrize("grid", [
    {"type": ["ci", "sim"], "t2lim": ["chi2", "Fdistrig"], "qlim": ["chi2box"]},
    {"type": ["alt"], "t2lim": ["chi2pom"], "qlim": ["chi2pom", "jm"]},
    {"type": ["dd"]},
])
def test_fold_engine_limits_vs_oracle(golden_dir, grid, restore_engine):
    g = _load(golden_dir, "cv_a.npz")
    recs, _ = _run_fold_engine(g["X"], g["y"], 5, [2, 3, 4], grid)
    o = O.cross_validate_simca_grid(g["X"], g["y"], 0, 5, 2, 4, cfg_grid=_combos(grid))
    assert [r["params"] for r in recs] == [r["params"] for r in o["results"]]
    np.testing.assert_allclose([r["spec"] for r in recs], [r["spec"] for r in o["results"]], atol=0.5)
    np.testing.assert_allclose([r["sens"] for r in recs], [r["sens"] for r in o["results"]], atol=0.5)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, path, X, y, bounds, grid):
    import torch.distributed as dist

    import ocm.cv as fe
    import ocm.dist as od

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        fe.engine = fake_engine

        def pct_sharded(v, pct, n_total, group=None):  # all-gather stand-in for the radix select
            got = [None] * world
            dist.all_gather_object(got, v.numpy())
            return float(np.percentile(np.concatenate(got), pct))

        od.percentile_sharded = pct_sharded
        lo, hi = bounds[rank]
        recs, by = _run_fold_engine(X, y, 4, [2, 3, 4], grid, row_offset=lo, group=dist.group.WORLD,
                                    Xlocal=X[lo:hi])
        if rank == 0:
            np.savez(path, spec=[r["spec"] for r in recs], sens=[r["sens"] for r in recs],
                     pred=np.stack([b["prediction"] for b in by]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("grid", [{}, {"type": ["alt", "ci"], "t2lim": ["perc", "Fdist"], "qlim": ["perc", "jm"]}])
def test_fold_engine_gloo_world2_matches_single(golden_dir, tmp_path, grid, restore_engine):
    g = _load(golden_dir, "cv_a.npz")
    X, y = g["X"], g["y"]
    # uneven row blocks: a fold boundary and the other-class block straddle ranks
    bounds = [(0, 333), (333, X.shape[0])]
    path = str(tmp_path / "r0.npz")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, path, X, y, bounds, grid)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    got = np.load(path)
    recs, by = _run_fold_engine(X, y, 4, [2, 3, 4], grid)
    np.testing.assert_allclose(got["spec"], [r["spec"] for r in recs], atol=1e-9)
    np.testing.assert_allclose(got["sens"], [r["sens"] for r in recs], atol=1e-9)
    np.testing.assert_array_equal(got["pred"], np.stack([b["prediction"] for b in by]))


def test_generic_loop_accepts_tensor_predictions():
    """The drop-in's predict returns a (m, C) tensor for tensor inputs; the
    generic CV loop (utils/CVSIMCA.py) must pool it like the reference's
    NumPy arrays."""
    from utils.CVSIMCA import _fold_predictions

    class Est:
        def predict(self, X):
            return torch.ones((X.shape[0], 1), dtype=torch.float64)

    got = _fold_predictions(Est(), torch.zeros((5, 3)), np.zeros(5))
    assert isinstance(got, np.ndarray) and got.shape == (5,) and got.sum() == 5


def _grid_hook_worker(rank, world, port, path, X, y, grid):
    """Both ranks call the drop-in hook ocm.cv.grid with the FULL X, as
    utils.cross_validate_simca_grid does under torchrun."""
    import torch.distributed as dist

    import ocm.cv as fe
    import ocm.dist as od
    from utils.CVSIMCA import ClasswiseKFoldWithExternalVal
    from utils.SIMCA import SIMCA

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        fe.engine = fake_engine

        def pct_sharded(v, pct, n_total, group=None):
            got = [None] * world
            dist.all_gather_object(got, v.numpy(), group=group)
            return float(np.percentile(np.concatenate(got), pct))

        od.percentile_sharded = pct_sharded
        seen = []
        orig = fe.cv_grid

        def spy(*a, **k):
            seen.append((k.get("group") is not None, int(k.get("row_offset", 0)), int(a[0].shape[0])))
            return orig(*a, **k)

        fe.cv_grid = spy
        recs, by = fe.grid(SIMCA(verbose=False), X, y, ClasswiseKFoldWithExternalVal(n_splits=4, cls_label=0),
                           [2, 3, 4], grid, None, True)
        np.savez(path + f".{rank}.npz", spec=[r["spec"] for r in recs], sens=[r["sens"] for r in recs],
                 pred=np.stack([b["prediction"] for b in by]), seen=np.array(seen))
    finally:
        dist.destroy_process_group()


def test_dropin_hook_shards_under_world_group(golden_dir, tmp_path, restore_engine):
    """under an initialised world of two ranks the drop-in hook
    gives each rank its contiguous row block (group = WORLD) and both ranks get
    the single-process records; with no process group it runs on all rows."""
    import ocm.cv as fe
    from utils.CVSIMCA import ClasswiseKFoldWithExternalVal
    from utils.SIMCA import SIMCA

    g = _load(golden_dir, "cv_a.npz")
    X, y = g["X"], g["y"]
    grid = {"type": ["alt", "ci"], "t2lim": ["perc", "Fdist"], "qlim": ["perc", "jm"]}
    path = str(tmp_path / "hook")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_grid_hook_worker, args=(r, 2, port, path, X, y, grid)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    fe.engine = fake_engine
    recs, by = fe.grid(SIMCA(verbose=False), X, y, ClasswiseKFoldWithExternalVal(n_splits=4, cls_label=0),
                       [2, 3, 4], grid, None, True)
    n = X.shape[0]
    for r in range(2):
        got = np.load(path + f".{r}.npz")
        from ocm.synth import shard_bounds

        lo, hi = shard_bounds(n, r, 2)
        assert got["seen"].tolist() == [[1, lo, hi - lo]]
        np.testing.assert_allclose(got["spec"], [x["spec"] for x in recs], atol=1e-9)
        np.testing.assert_allclose(got["sens"], [x["sens"] for x in recs], atol=1e-9)
        np.testing.assert_array_equal(got["pred"], np.stack([b["prediction"] for b in by]))
