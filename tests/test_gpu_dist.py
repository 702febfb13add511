"""The REAL engine under more than one rank (ocm/dist.py, ocm/cv.py), on the
one GPU of the box: two processes share cuda:0 and talk over ``gloo`` (RCCL
refuses two ranks on one device; the driver's 8-GPU run covers RCCL).  What
runs is the product path end to end — libocm kernels, the row-sharded Gram
all-reduce, the per-rank eigensolve, the sharded moments / radix-select
percentiles, the CV fold engine's reduce-to-owner Grams, model broadcasts and
device all-gathers — against the single-process run of the same engine.

Rank blocks are uneven and cut through i8×3 chunks and scale blocks, so the
digit representation (one power-of-two scale per 1536-row block of each
rank's rows) and the fp64 summation order differ from the single-process
run: the θ tail sums move by ~1e-7 relative (measured 3.5e-7 on Q_limit), so
limits are held to the parity tolerance rtol 1e-5 and at most
two boundary rows may flip.
"""
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs a HIP device")]

CFGS = [dict(type="alt", t2lim="Fdist", qlim="jm"), dict(type="dd"), dict(type="ci", t2lim="perc", qlim="perc")]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    from oracle import simca_oracle as O

    X = O.synth_spectra(9000, 256, 8, rank=24, seed=5, outlier_frac=0.05)
    return X, [(0, 3700), (3700, 9000)]


def _simca_worker(rank, world, port, path):
    import torch.distributed as dist

    from ocm.dist import ShardedSIMCA

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        X, bounds = _data()
        lo, hi = bounds[rank]
        Xl = torch.from_numpy(X[lo:hi]).cuda()
        out = {}
        for i, cfg in enumerate(CFGS):
            m = ShardedSIMCA(n_components=8, **cfg).fit(Xl)
            acc = m.predict(Xl).cpu()
            got = [torch.empty(0)] * world
            dist.all_gather_object(got, acc)
            out[f"lim{i}"] = np.array([m.T2_limit, m.Q_limit, float(m.D_limit)])
            out[f"acc{i}"] = torch.cat(got).numpy()
        if rank == 0:
            np.savez(path, **out)
    finally:
        dist.destroy_process_group()


def _spawn(target, path, world=2, timeout=240):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, path)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=timeout)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


def test_sharded_simca_two_ranks_real_engine(tmp_path):
    from ocm.dist import ShardedSIMCA

    path = str(tmp_path / "r.npz")
    _spawn(_simca_worker, path)
    got = np.load(path)
    X, _ = _data()
    Xd = torch.from_numpy(X).cuda()
    for i, cfg in enumerate(CFGS):
        ref = ShardedSIMCA(n_components=8, **cfg).fit(Xd)
        acc = ref.predict(Xd).cpu().numpy()
        np.testing.assert_allclose(got[f"lim{i}"], [ref.T2_limit, ref.Q_limit, float(ref.D_limit)], rtol=1e-5)
        diff = got[f"acc{i}"] != acc
        assert diff.sum() <= 2, (cfg, int(diff.sum()))  # rows on the decision boundary only


def _simca4_worker(rank, world, port, path):
    import torch.distributed as dist

    from ocm.dist import ShardedSIMCA

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        X, _ = _data()
        bounds = [(0, 2100), (2100, 2100), (2100, 5000), (5000, 9000)]
        lo, hi = bounds[rank]
        m = ShardedSIMCA(n_components=8, type="alt", t2lim="Fdist", qlim="jm").fit(torch.from_numpy(X[lo:hi]).cuda())
        acc = m.predict(torch.from_numpy(X[lo:hi]).cuda()).cpu()
        got = [torch.empty(0)] * world
        dist.all_gather_object(got, acc)
        if rank == 0:
            np.savez(path, lim=np.array([m.T2_limit, m.Q_limit, float(m.D_limit)]), acc=torch.cat(got).numpy())
    finally:
        dist.destroy_process_group()


def test_sharded_simca_four_ranks_with_empty_rank(tmp_path):
    """Four ranks on the one GPU (θ3 trace split four ways, one rank without
    rows) against the single-process run of the real engine."""
    from ocm.dist import ShardedSIMCA

    path = str(tmp_path / "r4.npz")
    _spawn(_simca4_worker, path, world=4, timeout=300)
    got = np.load(path)
    X, _ = _data()
    Xd = torch.from_numpy(X).cuda()
    ref = ShardedSIMCA(n_components=8, type="alt", t2lim="Fdist", qlim="jm").fit(Xd)
    acc = ref.predict(Xd).cpu().numpy()
    np.testing.assert_allclose(got["lim"], [ref.T2_limit, ref.Q_limit, float(ref.D_limit)], rtol=1e-5)
    assert (got["acc"] != acc).sum() <= 2


def _offset_data():
    """spectra on a large baseline with small variance (μ ≈ 1e3,
    tail λ ≈ 1e-6): each rank's moments are packed about ONE all-reduced
    shift, so nothing of size |μ|² cancels in the covariance."""
    X, bounds = _data()
    return (X.astype(np.float64) * 1e-2 + 1e3).astype(np.float32), bounds


def _simca_offset_worker(rank, world, port, path):
    import torch.distributed as dist

    from ocm.dist import ShardedSIMCA

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        X, bounds = _offset_data()
        lo, hi = bounds[rank]
        m = ShardedSIMCA(n_components=8, type="alt", t2lim="Fdist", qlim="jm").fit(torch.from_numpy(X[lo:hi]).cuda())
        if rank == 0:
            np.savez(path, lim=np.array([m.T2_limit, m.Q_limit, float(m.D_limit)]))
    finally:
        dist.destroy_process_group()


def test_sharded_simca_large_offset(tmp_path):
    """Two ranks on offset spectra == the single-process fit, and the jm Q limit
    == the fp64 oracle's (θ1..θ3 of the tail eigenvalues survive the offset)."""
    from ocm.dist import ShardedSIMCA

    path = str(tmp_path / "off.npz")
    _spawn(_simca_offset_worker, path)
    got = np.load(path)["lim"]
    X, _ = _offset_data()
    ref = ShardedSIMCA(n_components=8, type="alt", t2lim="Fdist", qlim="jm").fit(torch.from_numpy(X).cuda())
    np.testing.assert_allclose(got, [ref.T2_limit, ref.Q_limit, float(ref.D_limit)], rtol=1e-5)
    Xc = X.astype(np.float64) - X.astype(np.float64).mean(0)
    lam = np.linalg.eigvalsh(Xc.T @ Xc / (X.shape[0] - 1))[::-1]
    tail = lam[8:]
    th = (tail.sum(), (tail ** 2).sum(), (tail ** 3).sum())
    h0 = 1 - 2 * th[0] * th[2] / (3 * th[1] ** 2)
    from scipy.special import erfinv
    ca = np.sqrt(2) * erfinv(2 * 0.95 - 1)
    q_ref = th[0] * (ca * np.sqrt(2 * th[1] * h0 ** 2) / th[0] + 1 + th[1] * h0 * (h0 - 1) / th[0] ** 2) ** (1 / h0)
    np.testing.assert_allclose(got[1], q_ref, rtol=1e-4)


def _cv_worker(rank, world, port, path):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        res = _cv_run(rank, world)
        if rank == 0:
            np.savez(path, **res)
    finally:
        dist.destroy_process_group()


def _cv_run(rank=0, world=1):
    """The fold engine (ocm.cv.cv_grid, real libocm) on this rank's contiguous
    row block; the block boundary cuts through a fold and the other-class rows."""
    from sklearn.model_selection import KFold

    import ocm.cv as fe
    from oracle import simca_oracle as O

    X0 = O.synth_spectra(2400, 256, 8, rank=24, seed=21)
    X1 = O.synth_spectra(600, 256, 8, rank=24, seed=22, outlier_frac=1.0)
    X = np.concatenate([X0, X1]).astype(np.float32)
    y = np.concatenate([np.zeros(2400, np.int64), np.ones(600, np.int64)])
    cls_idx = np.flatnonzero(y == 0)
    folds = [cls_idx[te] for _, te in KFold(n_splits=5).split(cls_idx)]
    cuts = [0, 1333, 3000] if world == 2 else [0, 3000]
    lo, hi = cuts[rank], cuts[rank + 1]
    combos = [{"type": "alt", "t2lim": "Fdist", "qlim": "jm"}, {"type": "ci", "t2lim": "perc", "qlim": "chi2pom"}]
    base = dict(n_components=2, model_class=None, type="alt", t2lim="Fdist", t2cl=0.95, qlim="jm", qcl=0.95,
                dcl=0.95, maxPC=20, criteria="compl", verbose=False)
    import torch.distributed as dist

    recs, by = fe.cv_grid(torch.from_numpy(X[lo:hi]).cuda(), y, folds, cls_idx, [6, 7, 8], combos, base, [0], True,
                          row_offset=lo, group=dist.group.WORLD if world > 1 else None)
    return {"spec": np.array([r["spec"] for r in recs]), "sens": np.array([r["sens"] for r in recs]),
            "pred": np.stack([np.asarray(b["prediction"]) for b in by])}


def test_cv_fold_engine_two_ranks_real_engine(tmp_path):
    path = str(tmp_path / "cv.npz")
    _spawn(_cv_worker, path)
    got = np.load(path)
    ref = _cv_run()
    np.testing.assert_allclose(got["spec"], ref["spec"], atol=1e-9)
    np.testing.assert_allclose(got["sens"], ref["sens"], atol=1e-9)
    diff = got["pred"] != ref["pred"]
    assert diff.sum() <= 2, int(diff.sum())


def _cv_dropin_data():
    from oracle import simca_oracle as O

    X0 = O.synth_spectra(2400, 256, 8, rank=24, seed=21)
    X1 = O.synth_spectra(600, 256, 8, rank=24, seed=22, outlier_frac=1.0)
    X = np.concatenate([X0, X1]).astype(np.float32)
    y = np.concatenate([np.zeros(2400, np.int64), np.ones(600, np.int64)])
    return X, y


CV_GRID = {"type": ["alt", "ci"], "t2lim": ["Fdist", "perc"], "qlim": ["jm", "perc"]}


def _cv_dropin_run():
    """The reference entry point, unchanged: utils.cross_validate_simca_grid on
    the FULL X (utils/CVSIMCA.py:103-269).  Returns its records and pooled
    predictions plus the ``group`` the fold engine was called with."""
    import contextlib
    import io

    import ocm.cv as fe
    from utils import SIMCA, ClasswiseKFoldWithExternalVal, cross_validate_simca_grid

    X, y = _cv_dropin_data()
    seen = []
    orig = fe.cv_grid

    def spy(*a, **k):
        seen.append((k.get("group") is not None, int(k.get("row_offset", 0)), int(a[0].shape[0])))
        return orig(*a, **k)

    fe.cv_grid = spy
    try:
        with contextlib.redirect_stdout(io.StringIO()):
            res = cross_validate_simca_grid(SIMCA(verbose=False), X, y, ClasswiseKFoldWithExternalVal(n_splits=5,
                                            cls_label=0), LV_min=6, LV_max=8, param_grid=CV_GRID,
                                            print_summary=False, store_predictions=True)
    finally:
        fe.cv_grid = orig
    recs = res["results"]
    return {"spec": np.array([r["spec"] for r in recs]), "sens": np.array([r["sens"] for r in recs]),
            "pred": np.stack([np.asarray(b["prediction"]) for b in res["by_combo"]]),
            "best_lv": np.array(res["best_LV"]), "seen": np.array(seen, dtype=np.int64)}


def _cv_dropin_worker(rank, world, port, path):
    import os

    import torch.distributed as dist

    import vae_model as V

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        res = _cv_dropin_run()
        # compute_q_h_f under an initialised group stays per batch
        # (vae_model.py:162-182): every rank gets the reference's numbers
        g = dict(np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "qhf.npz")))
        q, h, f, qc, hc, fc = V.compute_q_h_f(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["x_rec"]).cuda(),
                                              torch.from_numpy(g["z"]).cuda())
        res.update(q=q.cpu().numpy(), h=h.cpu().numpy(), f=f.cpu().numpy(), crit=np.array([qc, hc, fc]))
        np.savez(path + f".{rank}.npz", **res)
    finally:
        dist.destroy_process_group()


def test_cv_dropin_under_process_group_shards_and_matches(tmp_path, golden_dir):
    """an unchanged driver under torchrun (two ranks, each
    calling utils.cross_validate_simca_grid on the full X, a perc combo
    included) runs the fold engine row-sharded — each rank on its contiguous
    block, group = WORLD — and both ranks return the single-process records
    and pooled predictions; compute_q_h_f under the same group equals the
    reference fixture (qhf.npz) on every rank."""
    path = str(tmp_path / "dropin")
    _spawn(_cv_dropin_worker, path)
    ref = _cv_dropin_run()
    assert ref["seen"].tolist() == [[0, 0, 3000]]  # one process: no group, all rows
    g = np.load(f"{golden_dir}/qhf.npz")
    for r in range(2):
        got = np.load(path + f".{r}.npz")
        assert got["seen"].tolist() == [[1, [0, 1500][r], 1500]], got["seen"]
        np.testing.assert_allclose(got["spec"], ref["spec"], atol=1e-9)
        np.testing.assert_allclose(got["sens"], ref["sens"], atol=1e-9)
        diff = got["pred"] != ref["pred"]
        # the sharded fold Grams sum in another order: at most two boundary
        # flips over all 24 records' pooled predictions
        print("pooled prediction flips:", int(diff.sum()), "rows:", np.flatnonzero(diff.any(0)).tolist())
        assert diff.sum() <= 2, int(diff.sum())
        assert int(got["best_lv"]) == int(ref["best_lv"])
        np.testing.assert_allclose(got["q"], g["q"], rtol=1e-5)
        np.testing.assert_allclose(got["h"], g["h"], rtol=1e-4, atol=1e-6)
        np.testing.assert_allclose(got["f"], g["f"], rtol=1e-4)
        np.testing.assert_allclose(got["crit"], g["crit"], rtol=1e-4)


def _dropin_data(seed):
    from oracle import simca_oracle as O

    X = O.synth_spectra(9000, 256, 8, rank=24, seed=seed, outlier_frac=0.05)
    y = (np.random.default_rng(seed).random(9000) < 0.2).astype(np.int64)  # other-class rows interleaved
    return X, y


DROPIN_CFGS = [dict(type="alt", t2lim="Fdist", qlim="jm"), dict(type="ci", t2lim="perc", qlim="perc")]


def _dropin_simca(X, y, cfg):
    """An unchanged driver's calls (simca_nuts.py:186-189): fit, predict, transform."""
    from utils import SIMCA

    m = SIMCA(n_components=8, model_class=0, verbose=False, **cfg).fit(X, y)
    pred = m.predict(X)
    t2, t2r, q, qr = m.transform(X)
    info = m._model[0]
    return {"lim": np.array([info["T2_limit"], info["Q_limit"], float(info["D_limit"])]), "T2": info["T2"],
            "Q": info["Q"], "T": info["T"], "pred": np.asarray(pred), "tr_t2": t2, "tr_q": q,
            "sharded": np.array(getattr(m, "_sharded", False))}


def _dropin_simca_worker(rank, world, port, path):
    import torch.distributed as dist

    torch.cuda.set_device(0)
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        out = {}
        for tag, seed in (("same", 31), ("own", 40 + rank)):  # replicated data, then per-rank data
            X, y = _dropin_data(seed)
            for i, cfg in enumerate(DROPIN_CFGS):
                for key, v in _dropin_simca(X, y, cfg).items():
                    out[f"{tag}_{key}{i}"] = v
        np.savez(f"{path}.{rank}.npz", **out)
    finally:
        dist.destroy_process_group()


def test_simca_dropin_under_process_group(tmp_path):
    """an unchanged ``SIMCA(...).fit(X, y); predict(X);
    transform(X)`` on both ranks of a world-2 group.  With the same X and y it
    runs row-sharded (one packed all-reduce, per-row arrays all-gathered) and
    equals the single-process run (limits rtol 1e-5, T² / Q rtol 1e-4, at most
    two boundary rows); with different X per rank each rank gets exactly its
    own single-process result (utils/SIMCA.py:27-154 is per process)."""
    path = str(tmp_path / "dropin_simca")
    _spawn(_dropin_simca_worker, path)
    for r in range(2):
        got = np.load(f"{path}.{r}.npz")
        for tag, seed, sharded in (("same", 31, True), ("own", 40 + r, False)):
            X, y = _dropin_data(seed)
            for i, cfg in enumerate(DROPIN_CFGS):
                ref = _dropin_simca(X, y, cfg)
                assert bool(got[f"{tag}_sharded{i}"]) == sharded, (tag, r)
                # per-rank data: the same single-process computation in another process
                tol = dict(rtol=1e-5) if sharded else dict(rtol=1e-9)
                np.testing.assert_allclose(got[f"{tag}_lim{i}"], ref["lim"], **tol)
                tol = dict(rtol=1e-4, atol=1e-6) if sharded else dict(rtol=1e-9, atol=1e-12)
                for key in ("T2", "Q", "tr_t2", "tr_q"):
                    np.testing.assert_allclose(got[f"{tag}_{key}{i}"], ref[key], **tol, err_msg=f"{tag} {key} {cfg}")
                np.testing.assert_allclose(np.abs(got[f"{tag}_T{i}"]), np.abs(ref["T"]), rtol=1e-3, atol=1e-3)
                diff = got[f"{tag}_pred{i}"] != ref["pred"]
                assert diff.sum() <= (2 if sharded else 0), (tag, cfg, int(diff.sum()))


def test_cv_engine_over_rccl_world1():
    """The nccl branches of the distributed CV fold engine on a real RCCL
    group (one rank: the box has one GPU) equal the engine without a group."""
    import json
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "nccl_world1_worker.py")], capture_output=True, text=True,
                       timeout=240, cwd=os.path.dirname(here))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["backend"] == "nccl"
    # the distributed path packs the train moments about a zero shift and
    # rebuilds C from the packed triangle (a different fp64 summation than the
    # one-process path): rows on the decision boundary may flip
    np.testing.assert_allclose(res["spec"], res["spec_ref"], atol=0.2)
    np.testing.assert_allclose(res["sens"], res["sens_ref"], atol=0.2)
    assert res["pred_diff"] <= 3
