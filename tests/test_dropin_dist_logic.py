"""Multi-rank routing of the reference entry points on the CPU (gloo, world 2).

``utils.SIMCA`` fit / predict / transform and ``cross_validate_simca_grid``
called unchanged on every rank (as a driver under torchrun does,
simca_nuts.py:186-189):
* with the SAME X and labels on both ranks they run row-sharded (each rank its
  contiguous block, one all-reduce of the moments, per-row arrays all-gathered)
  and every rank returns the single-process result;
* with DIFFERENT X per rank each rank gets its own single-process result
  (the reference's per-process behaviour, utils/SIMCA.py:27-154,
  utils/CVSIMCA.py:103-269);
* inside ``ocm.replica.per_process()`` nothing is collective (a call made on
  one rank only returns).

The device entry points are replaced by tests/fake_engine.py (exact NumPy
arithmetic); the GPU suite runs the same routing on the real engine
(tests/test_gpu_dist.py).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

import fake_engine


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data(seed):
    from oracle import simca_oracle as O

    X = O.synth_spectra(1300, 48, 4, rank=10, seed=seed, outlier_frac=0.05)
    y = (np.random.default_rng(seed).random(1300) < 0.3).astype(np.int64)  # class 1 rows interleaved
    return X, y


CFG = [dict(type="alt", t2lim="Fdist", qlim="jm"), dict(type="ci", t2lim="perc", qlim="perc"), dict(type="dd")]


def _run(X, y, cfg):
    from utils.SIMCA import SIMCA

    m = SIMCA(n_components=4, model_class=0, verbose=False, **cfg).fit(X, y)
    pred = m.predict(X, y_true=y)
    t2, t2r, q, qr = m.transform(X)
    info = m._model[0]
    return {"lim": np.array([info["T2_limit"], info["Q_limit"], float(info["D_limit"])]), "T": info["T"],
            "T2": info["T2"], "Q": info["Q"], "T2red": info["T2red"], "pred": np.asarray(pred),
            "tr_t2": np.asarray(t2), "tr_q": np.asarray(q), "tr_qr": np.asarray(qr),
            "spec": np.array(m.metrics[0]["specificity"]), "sharded": np.array(getattr(m, "_sharded", False))}


def _simca_module():
    import sys

    import utils.SIMCA  # noqa: F401  (the package re-exports the class under the same name)

    return sys.modules["utils.SIMCA"]


def _patch():
    import ocm.dist as od

    _simca_module().engine = fake_engine
    od.engine = fake_engine


def _worker(rank, world, port, path, same):
    import torch.distributed as dist

    from ocm.replica import per_process

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        _patch()
        X, y = _data(7 if same else 7 + rank)
        out = {}
        for i, cfg in enumerate(CFG):
            for key, v in _run(X, y, cfg).items():
                out[f"{key}{i}"] = v
        if rank == 0:  # a call made on one rank only: no collective inside per_process()
            with per_process():
                out["solo"] = _run(X, y, CFG[0])["lim"]
        np.savez(f"{path}.{rank}.npz", **out)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def _spawn(path, same, world=2):
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, path, same)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.exitcode is None:
            p.kill()
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]


@pytest.fixture
def restore():
    import ocm.dist as od
    import ocm.engine as real

    yield
    _simca_module().engine = real
    od.engine = real


@pytest.mark.parametrize("same", [True, False], ids=["replicated", "per_rank_data"])
def test_simca_dropin_routing_gloo_world2(tmp_path, same, restore):
    path = str(tmp_path / "r")
    _spawn(path, same)
    _patch()
    for r in range(2):
        got = np.load(f"{path}.{r}.npz")
        X, y = _data(7 if same else 7 + r)
        for i, cfg in enumerate(CFG):
            ref = _run(X, y, cfg)
            assert bool(got[f"sharded{i}"]) == same
            assert not bool(ref["sharded"])
            np.testing.assert_allclose(got[f"lim{i}"], ref["lim"], rtol=1e-9, err_msg=str(cfg))
            for key in ("T2", "Q", "T2red", "tr_t2", "tr_q", "tr_qr"):
                np.testing.assert_allclose(got[f"{key}{i}"], ref[key], rtol=1e-9, atol=1e-12, err_msg=key)
            np.testing.assert_allclose(np.abs(got[f"T{i}"]), np.abs(ref["T"]), rtol=1e-7, atol=1e-9)
            np.testing.assert_array_equal(got[f"pred{i}"], ref["pred"])
            np.testing.assert_allclose(got[f"spec{i}"], ref["spec"], rtol=1e-12)
        if r == 0:
            np.testing.assert_allclose(got["solo"], _run(X, y, CFG[0])["lim"], rtol=1e-12)


def _cv_worker(rank, world, port, path):
    """Ranks holding different spectra call the CV drop-in: per-process CV."""
    import torch.distributed as dist

    import ocm.cv as fe
    from utils.CVSIMCA import ClasswiseKFoldWithExternalVal
    from utils.SIMCA import SIMCA

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        fe.engine = fake_engine
        X, y = _data(11 + rank)
        seen = []
        orig = fe.cv_grid

        def spy(*a, **k):
            seen.append((k.get("group") is not None, int(k.get("row_offset", 0)), int(a[0].shape[0])))
            return orig(*a, **k)

        fe.cv_grid = spy
        recs, _ = fe.grid(SIMCA(verbose=False), X, y, ClasswiseKFoldWithExternalVal(n_splits=4, cls_label=0),
                          [2, 3], {"type": ["alt"]}, None, False)
        np.savez(f"{path}.{rank}.npz", spec=[x["spec"] for x in recs], sens=[x["sens"] for x in recs],
                 seen=np.array(seen))
    finally:
        dist.destroy_process_group()


def test_cv_dropin_per_rank_data_runs_per_process(tmp_path, restore):
    import ocm.cv as fe
    from utils.CVSIMCA import ClasswiseKFoldWithExternalVal
    from utils.SIMCA import SIMCA

    path = str(tmp_path / "cv")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_cv_worker, args=(r, 2, port, path)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    try:
        fe.engine = fake_engine
        for r in range(2):
            got = np.load(f"{path}.{r}.npz")
            X, y = _data(11 + r)
            assert got["seen"].tolist() == [[0, 0, X.shape[0]]]  # no group, all of this rank's rows
            recs, _ = fe.grid(SIMCA(verbose=False), X, y, ClasswiseKFoldWithExternalVal(n_splits=4, cls_label=0),
                              [2, 3], {"type": ["alt"]}, None, False)
            np.testing.assert_allclose(got["spec"], [x["spec"] for x in recs], rtol=1e-12)
            np.testing.assert_allclose(got["sens"], [x["sens"] for x in recs], rtol=1e-12)
    finally:
        import ocm.engine as real

        fe.engine = real


def test_fingerprint_separates_inputs():
    from ocm.replica import fingerprint

    X, y = _data(3)
    a = fingerprint(X, y)
    assert (a == fingerprint(X.copy(), y.copy())).all()
    assert (a == fingerprint(torch.from_numpy(X), torch.from_numpy(y))).all()
    X2 = X.copy()
    X2[0, 0] += 1.0
    assert (a != fingerprint(X2, y)).any()
    y2 = y.copy()
    y2[-1] ^= 1
    assert (a != fingerprint(X, y2)).any()
    assert (a != fingerprint(X.astype(np.float64), y)).any()
    assert fingerprint(X, y, eligible=False)[0] == 0
