"""Multi-rank logic of the row-sharded SIMCA (ocm/dist.py) on the CPU.

The libocm entry points are replaced by tests/fake_engine.py; what runs is
ocm.dist's own logic under torch.distributed ``gloo``: the distributed radix
select (histogram all-reduce per pass) against np.percentile, and
ShardedSIMCA's one-all-reduce fit (Gram / column sums / count / moments) and
local decisions at world size 2 against the single-process run.
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


def test_interp_matches_numpy():
    from ocm.dist import _interp

    rng = np.random.default_rng(0)
    for dt in (np.float64, np.float32):
        for n in (1, 2, 7, 1000, 1001):
            a = (rng.standard_normal(n) * 10).astype(dt)
            if n > 10:
                a[::7] = a[0]  # ties
            s = np.sort(a)
            for pct in (0, 5, 50, 95, 99.9, 100, 37.3):
                got = _interp(lambda r: s[r], n, pct, dt == np.float32)
                assert got == float(np.percentile(a, pct)), (dt, n, pct)


def test_fake_radix_select_single_rank():
    """The fake histogram pass implements the kernel's key / digit contract."""
    from ocm.dist import _interp, _key_to_value

    rng = np.random.default_rng(1)
    for dt in (np.float64, np.float32):
        a = np.concatenate([rng.standard_normal(500), -rng.standard_normal(300), [0.0, -0.0]]).astype(dt)
        t = torch.from_numpy(a)
        nbits = 64 if dt == np.float64 else 32

        def kth(rank):
            prefix = 0
            for shift in range(nbits - 8, -1, -8):
                c = np.cumsum(fake_engine.radix_hist(t, prefix, shift).numpy())
                dgt = int(np.searchsorted(c, rank, side="right"))
                rank -= int(c[dgt - 1]) if dgt > 0 else 0
                prefix |= dgt << shift
            return _key_to_value(prefix, 0 if dt == np.float64 else 1)

        for pct in (1, 50, 95):
            assert _interp(kth, a.size, pct, dt == np.float32) == float(np.percentile(a, pct))


def _pct_worker(rank, world, port, path, parts, pcts):
    import torch.distributed as dist

    import ocm.dist as od

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        od.engine = fake_engine
        v = torch.from_numpy(parts[rank])
        n = sum(p.size for p in parts)
        res = [od.percentile_sharded(v, q, n) for q in pcts]
        if rank == 0:
            np.save(path, np.array(res))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("dt", [np.float64, np.float32])
def test_percentile_sharded_gloo_world2(tmp_path, dt):
    rng = np.random.default_rng(2)
    a = (rng.gamma(2.0, 3.0, 2001)).astype(dt)
    a[100:140] = a[5]
    parts = [a[:700].copy(), a[700:].copy()]
    pcts = [0, 5, 50, 95, 99, 100]
    path = str(tmp_path / "p.npy")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_pct_worker, args=(r, 2, port, path, parts, pcts)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    got = np.load(path)
    np.testing.assert_array_equal(got, [float(np.percentile(a, q)) for q in pcts])


def _simca_worker(rank, world, port, path, X, bounds, cfg):
    import torch.distributed as dist

    import ocm.dist as od

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        od.engine = fake_engine
        lo, hi = bounds[rank]
        Xl = torch.from_numpy(X[lo:hi])
        m = od.ShardedSIMCA(n_components=4, **cfg).fit(Xl)
        acc = m.predict(Xl).numpy()
        got = [None] * world
        dist.all_gather_object(got, acc)
        if rank == 0:
            np.savez(path, T2=m.T2_limit, Q=m.Q_limit, D=float(m.D_limit), acc=np.concatenate(got))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cfg,p", [(dict(type="alt", t2lim="Fdist", qlim="jm"), 48),
                                   (dict(type="alt", t2lim="Fdist", qlim="jm"), 160),
                                   (dict(type="dd"), 48),
                                   (dict(type="ci", t2lim="perc", qlim="perc"), 48)])
def test_sharded_simca_gloo_world2_matches_single(tmp_path, cfg, p):
    """p = 160: three 64-column tiles, so the θ3 trace tiles are split
    between the ranks (ocm_eig_topk_ex slices) and summed by the all-reduce."""
    import ocm.dist as od
    from oracle import simca_oracle as O

    X = O.synth_spectra(1500, p, 4, rank=10, seed=3, outlier_frac=0.05)
    bounds = [(0, 640), (640, 1500)]
    path = str(tmp_path / "r.npz")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_simca_worker, args=(r, 2, port, path, X, bounds, cfg)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    got = np.load(path)
    saved = od.engine
    od.engine = fake_engine
    try:
        ref = od.ShardedSIMCA(n_components=4, **cfg).fit(torch.from_numpy(X))
        acc = ref.predict(torch.from_numpy(X)).numpy()
    finally:
        od.engine = saved
    np.testing.assert_allclose([got["T2"], got["Q"], got["D"]], [ref.T2_limit, ref.Q_limit, float(ref.D_limit)],
                               rtol=1e-9)
    np.testing.assert_array_equal(got["acc"], acc)


def test_sharded_simca_gloo_world4_with_empty_rank(tmp_path):
    """Four ranks (the θ3 trace tiles split four ways), one of them holding no
    rows, against the single-process run: the zero-row rank contributes zero
    moments to the one all-reduce and still scores its (empty) block."""
    import ocm.dist as od
    from oracle import simca_oracle as O

    cfg = dict(type="alt", t2lim="Fdist", qlim="jm")
    X = O.synth_spectra(1500, 160, 4, rank=10, seed=4, outlier_frac=0.05)
    bounds = [(0, 400), (400, 400), (400, 900), (900, 1500)]
    path = str(tmp_path / "r4.npz")
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=_simca_worker, args=(r, 4, port, path, X, bounds, cfg)) for r in range(4)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
        assert p.exitcode == 0
    got = np.load(path)
    saved = od.engine
    od.engine = fake_engine
    try:
        ref = od.ShardedSIMCA(n_components=4, **cfg).fit(torch.from_numpy(X))
        acc = ref.predict(torch.from_numpy(X)).numpy()
    finally:
        od.engine = saved
    np.testing.assert_allclose([got["T2"], got["Q"], got["D"]], [ref.T2_limit, ref.Q_limit, float(ref.D_limit)],
                               rtol=1e-9)
    np.testing.assert_array_equal(got["acc"], acc)
