"""C5 data-parallel pieces on the CPU over torch.distributed ``gloo`` (world 2).

* The trainer's gradient averaging (one all-reduce of a flat gradient buffer,
  ocm/vae_train.py) gives the same parameters after N steps as a single
  process that runs each rank's half-batch with the same seeds, averages the
  two gradients and takes the Adam step — DDP's semantics (per-rank
  BatchNorm statistics), reference step vae_bce_nut.py:178-203.
* The latent statistics and the f-distance decision (utils/final_vaesimca.py:
  428-442, 500-533) over row shards equal the single-process result on the
  concatenated rows (global moments, Gram and percentiles).
* The synthetic shard generator (ocm/synth.py) gives the same global matrix
  for any world size.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

L, D, B, STEPS = 64, 4, 16, 3


def _model():
    import vae_model as V

    torch.manual_seed(7)
    return V.ConvVAE1D(L, D, torch.zeros(L), torch.ones(L), conv_blocks=2, n_filters=2, kernel_size=5, hidden_fc=8,
                       dropout=0.0)


def _batches():
    g = torch.Generator().manual_seed(11)
    return [torch.rand((2 * B, L), generator=g) for _ in range(STEPS)]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ddp_worker(rank, world, port, path):
    import torch.distributed as dist

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        from ocm.vae_train import GraphedVAETrainer

        m = _model()
        if rank == 1:  # different init on rank 1: the trainer broadcasts rank 0's state
            with torch.no_grad():
                for p in m.parameters():
                    p.add_(1.0)
        tr = GraphedVAETrainer(m, B, lr=1e-3, weight_decay=1e-4, dtype=torch.float32, graph=False)
        for s, xb in enumerate(_batches()):
            torch.manual_seed(100 * s + rank)  # ε of this rank's half
            tr.step(xb[rank * B:(rank + 1) * B])
        tr.sync_buffers()
        np.savez(f"{path}.{rank}.npz", **{k: v.detach().numpy() for k, v in m.state_dict().items()})
    finally:
        dist.destroy_process_group()


def test_grad_allreduce_matches_half_batch_average(tmp_path):
    import vae_model as V

    ctx = mp.get_context("spawn")
    port = _free_port()
    path = str(tmp_path / "ddp")
    procs = [ctx.Process(target=_ddp_worker, args=(r, 2, port, path)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    got = {r: dict(np.load(f"{path}.{r}.npz")) for r in range(2)}

    # single process: per-half forward/backward, averaged gradients, Adam
    m = _model()
    opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=1e-4, foreach=True)
    m.train()
    for s, xb in enumerate(_batches()):
        opt.zero_grad()
        for r in range(2):
            torch.manual_seed(100 * s + r)
            x = xb[r * B:(r + 1) * B]
            x_rec, mu, logvar = m(x)
            loss = V.bce_recon_term(x, x_rec) + V.kl_term(mu, logvar)
            (loss / 2).backward()
        opt.step()
    for name, v in m.named_parameters():
        for r in range(2):
            np.testing.assert_allclose(got[r][name], v.detach().numpy(), rtol=2e-5, atol=1e-6, err_msg=name)
    for k in got[0]:  # buffers identical across ranks after sync_buffers
        np.testing.assert_array_equal(got[0][k], got[1][k])


def _latent_worker(rank, world, port, path):
    import torch.distributed as dist

    import fake_engine
    import ocm.vae as vae

    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        import ocm.dist as od

        vae.engine = od.engine = fake_engine
        Z, qc, Zt, qt = _latent_data()
        lo, hi = (0, 130) if rank == 0 else (130, 300)
        tlo, thi = (0, 50) if rank == 0 else (50, 120)
        g = vae.latent_stats(Z[lo:hi], qc[lo:hi], group=dist.group.WORLD)
        acc, f, fcrit = vae.full_distance_decision(Zt[tlo:thi], g[0].to(torch.float32), qt[tlo:thi],
                                                   group=dist.group.WORLD)
        np.savez(f"{path}.{rank}.npz", mean=g[0].numpy(), inv=g[1].numpy(), t2=g[2], q=g[3], acc=acc.numpy(),
                 f=f.numpy(), fcrit=fcrit)
    finally:
        dist.destroy_process_group()


def _latent_data():
    g = torch.Generator().manual_seed(3)
    Z = torch.randn((300, 6), generator=g) * torch.linspace(0.5, 3, 6) + 2.0
    qc = torch.rand(300, generator=g) * 5
    Zt = torch.randn((120, 6), generator=g) * 2.0 + 2.0
    qt = torch.rand(120, generator=g) * 6
    return Z, qc.float(), Zt, qt.float()


def test_latent_stats_and_f_distance_over_shards(tmp_path, restore_vae_engine):
    import fake_engine
    import ocm.vae as vae

    ctx = mp.get_context("spawn")
    port = _free_port()
    path = str(tmp_path / "lat")
    procs = [ctx.Process(target=_latent_worker, args=(r, 2, port, path)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=180)
        assert p.exitcode == 0
    got = {r: dict(np.load(f"{path}.{r}.npz")) for r in range(2)}
    vae.engine = fake_engine
    Z, qc, Zt, qt = _latent_data()
    mean, inv, t2lim, qlim = vae.latent_stats(Z, qc)
    acc, f, fcrit = vae.full_distance_decision(Zt, mean.to(torch.float32), qt)
    for r in range(2):
        g = got[r]
        np.testing.assert_allclose(g["mean"], mean.numpy(), rtol=1e-12)
        np.testing.assert_allclose(g["inv"], inv.numpy(), rtol=1e-9)
        assert float(g["t2"]) == pytest.approx(t2lim, rel=1e-12) and float(g["q"]) == pytest.approx(qlim, rel=1e-6)
        assert float(g["fcrit"]) == pytest.approx(fcrit, rel=1e-10)
    np.testing.assert_allclose(np.concatenate([got[0]["f"], got[1]["f"]]), f.numpy(), rtol=1e-10)
    np.testing.assert_array_equal(np.concatenate([got[0]["acc"], got[1]["acc"]]), acc.numpy())


@pytest.fixture
def restore_vae_engine():
    import ocm.engine as real
    import ocm.vae as vae

    yield
    vae.engine = real


@pytest.mark.parametrize("world", [1, 3])
def test_synth_shards_are_world_size_independent(world):
    from ocm.synth import spectra_shard

    n, p = 70_000, 32  # two generator chunks
    ref = spectra_shard(n, p, 0, 1, torch.device("cpu"), seed=5, k=4, rank_count=8)
    parts = [spectra_shard(n, p, r, world, torch.device("cpu"), seed=5, k=4, rank_count=8) for r in range(world)]
    np.testing.assert_array_equal(torch.cat(parts).numpy(), ref.numpy())
    assert ref.shape == (n, p) and torch.isfinite(ref).all()
