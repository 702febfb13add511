"""The VAE trainer's step (ocm/vae_train.py, eager mode on the CPU) equals the
reference's training step (forward → beta_vae_bce_loss → zero_grad →
backward → Adam.step, vae_bce_nut.py:178-203) run with the reference-format
loss on an identical copy of the model."""
import copy
import os

import numpy as np
import pytest
import torch

import vae_model as V


@pytest.mark.parametrize("loss", ["bce", "cosine"])
def test_trainer_step_matches_reference_step(loss):
    from ocm.vae_train import GraphedVAETrainer

    L, d, B = 64, 4, 16
    g = torch.Generator().manual_seed(0)
    x = 1.0 + 0.3 * torch.randn(B, L, generator=g)
    torch.manual_seed(0)
    m1 = V.ConvVAE1D(L, d, np.zeros(L, np.float32), np.ones(L, np.float32), conv_blocks=2, n_filters=2,
                     kernel_size=5, hidden_fc=16)
    m2 = copy.deepcopy(m1)
    tr = GraphedVAETrainer(m1, B, lr=1e-3, weight_decay=1e-4, beta=0.7, loss=loss, dtype=torch.float32, graph=False)
    opt = torch.optim.Adam(m2.parameters(), lr=1e-3, weight_decay=1e-4)
    fn = V.beta_vae_bce_loss if loss == "bce" else V.beta_vae_cosine_loss
    for it in range(3):
        torch.manual_seed(100 + it)
        total, recon, kl = tr.step(x)
        m2.train()
        torch.manual_seed(100 + it)
        x_rec, mu, logvar = m2(x)
        ref_total, ref_recon, ref_kl = fn(x, x_rec, mu, logvar, beta=0.7)
        opt.zero_grad()
        ref_total.backward()
        opt.step()
        np.testing.assert_allclose([float(total), float(recon), float(kl)], [float(ref_total), ref_recon, ref_kl],
                                   rtol=1e-6)
    for (n1, p1), (n2, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        torch.testing.assert_close(p1, p2, rtol=1e-6, atol=1e-7, msg=n1)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_graph_step_trains_like_eager(dtype):
    """HIP-graph replays start from the initial weights (the capture warm-up is
    undone) and train like the eager step: finite, decreasing losses whose
    tail mean matches the eager run's (ε differs between the two generators,
    so trajectories agree statistically, not bitwise)."""
    from ocm.vae_train import GraphedVAETrainer

    dev = torch.device("cuda", 0)
    L, d, B = 256, 8, 128
    g = torch.Generator(device="cpu").manual_seed(0)
    X = (1.0 + 0.3 * torch.randn(B * 8, L, generator=g)).to(dev)
    mean, std = X.mean(0).cpu().numpy(), X.std(0).cpu().numpy()
    torch.manual_seed(0)
    m1 = V.ConvVAE1D(L, d, mean, std, conv_blocks=2, n_filters=3, kernel_size=5, hidden_fc=32).to(dev)
    m2 = copy.deepcopy(m1)
    sd0 = {k: v.clone() for k, v in m1.state_dict().items()}
    tg = GraphedVAETrainer(m1, B, lr=1e-3, dtype=dtype, graph=True)
    for k, v in m1.state_dict().items():  # capture left the model at its initial state
        torch.testing.assert_close(v, sd0[k], rtol=0, atol=0, msg=k)
    te = GraphedVAETrainer(m2, B, lr=1e-3, dtype=dtype, graph=False)
    lg, le = [], []
    for i in range(60):
        xb = X[(i % 8) * B:(i % 8 + 1) * B]
        lg.append(float(tg.step(xb)[0]))
        le.append(float(te.step(xb)[0]))
    assert all(np.isfinite(lg)) and all(np.isfinite(le))
    assert np.mean(lg[-10:]) < 0.5 * lg[0]
    np.testing.assert_allclose(np.mean(lg[-10:]), np.mean(le[-10:]), rtol=0.2)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_graph_replays_queued_after_sync_stay_finite():
    """Regression: bench-shaped replays queued back to back after a host sync
    (the ROCm graph packet-capture race turned the loss NaN two replays after
    the sync, every run).  The flag is set in conftest / ocm before HIP init."""
    import os

    from ocm.vae_train import GraphedVAETrainer

    assert os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") == "0"
    dev = torch.device("cuda", 0)
    L, d, B = 1024, 16, 256
    g = torch.Generator(device="cpu").manual_seed(1)
    X = (1.0 + 0.3 * torch.randn(B * 8, L, generator=g)).to(dev)
    mean, std = X.mean(0).cpu().numpy(), X.std(0).cpu().numpy()
    torch.manual_seed(0)
    m = V.ConvVAE1D(L, d, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
    tr = GraphedVAETrainer(m, B, lr=1e-3, dtype=torch.bfloat16, graph=True)
    assert tr.graphed
    losses = torch.zeros(80, device=dev)
    for i in range(80):
        losses[i].copy_(tr.step(X[(i % 8) * B:(i % 8 + 1) * B])[0])
        if i in (9, 39):
            torch.cuda.synchronize()
    assert bool(torch.isfinite(losses).all()), losses.cpu()
    assert all(bool(torch.isfinite(p).all()) for p in m.parameters())


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(512, 3, 2048), (64, 12, 512), (7, 5, 33)])
def test_fast_batchnorm_matches_torch(dtype, shape):
    """libocm training-mode BN == torch.nn.BatchNorm1d: output, running
    statistics, num_batches_tracked and the input / weight / bias gradients."""
    from ocm.bn import FastBatchNorm1d

    dev = torch.device("cuda", 0)
    N, C, L = shape
    g = torch.Generator(device="cpu").manual_seed(C * L)
    x0 = (3.0 + 2.0 * torch.randn(N, C, L, generator=g)).to(dev)
    ref = torch.nn.BatchNorm1d(C).to(dev)
    fast = FastBatchNorm1d(C).to(dev)
    with torch.no_grad():
        ref.weight.copy_(torch.linspace(0.5, 1.5, C))
        ref.bias.copy_(torch.linspace(-0.2, 0.3, C))
    fast.load_state_dict(ref.state_dict())
    xr = x0.to(dtype).requires_grad_(True)
    xf = x0.to(dtype).requires_grad_(True)
    yr, yf = ref(xr), fast(xf)
    gy = torch.randn(N, C, L, generator=g).to(dev).to(dtype)
    (yr.float() * gy.float()).sum().backward()
    (yf.float() * gy.float()).sum().backward()
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(yf.float(), yr.float(), **tol)
    torch.testing.assert_close(xf.grad.float(), xr.grad.float(), **tol)
    torch.testing.assert_close(fast.weight.grad, ref.weight.grad, rtol=1e-3, atol=1e-2 * N * L / 1000)
    torch.testing.assert_close(fast.bias.grad, ref.bias.grad, rtol=1e-3, atol=1e-2 * N * L / 1000)
    torch.testing.assert_close(fast.running_mean, ref.running_mean, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(fast.running_var, ref.running_var, rtol=1e-3, atol=1e-4)
    assert int(fast.num_batches_tracked) == int(ref.num_batches_tracked) == 1
    # the one-launch forms (L % 8 = 0 here: the first two shapes) never gave up waiting
    import ctypes

    from ocm import _lib
    torch.cuda.synchronize()
    n = ctypes.c_int64(-1)
    assert _lib.load().ocm_bn_fused_timeouts(ctypes.byref(n)) == 0 and n.value == 0


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(8192, 3, 2048), (40000, 12, 16), (7, 5, 33)])
@pytest.mark.parametrize("elu", [False, True])
def test_eval_batchnorm_matches_torch(dtype, shape, elu):
    """Eval-mode FastBatchNorm1d under no_grad (ocm_bn_fwd_eval, the latent
    encoding) == nn.BatchNorm1d(.eval()) (+ ELU) on trained running statistics,
    including N·C past a 65535-row grid and a length that is not a multiple of 8."""
    from ocm.bn import FastBatchNorm1d

    dev = torch.device("cuda", 0)
    N, C, L = shape
    g = torch.Generator(device="cpu").manual_seed(C * L + 7)
    ref = torch.nn.BatchNorm1d(C).to(dev)
    fast = FastBatchNorm1d(C).to(dev)
    if elu:
        fast.fuse_elu()
    with torch.no_grad():
        ref.weight.copy_(torch.linspace(0.5, 1.5, C))
        ref.bias.copy_(torch.linspace(-0.2, 0.3, C))
        ref.running_mean.copy_(torch.linspace(-1.0, 2.0, C))
        ref.running_var.copy_(torch.linspace(0.3, 4.0, C))
    fast.load_state_dict(ref.state_dict())
    ref.eval()
    fast.eval()
    x = (0.5 + 2.0 * torch.randn(N, C, L, generator=g)).to(dev).to(dtype)
    with torch.no_grad():
        yr = ref(x.float())
        if elu:
            yr = torch.nn.functional.elu(yr)
        yf = fast(x)
    assert yf.dtype == dtype and yf.shape == x.shape
    tol = dict(rtol=1e-2, atol=1e-2) if dtype == torch.bfloat16 else dict(rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(yf.float(), yr, **tol)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("shape", [(512, 3, 2048), (64, 12, 512), (7, 5, 33)])
def test_fused_batchnorm_elu_matches_torch(dtype, shape):
    """FastBatchNorm1d.fuse_elu() == nn.BatchNorm1d followed by nn.ELU: output,
    running statistics and the input / weight / bias gradients (the ELU's
    backward formed from the saved output inside the BN kernels).  The
    reference runs in float32 on the same (bf16-valued) inputs: the fused
    kernels keep z and the ELU's input gradient in float32 where torch's bf16
    modules round both to bf16 (2⁻⁸), which moves a small channel's Σ dz·x̂ by
    more than that rounding of the output does."""
    from ocm.bn import FastBatchNorm1d

    dev = torch.device("cuda", 0)
    N, C, L = shape
    g = torch.Generator(device="cpu").manual_seed(C * L + 1)
    x0 = (0.5 + 2.0 * torch.randn(N, C, L, generator=g)).to(dev)
    ref = torch.nn.BatchNorm1d(C).to(dev)
    fast = FastBatchNorm1d(C).fuse_elu().to(dev)
    with torch.no_grad():
        ref.weight.copy_(torch.linspace(0.5, 1.5, C))
        ref.bias.copy_(torch.linspace(-0.2, 0.3, C))
    fast.load_state_dict(ref.state_dict())
    xr = x0.to(dtype).float().requires_grad_(True)
    xf = x0.to(dtype).requires_grad_(True)
    yr, yf = torch.nn.functional.elu(ref(xr)), fast(xf)
    gy = torch.randn(N, C, L, generator=g).to(dev).to(dtype)
    (yr * gy.float()).sum().backward()
    (yf.float() * gy.float()).sum().backward()
    tol = dict(rtol=2e-2, atol=2e-2) if dtype == torch.bfloat16 else dict(rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(yf.float(), yr.float(), **tol)
    torch.testing.assert_close(xf.grad.float(), xr.grad.float(), **tol)
    gtol = dict(rtol=1e-2, atol=5e-3 * (N * L) ** 0.5) if dtype == torch.bfloat16 else \
        dict(rtol=1e-3, atol=1e-2 * N * L / 1000)
    torch.testing.assert_close(fast.weight.grad, ref.weight.grad, **gtol)
    torch.testing.assert_close(fast.bias.grad, ref.bias.grad, **gtol)
    torch.testing.assert_close(fast.running_mean, ref.running_mean, rtol=1e-4, atol=1e-4)
    fast.eval()
    ref.eval()
    torch.testing.assert_close(fast(x0), torch.nn.functional.elu(ref(x0)))
    import ctypes

    from ocm import _lib
    torch.cuda.synchronize()
    n = ctypes.c_int64(-1)
    assert _lib.load().ocm_bn_fused_timeouts(ctypes.byref(n)) == 0 and n.value == 0


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_c4_graph_step_with_grad_allreduce():
    """C5's data-parallel step at the C4 network shape (cb=3, nf=3, ks=7,
    hid=64, d=32; B=512 × L=2048, bf16): the flat-gradient RCCL all-reduce is
    captured into the step's HIP graph (one replay per step), every .grad is a
    view of the one buffer, and the step trains like the single-GPU graph step.
    World size 1 (one GPU per box), in a child process with its own RCCL group:
    three trainers built and closed in turn (a sweep), each
    captured while the caller's eager all-reduce is still tracked by the
    watchdog, then a normal exit.  World 2 runs over gloo on the CPU
    (tests/test_vae_ddp.py)."""
    import json
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    r = subprocess.run([sys.executable, os.path.join(here, "c4_ddp_worker.py")], capture_output=True, text=True,
                       timeout=240, cwd=os.path.dirname(here))
    assert r.returncode == 0, r.stderr[-3000:]  # a normal exit: trainers closed, process group destroyed
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["exit"] == "normal" and len(res["points"]) == 3
    for pt in res["points"]:
        assert pt["allreduce"] and pt["graphed"] and pt["grads_are_views"] and pt["own_comm"]
        print("flight recorder: pending before", pt["pending_before"], "at capture", pt["pending_at_capture"],
              "after", pt["pending_after"], "trainer build", round(pt["build_s"], 3), "s")
        # the caller's eager all-reduce (held behind a GPU spin) was still tracked
        # when the capture began, and the guard waited it out (ocm/rccl.py)
        assert pt["pending_before"] >= 1 and pt["pending_at_capture"] >= 1
        assert not pt["pending_after"]
        assert pt["closed"] and pt["step_after_close_raises"]
        la, lb = np.array(pt["loss_ddp"]), np.array(pt["loss_single"])
        assert np.isfinite(la).all() and np.isfinite(lb).all() and pt["params_finite"]
        assert la[-5:].mean() < la[0]
        np.testing.assert_allclose(la[-5:].mean(), lb[-5:].mean(), rtol=0.05)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_c5_shape_rank_share_and_latent_simca(tmp_path):
    """C5 (BASELINE.json: VAE-SIMCA DDP, 10M × 4096) at one rank's share of the
    global matrix (10M / 8 = 1.25M rows × 4096, 20.5 GB of on-device Philox
    shards, scripts/bench_vae_ddp.py): the L = 4096 network (1.59 M params),
    B = 512, bf16 graphed steps, then SIMCA-on-latents on its latents
    (utils/final_vaesimca.py:428-442, 510-533) checked against the oracle.
    Child process: the step graph holds its resources until the process ends."""
    import json
    import os
    import subprocess
    import sys

    from oracle import simca_oracle as O

    here = os.path.dirname(os.path.abspath(__file__))
    dump = str(tmp_path / "c5.npz")
    r = subprocess.run([sys.executable, os.path.join(os.path.dirname(here), "scripts", "bench_vae_ddp.py"),
                        "--rows", "1250000", "--steps", "20", "--warmup", "5", "--latent-rows", "65536",
                        "--dump", dump], capture_output=True, text=True, timeout=300, cwd=os.path.dirname(here))
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["config"]["params"] > 1_500_000 and res["params_finite"]
    assert np.isfinite(res["final_loss"]) and res["final_loss"] < res["loss_after_warmup"]
    g = np.load(dump)
    mean, inv, t2thr, qthr = O.latent_stats(g["mus"].astype(np.float64), g["q"].astype(np.float64))
    np.testing.assert_allclose(g["lmean"], mean, rtol=1e-6, atol=1e-7)
    np.testing.assert_allclose(g["inv"], inv, rtol=1e-5, atol=1e-6 * np.abs(inv).max())
    np.testing.assert_allclose([float(g["t2lim"]), float(g["qlim"])], [t2thr, qthr], rtol=1e-5)
    acc, f, fcrit = O.full_distance_decision(g["mus"].astype(np.float64), mean, g["q"].astype(np.float64))
    np.testing.assert_allclose(float(g["fcrit"]), fcrit, rtol=1e-6)
    band = np.abs(f - fcrit) > 1e-5 * fcrit
    np.testing.assert_array_equal(g["accept"][band], acc[band])
    assert 0.5 < res["latents"]["accept_rate"] <= 1.0


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("loss", ["bce", "euclidean"])
def test_fused_step_matches_torch_step(loss):
    """The libocm loss path (ocm/vae_fused.py: reparameterisation + KL, the
    de-standardised reconstruction term + total and their backward passes)
    against the torch step on the GPU, eager float32, identical ε draws:
    losses to 1e-5 over 3 steps and every parameter gradient to 1e-4 of its
    norm.  (Parameter values are not compared after several Adam steps: the
    biases a BatchNorm cancels have rounding-level gradients, which Adam
    turns into ±lr steps in either implementation.)"""
    from ocm.vae_train import GraphedVAETrainer

    dev = torch.device("cuda", 0)
    L, d, B = 256, 8, 64
    g = torch.Generator(device="cpu").manual_seed(3)
    X = (1.0 + 0.3 * torch.randn(B * 3, L, generator=g)).to(dev)
    mean, std = X.mean(0).cpu().numpy(), X.std(0).cpu().numpy()
    torch.manual_seed(0)
    m1 = V.ConvVAE1D(L, d, mean, std, conv_blocks=2, n_filters=3, kernel_size=5, hidden_fc=32).to(dev)
    m2 = copy.deepcopy(m1)
    tf = GraphedVAETrainer(m1, B, lr=1e-3, weight_decay=1e-4, beta=0.7, loss=loss, dtype=torch.float32, graph=False)
    tt = GraphedVAETrainer(m2, B, lr=1e-3, weight_decay=1e-4, beta=0.7, loss=loss, dtype=torch.float32, graph=False,
                           fused=False)
    assert tf.fused and not tt.fused
    for i in range(3):
        xb = X[i * B:(i + 1) * B]
        torch.manual_seed(50 + i)
        a = [float(v) for v in tf.step(xb)]
        torch.manual_seed(50 + i)
        b = [float(v) for v in tt.step(xb)]
        np.testing.assert_allclose(a, b, rtol=1e-5, atol=1e-7)
        if i == 0:  # identical weights before the first update: the gradients must agree
            gmax = max(float(p.grad.norm()) for p in m2.parameters())
            for (n1, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
                scale = float(p2.grad.norm())
                # BN-cancelled biases: rounding-level gradients, compared at the global scale
                tol = 1e-4 * scale if scale > 1e-5 * gmax else 1e-6 * gmax
                assert float((p1.grad - p2.grad).norm()) <= tol, n1


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_fused_adam_matches_torch_adam():
    """ocm_adam_step (one launch over a table of tensors) = torch.optim.Adam
    with L2 weight decay, 10 steps on the same gradients."""
    from ocm.vae_fused import FusedAdam

    dev = torch.device("cuda", 0)
    rng = torch.Generator(device="cpu").manual_seed(5)
    shapes = [(3, 1, 7), (3,), (64, 32), (1000,), (5, 5)]
    p1 = [torch.randn(s, generator=rng).to(dev).requires_grad_() for s in shapes]
    p2 = [p.detach().clone().requires_grad_() for p in p1]
    fa = FusedAdam(p1, lr=2e-3, weight_decay=1e-3)
    ta = torch.optim.Adam(p2, lr=2e-3, weight_decay=1e-3)
    for _ in range(10):
        grads = [torch.randn(s, generator=rng).to(dev) for s in shapes]
        for p, gr in zip(p1, grads):
            p.grad = gr.clone()
        for p, gr in zip(p2, grads):
            p.grad = gr.clone()
        fa.step()
        ta.step()
    for a, b in zip(p1, p2):
        torch.testing.assert_close(a.detach(), b.detach(), rtol=1e-5, atol=1e-6)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("layout", ["grad_none", "flat_views"])
def test_bf16_fused_step_matches_bf16_torch_step(layout):
    """the production step (bf16, fused: cast_bf16 +
    functional_call, libocm losses, FusedAdam) against the fused=False bf16
    step (torch autocast, torch losses, torch Adam) with the same ε seeds, at
    the C4 network's layer plan (L = 512).  Losses to 1e-2 and every parameter
    gradient to 5e-2 of its norm (bf16 roundings sit in different places),
    once with .grad = None before backward (one process) and once with the
    gradients as views of the flat all-reduce buffer (world-1 gloo group), the
    layout in which the cast's backward writes straight into the views."""
    import socket

    import torch.distributed as dist

    from ocm.vae_train import GraphedVAETrainer

    dev = torch.device("cuda", 0)
    L, d, B = 512, 16, 128
    g = torch.Generator(device="cpu").manual_seed(11)
    X = (1.0 + 0.3 * torch.randn(B * 2, L, generator=g)).to(dev)
    mean, std = X.mean(0).cpu().numpy(), X.std(0).cpu().numpy()
    torch.manual_seed(0)
    m1 = V.ConvVAE1D(L, d, mean, std, conv_blocks=3, n_filters=3, kernel_size=7, hidden_fc=64).to(dev)
    m2 = copy.deepcopy(m1)
    flat = layout == "flat_views"
    if flat:
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        tf = GraphedVAETrainer(m1, B, lr=1e-3, dtype=torch.bfloat16, graph=False, grad_allreduce=flat)
        tt = GraphedVAETrainer(m2, B, lr=1e-3, dtype=torch.bfloat16, graph=False, grad_allreduce=flat, fused=False)
        assert tf.fused and not tt.fused and tf.allreduce == flat
        for i in range(2):
            xb = X[i * B:(i + 1) * B]
            torch.manual_seed(70 + i)
            a = [float(v) for v in tf.step(xb)]
            torch.manual_seed(70 + i)
            b = [float(v) for v in tt.step(xb)]
            np.testing.assert_allclose(a, b, rtol=1e-2)
            if i == 0:
                if flat:
                    lo = tf.flat_grad.data_ptr()
                    hi = lo + tf.flat_grad.numel() * 4
                    assert all(lo <= p.grad.data_ptr() < hi for p in m1.parameters())
                gmax = max(float(p.grad.norm()) for p in m2.parameters())
                for (n1, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
                    scale = float(p2.grad.norm())
                    tol = 5e-2 * scale if scale > 1e-3 * gmax else 5e-4 * gmax
                    assert float((p1.grad - p2.grad).norm()) <= tol, (n1, float((p1.grad - p2.grad).norm()), scale)
    finally:
        if flat:
            dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_cast_bf16_accumulates_into_existing_grads():
    """without the caller's 'freshly zeroed' promise the cast's
    backward returns its gradients, so autograd adds them to a .grad that is
    already there (gradient accumulation keeps working); FusedAdam skips a
    parameter without a gradient, as torch.optim.Adam does."""
    from ocm import vae_fused as vf

    dev = torch.device("cuda", 0)
    w = torch.randn(8, 4, device=dev, requires_grad=True)
    u = torch.randn(3, device=dev, requires_grad=True)
    x = torch.randn(5, 4, device=dev, dtype=torch.bfloat16)
    (wb,) = vf.cast_bf16(w)
    (x @ wb.t()).float().sum().backward()
    g1 = w.grad.clone()
    (wb,) = vf.cast_bf16(w)
    (x @ wb.t()).float().sum().backward()  # accumulates: 2 × the first gradient
    torch.testing.assert_close(w.grad, 2 * g1)
    u_before, w_before = u.detach().clone(), w.detach().clone()
    opt = vf.FusedAdam([w, u], lr=1e-2)
    opt.step()  # u.grad is None: u is left alone, w takes its step
    torch.testing.assert_close(u.detach(), u_before)
    assert float((w.detach() - w_before).abs().max()) > 1e-3


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("k,n,act,bias", [(6144, 64, True, True), (64, 32, False, True), (32, 64, True, True),
                                          (64, 6144, True, True), (128, 64, True, True), (256, 128, True, False)])
def test_linear_act_matches_torch(k, n, act, bias):
    """vae_fused.linear_act (the bf16 step's bottleneck Linear layers, round 6)
    against F.linear (+ F.elu) under torch autograd on the same bf16 tensors:
    the forward is the same torch call; the backward's ELU gradient and bias
    sum (one ocm_vae_act_bias_bwd launch) and the two GEMM gradients built on
    them (the K = 6144 input gradient through gemm_sk) match torch's to bf16
    roundings."""
    from torch import nn

    from ocm import vae_fused as vf

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(k + n)
    lin = nn.Linear(k, n, bias=bias).to(dev).to(torch.bfloat16)
    x = torch.randn(512, k, generator=g).to(dev).to(torch.bfloat16)
    go = torch.randn(512, n, generator=g).to(dev).to(torch.bfloat16)
    xa = x.clone().requires_grad_(True)
    out = vf.linear_act(xa, lin, act)
    out.backward(go)
    ga = (xa.grad, lin.weight.grad.clone()) + ((lin.bias.grad.clone(),) if bias else ())
    lin.weight.grad = None
    if bias:
        lin.bias.grad = None
    xb = x.clone().requires_grad_(True)
    ref = torch.nn.functional.linear(xb, lin.weight, lin.bias)
    ref = torch.nn.functional.elu(ref) if act else ref
    ref.backward(go)
    gb = (xb.grad, lin.weight.grad) + ((lin.bias.grad,) if bias else ())
    if act and k <= 256:  # ocm_vae_linear_act: its own f32 sums, within one bf16 rounding of torch's output
        torch.testing.assert_close(out.detach().float(), ref.detach().float(), rtol=2 ** -7,
                                   atol=2 ** -7 * float(ref.detach().abs().max()))
    else:
        assert torch.equal(out, ref)  # the forward is torch's call
    for name, a, b in zip(("x", "W", "b"), ga, gb):
        a, b = a.float(), b.float()
        err = float((a - b).norm() / b.norm())
        print(name, "rel err", err)
        assert err < 1e-2, (name, err)


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("M,N,K,b_nk,bias", [(512, 64, 6144, True, True), (512, 64, 6144, False, False),
                                             (128, 192, 2048, True, False), (192, 128, 4096, False, True)])
def test_gemm_sk_matches_float_reference(M, N, K, b_nk, bias):
    """vae_fused.gemm_sk (ocm_gemm_bf16_sk, round 6: the bottleneck's K = 6144
    products split over K) against the float64 product of the same bf16
    operands, rounded to bf16: within two bf16 roundings everywhere."""
    from ocm import vae_fused as vf

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(M + N + K)
    A = torch.randn(M, K, generator=g).to(torch.bfloat16)
    B = torch.randn((N, K) if b_nk else (K, N), generator=g).to(torch.bfloat16)
    b = torch.randn(N, generator=g).to(torch.bfloat16) if bias else None
    C = vf.gemm_sk(A.to(dev), B.to(dev), b_nk, b.to(dev) if bias else None).cpu().double()
    ref = A.double() @ (B.double().t() if b_nk else B.double())
    if bias:
        ref = ref + b.double()
    err = (C - ref).abs() / (ref.abs() + 1e-2 * ref.abs().max())
    assert float(err.max()) < 2 ** -7, float(err.max())


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_linear_pair_matches_torch():
    """vae_fused.linear_pair (fc_mu and fc_logvar on one input, round 6: the
    input gradient as one GEMM + one accumulating GEMM) against two F.linear
    calls under torch autograd, bf16."""
    from torch import nn

    from ocm import vae_fused as vf

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(5)
    l1, l2 = nn.Linear(64, 32).to(dev).to(torch.bfloat16), nn.Linear(64, 32).to(dev).to(torch.bfloat16)
    x = torch.randn(512, 64, generator=g).to(dev).to(torch.bfloat16)
    g1, g2 = (torch.randn(512, 32, generator=g).to(dev).to(torch.bfloat16) for _ in range(2))
    xa = x.clone().requires_grad_(True)
    y1, y2 = vf.linear_pair(xa, l1, l2)
    torch.autograd.backward([y1, y2], [g1, g2])
    got = [xa.grad] + [p.grad.clone() for p in (l1.weight, l1.bias, l2.weight, l2.bias)]
    for p in (l1.weight, l1.bias, l2.weight, l2.bias):
        p.grad = None
    xb = x.clone().requires_grad_(True)
    r1, r2 = torch.nn.functional.linear(xb, l1.weight, l1.bias), torch.nn.functional.linear(xb, l2.weight, l2.bias)
    torch.autograd.backward([r1, r2], [g1, g2])
    want = [xb.grad] + [p.grad for p in (l1.weight, l1.bias, l2.weight, l2.bias)]
    assert torch.equal(y1, r1) and torch.equal(y2, r2)
    for a, b in zip(got, want):
        a, b = a.float(), b.float()
        assert float((a - b).norm() / b.norm()) < 1e-2


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
@pytest.mark.parametrize("adjacent", [True, False])
def test_linear_cat_packed_bottleneck_matches_pair(adjacent):
    """vae_fused.linear_cat + bottleneck_packed (round 6: [fc_mu; fc_logvar] as
    one product whose packed B×2d output the bottleneck reads in place) against
    linear_pair + bottleneck on the same bf16 tensors and ε: z and the KL equal,
    every gradient within bf16 roundings.  ``adjacent``: the two weights (and
    biases) back to back in one buffer, as cast_bf16 lays them out (a view, no
    copy); else torch.cat."""
    from torch import nn

    from ocm import vae_fused as vf

    dev = torch.device("cuda", 0)
    g = torch.Generator(device="cpu").manual_seed(9)
    l1, l2 = nn.Linear(64, 32).to(dev), nn.Linear(64, 32).to(dev)
    if adjacent:
        w1, b1, w2, b2 = vf.cast_bf16(l1.weight, l1.bias, l2.weight, l2.bias)
        assert w2.data_ptr() == w1.data_ptr() + w1.numel() * 2 and b2.data_ptr() == b1.data_ptr() + 64
    else:
        w1, b1, w2, b2 = (t.detach().to(torch.bfloat16).requires_grad_(True) for t in
                          (l1.weight, l1.bias, l2.weight, l2.bias))
    x = torch.randn(512, 64, generator=g).to(dev).to(torch.bfloat16)
    eps = torch.randn(512, 32, generator=g).to(dev).to(torch.bfloat16)
    gz = torch.randn(512, 32, generator=g).to(dev).to(torch.bfloat16)

    def run(packed):
        xa = x.clone().requires_grad_(True)
        if packed:
            ml = vf._LinearCat.apply(xa, w1, b1, w2, b2)
            z, kl = vf.bottleneck_packed(ml, eps)
        else:
            mu, lv = vf._LinearPair.apply(xa, w1, b1, w2, b2)
            z, kl = vf.bottleneck(mu, lv, eps)
        tgt = [t for t in (xa, w1, b1, w2, b2) if t.requires_grad]
        grads = torch.autograd.grad([z, kl], tgt, [gz, torch.tensor(0.7, device=dev)])
        return z.detach(), kl.detach(), grads

    z1, k1, g1 = run(True)
    z2, k2, g2 = run(False)
    assert torch.equal(z1, z2)
    torch.testing.assert_close(k1, k2, rtol=1e-6, atol=1e-6)
    for a, b in zip(g1, g2):
        a, b = a.float(), b.float()
        assert float((a - b).norm() / b.norm()) < 1e-2


_BN_FUSED_CHILD = r"""
import ctypes, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "ocm-vae-simca_amd"))
import torch
from ocm import _lib
from ocm.bn import FastBatchNorm1d
dev = torch.device("cuda", 0)
for (N, C, L) in [(512, 3, 2048), (64, 12, 512)]:
    g = torch.Generator(device="cpu").manual_seed(C * L + 3)
    x0 = (0.5 + 2.0 * torch.randn(N, C, L, generator=g)).to(dev)
    ref = torch.nn.BatchNorm1d(C).to(dev)
    fast = FastBatchNorm1d(C).fuse_elu().to(dev)
    fast.load_state_dict(ref.state_dict())
    xr = x0.bfloat16().float().requires_grad_(True)
    xf = x0.bfloat16().requires_grad_(True)
    yr, yf = torch.nn.functional.elu(ref(xr)), fast(xf)
    gy = torch.randn(N, C, L, generator=g).to(dev).bfloat16()
    (yr * gy.float()).sum().backward()
    (yf.float() * gy.float()).sum().backward()
    torch.testing.assert_close(yf.float(), yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(xf.grad.float(), xr.grad, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(fast.running_mean, ref.running_mean, rtol=1e-4, atol=1e-4)
torch.cuda.synchronize()
n = ctypes.c_int64(-1)
assert _lib.load().ocm_bn_fused_timeouts(ctypes.byref(n)) == 0 and n.value == 0
print("bn fused ok")
"""


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a HIP device")
def test_bn_one_launch_opt_in_matches_torch():
    """The opt-in one-launch BatchNorm (OCM_BN_FUSED=1: statistics and
    normalisation in one kernel with an in-kernel epoch wait, off by default)
    against nn.BatchNorm1d + ELU, in a child process (the switch is read once
    per process); no wait gave up."""
    import subprocess
    import sys

    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, OCM_BN_FUSED="1")
    r = subprocess.run([sys.executable, "-c", _BN_FUSED_CHILD, repo], capture_output=True, text=True, timeout=240,
                       env=env)
    assert r.returncode == 0 and "bn fused ok" in r.stdout, r.stderr[-3000:]
