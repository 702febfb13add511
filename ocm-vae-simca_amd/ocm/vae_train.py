"""HIP-graph-captured VAE training step (C4/C5).

The reference's step (vae_bce_nut.py:178-203; utils/final_vaesimca.py:362-375)
is  forward → beta_vae_bce_loss → zero_grad → backward → Adam.step, with two
``.item()`` host syncs inside the loss.  At B=512 × L=2048 with 1-12-channel
convolutions the step is launch-bound (≈150 small kernels), so on MI355X it
is captured ONCE into a HIP graph (torch.cuda.CUDAGraph is hipGraph on ROCm)
and replayed: one launch per step, no host round trip.  The loss terms stay
on the device (``last_recon`` / ``last_kl``); the ε of the reparameterisation
is drawn inside the graph from the graph-safe Philox generator, so every
replay samples fresh noise like the eager step.

Mixed precision: ``dtype=torch.bfloat16`` runs the network under bf16
autocast (the loss, BN statistics and Adam state stay fp32).

Multi-GPU (C5): one process per GPU, pass the bare model and
the process group.  The trainer broadcasts rank 0's parameters and buffers,
points every parameter's .grad into one flat fp32 buffer, and after the
backward pass all-reduces that buffer once with ncclAvg (one RCCL call over
xGMI, 3.2 MB at L = 2048, 6.4 MB at L = 4096) — DDP's gradient averaging,
captured into the same HIP graph as the step, so a replay is still one
launch.  The trainer's collectives run on an RCCL communicator of its own
(ocm/rccl.py), never on ProcessGroupNCCL, whose watchdog aborts the process
if it polls an event during a capture.  BatchNorm statistics stay per rank, as in DDP;
``sync_buffers()`` copies rank 0's running statistics to every rank
(DDP's broadcast_buffers) before evaluation.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist
from torch import nn

import vae_model as V

__all__ = ["GraphedVAETrainer"]

# the bf16 fused step's bottleneck Linear layers through vae_fused.linear_act
# (False: torch's autocast Linear + ELU, for A/B runs: scripts/vae_linear_ab.py)
LINEAR_FUSED = True
# fc_mu and fc_logvar as one packed product read in place by the bottleneck
# kernel (False: vae_fused.linear_pair + the two-tensor bottleneck; A/B)
PACKED_MU_LOGVAR = True
# the fused step's backward seeded from a persistent unit gradient (False:
# total.backward(), which fills a fresh one each step; A/B, scripts/vae_ab.py)
PERSISTENT_ONE = True


def _elu_dense(seq, pattern) -> bool:
    """``seq`` is an nn.Sequential of Linear / ELU(α = 1) / Identity laid out as
    ``pattern`` ("L", "E", "I")."""
    kinds = {"L": nn.Linear, "E": nn.ELU, "I": nn.Identity}
    if not isinstance(seq, nn.Sequential) or len(seq) != len(pattern):
        return False
    return all(type(mod) is kinds[k] and (k != "E" or float(mod.alpha) == 1.0) for mod, k in zip(seq, pattern))


class _FusedForward(nn.Module):
    """encode → z = μ + ε·exp(½logσ²) and the KL (libocm) → decode, as one
    module so torch.func.functional_call can run it on substituted (bf16)
    Linear parameters (vae_model.py:116-134).  With ``linear_fused`` (the bf16
    step of the stock layout: ELU, no dropout) the bottleneck's Linear layers
    run through vae_fused.linear_act, whose backward forms the ELU and bias
    gradients in one launch per layer."""

    def __init__(self, m, vf, linear_fused=False):
        super().__init__()
        self.m = m
        self._vf = vf
        self._lin_fused = bool(linear_fused) and _elu_dense(getattr(m, "fc", None), "LEI") \
            and _elu_dense(getattr(m, "fc_dec", None), "LEILE") \
            and isinstance(getattr(m, "fc_mu", None), nn.Linear) and isinstance(getattr(m, "fc_logvar", None), nn.Linear)

    def forward(self, xin):
        m, la = self.m, self._vf.linear_act
        if self._lin_fused:  # vae_model.py:116-134 with the Linear layers through linear_act
            h = la(m.encoder_conv(xin.unsqueeze(1)).flatten(1), m.fc[0], True)
            if PACKED_MU_LOGVAR and m.fc_mu.out_features == m.fc_logvar.out_features:
                # [μ | logσ²] from one product, read in place by the bottleneck
                ml = self._vf.linear_cat(h, m.fc_mu, m.fc_logvar)
                d = m.fc_mu.out_features
                eps = torch.randn((ml.shape[0], d), dtype=ml.dtype, device=ml.device)  # = randn_like(μ)
                z, kl = self._vf.bottleneck_packed(ml, eps)
            else:
                mu, logvar = self._vf.linear_pair(h, m.fc_mu, m.fc_logvar)
                eps = torch.randn_like(mu)
                z, kl = self._vf.bottleneck(mu, logvar, eps)
        else:
            mu, logvar = m.encode(xin)
            eps = torch.randn_like(mu)
            z, kl = self._vf.bottleneck(mu, logvar, eps)
        if not self._lin_fused:
            return m.decode(z), kl
        h = la(la(z, m.fc_dec[0], True), m.fc_dec[3], True)
        x = m.decoder_conv(h.view(z.shape[0], m._enc_out_channels, m._enc_out_length)).squeeze(1)
        L = m.input_length
        if x.shape[-1] > L:
            x = x[..., :L]
        elif x.shape[-1] < L:
            x = torch.nn.functional.pad(x, (0, L - x.shape[-1]))
        return x, kl


class GraphedVAETrainer:
    """One optimizer step per ``step(x)``; ``x`` (B, L) float32 on the device.

    loss: "bce" (vae_model.beta_vae_bce_loss: BCE-with-logits on the
    de-standardised output), "cosine" (beta_vae_cosine_loss), or the
    utils/final_vaesimca.py:208-224 variants "bce_prob" (probability BCE on the
    min-max scaled reconstruction, its "X_bce") and "euclidean" (MSE, its
    "X_euclidean"); lr / weight_decay as torch.optim.Adam
    (vae_bce_nut.py:155-159).  ``graph=True`` needs the runtime flag set by
    importing ``ocm`` before torch initialises the GPU, and raises otherwise
    (pass ``graph=False`` for eager steps)."""

    LOSSES = ("bce", "cosine", "bce_prob", "euclidean")

    def __init__(self, model, batch: int, lr=1e-3, weight_decay=0.0, beta=1.0, loss="bce",
                 dtype=torch.bfloat16, graph=True, warmup=3, restore=True, group=None, grad_allreduce=None,
                 fused=True):
        self.model = model
        self.module = getattr(model, "module", model)
        dev = next(self.module.parameters()).device
        self.group = group
        distributed = dist.is_available() and dist.is_initialized()
        # A ProcessGroupNCCL watchdog that polls a collective's end event while
        # any stream is capturing is refused by HIP and aborts the process
        # (round 4, DESIGN.md §5 caveat 5).  Eager collectives the CALLER issued
        # on its process groups are waited out here, on the watchdogs' own
        # records (flight recorder), before anything else: from here to the
        # capture the trainer issues none (its own collectives run on its RCCL
        # communicator, which no watchdog tracks, ocm/rccl.py).
        self.pending_at_capture = 0
        if graph and dev.type == "cuda":
            from .rccl import wait_pg_collectives_retired

            self.pending_at_capture = wait_pg_collectives_retired(group)
        self.world = dist.get_world_size(group) if distributed else 1
        # data-parallel gradient averaging (None: whenever the world has > 1 rank)
        self.allreduce = (self.world > 1) if grad_allreduce is None else bool(grad_allreduce and distributed)
        # the trainer's collectives run on an RCCL communicator of its own
        # (ocm/rccl.py) when the group is RCCL's: none of them is ever tracked
        # by a ProcessGroupNCCL watchdog, which would abort the process if it
        # polled one while the step is being captured; gloo groups (CPU, or
        # several ranks sharing one GPU in tests) use torch.distributed
        self._comm = None
        if self.allreduce:
            if dev.type == "cuda" and "nccl" in str(dist.get_backend(group)):
                from .rccl import Communicator

                self._comm = Communicator(group, dev)
            self._flatten_grads(dev)
            self._broadcast_state()
        self.beta = float(beta)
        if loss not in self.LOSSES:
            raise ValueError(f"loss must be one of {self.LOSSES}")
        self.loss = loss
        self.dtype = dtype
        # torch's fused Adam on the GPU (one multi-tensor kernel per step): 480 vs 437
        # steps/s for the foreach form on MI355X (C4 net, B = 512), losses equal to
        # 1e-4; OCM_VAE_ADAM=foreach for A/B.  Eager CPU steps keep the reference's
        # Adam arithmetic exactly (tests/test_vae_train.py)
        # On the GPU the small tensors of the step run on libocm (ocm/vae_fused.py):
        # the reparameterisation + KL, the de-standardisation + reconstruction
        # term + total and their backward passes in four launches, Adam in one —
        # the graphed step is bound by its kernel count.  Eager CPU steps keep
        # the reference's torch arithmetic exactly (tests/test_vae_train.py);
        # fused=False keeps torch on the GPU too (A/B, tests).
        self.fused = (dev.type == "cuda" and fused and loss in ("bce", "euclidean")
                      and hasattr(self.module, "encode") and hasattr(self.module, "decode"))
        if self.fused:
            from . import vae_fused

            self._vf = vae_fused
            self.opt = vae_fused.FusedAdam(model.parameters(), lr=lr, weight_decay=weight_decay)
            self._rbufs = vae_fused.ReconBuffers(self.module.spec_mean, self.module.spec_std)
            # bf16 steps: the Linear layers run on bf16 copies of their
            # parameters made in one launch per step (vae_fused.cast_bf16)
            self._fwd = _FusedForward(self.module, vae_fused, linear_fused=dtype == torch.bfloat16 and LINEAR_FUSED)
            self._lin = [("m." + n, p) for n, p in self.module.named_parameters()
                         if p.requires_grad and "." in n
                         and isinstance(self.module.get_submodule(n.rsplit(".", 1)[0]), nn.Linear)]
        else:
            gpu_fused = dev.type == "cuda"
            self.opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay, capturable=graph,
                                        **({"fused": True} if gpu_fused else {"foreach": True}))
        self.x = torch.zeros((batch, self.module.input_length), dtype=torch.float32, device=dev)
        self.graph = None
        self.restore = restore
        if graph and os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") != "0":
            # the runtime's packet-capture replay races (ocm/__init__.py); the
            # flag only takes effect if set before HIP initialises
            raise RuntimeError("GraphedVAETrainer(graph=True): DEBUG_CLR_GRAPH_PACKET_CAPTURE is not 0, and HIP-graph "
                               "replays race on this runtime without it (ocm/__init__.py).  Import ocm (or set the "
                               "variable to 0) before torch initialises the GPU, or pass graph=False for eager steps")
        self.graphed = graph
        if graph:
            self._capture(warmup)

    def _flatten_grads(self, dev):
        """Every parameter's .grad becomes a view of one flat buffer (one
        all-reduce per step; zero_grad(set_to_none=False) keeps the views)."""
        params = [p for p in self.module.parameters() if p.requires_grad]
        self.flat_grad = torch.zeros(sum(p.numel() for p in params), dtype=torch.float32, device=dev)
        o = 0
        for p in params:
            p.grad = self.flat_grad[o:o + p.numel()].view_as(p)
            o += p.numel()

    def _broadcast_state(self):
        self._broadcast(self.module.state_dict().values())

    def _broadcast(self, tensors):
        """Group rank 0's values of ``tensors`` on every rank, in place."""
        with torch.no_grad():
            if self._comm is not None:
                for t in tensors:
                    self._comm.broadcast(t, 0)
                return
            src = dist.get_global_rank(self.group, 0) if self.group is not None else 0
            for t in tensors:
                dist.broadcast(t, src=src, group=self.group)

    def _average_grads(self):
        """DDP averaging: one all-reduce of the flat gradient (ncclAvg on the
        trainer's communicator: the division runs inside the collective)."""
        if self._comm is not None:
            self._comm.all_reduce(self.flat_grad, average=True)
        else:
            dist.all_reduce(self.flat_grad, group=self.group)
            self.flat_grad.div_(self.world)

    def sync_buffers(self):
        """Rank 0's BatchNorm running statistics on every rank (DDP broadcast_buffers)."""
        if not self.allreduce:
            return
        self._broadcast(list(self.module.buffers()))

    def _body(self):
        # one process: gradients set to None, so backward hands each parameter
        # its freshly computed gradient (no per-parameter memset + accumulate
        # kernel: 43 adds and 11 fills per step in the r03g trace); with the
        # flat all-reduce buffer the .grad views must persist
        if self.fused and self.allreduce:
            self.flat_grad.zero_()  # one fill for every gradient view
        else:
            self.opt.zero_grad(set_to_none=not self.allreduce)
        if self.fused:
            return self._body_fused()
        with torch.autocast("cuda", dtype=self.dtype, enabled=self.dtype != torch.float32):
            x_rec, mu, logvar = self.model(self.x)
        x_rec, mu, logvar = x_rec.float(), mu.float(), logvar.float()
        if self.loss == "bce":
            recon = V.bce_recon_term(self.x, x_rec)
        elif self.loss == "cosine":
            recon = V.cosine_recon_term(self.x, x_rec)
        elif self.loss == "bce_prob":
            recon = V.bce_prob_recon_term(self.x, x_rec)
        else:
            recon = V.mse_recon_term(self.x, x_rec)
        kl = V.kl_term(mu, logvar)
        total = recon + self.beta * kl
        total.backward()
        if self.allreduce:
            self._average_grads()
        self.opt.step()
        return total.detach(), recon.detach(), kl.detach()

    def _body_fused(self):
        """The same step as _body with the loss terms and Adam on libocm: the
        network (encode / decode, vae_model.py:116-134) under autocast, then
        z = μ + ε·exp(½logσ²) and the KL (one launch), the de-standardised
        reconstruction term and the total (one launch)."""
        m = self.module
        if self.dtype == torch.bfloat16 and self._lin:
            # the flat all-reduce buffer was zeroed above: the cast's backward
            # may write the Linear gradients straight into its views
            casted = self._vf.cast_bf16(*[p for _, p in self._lin], into_zeroed_grads=self.allreduce)
            xin = self._vf.standardise(self.x, m.spec_mean, m.spec_std)
            with torch.autocast("cuda", dtype=self.dtype):
                xs, kl = torch.func.functional_call(self._fwd, dict(zip([n for n, _ in self._lin], casted)), (xin,))
        else:
            with torch.autocast("cuda", dtype=self.dtype, enabled=self.dtype != torch.float32):
                xs, kl = self._fwd((self.x - m.spec_mean) / m.spec_std)
        total, recon = self._vf.recon_total(self.x, xs, kl, self._rbufs, self.loss, self.beta)
        # d total / d total = 1 from a persistent tensor: backward() would fill a
        # fresh one (a kernel of its own) every step
        if not PERSISTENT_ONE:
            total.backward()
        else:
            if getattr(self, "_one", None) is None or self._one.device != total.device:
                self._one = torch.ones((), dtype=total.dtype, device=total.device)
            torch.autograd.backward(total, self._one)
        if self.allreduce:
            self._average_grads()
        self.opt.step()
        return total.detach(), recon, kl.detach()

    def _capture(self, warmup):
        self.model.train()
        # the warm-up steps (allocator, kernel selection, optimizer state
        # creation) run on the zero batch buffer: snapshot the model and put it
        # back afterwards, in place, so the first replay is training step 1
        saved = {k: v.detach().clone() for k, v in self.module.state_dict().items()}
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(warmup):
                self._body()
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        # (the caller's eager ProcessGroupNCCL collectives were waited out when
        # the trainer started, __init__)
        mode = "global"
        if self.allreduce:
            if self._comm is None:
                raise ValueError("GraphedVAETrainer(graph=True) with a gradient all-reduce needs an RCCL ('nccl') "
                                 "process group; pass graph=False for a gloo group")
            mode = "thread_local"
        with torch.cuda.graph(self.graph, capture_error_mode=mode):
            self.out = self._body()
        if self.fused:
            self.opt.flush_pending()
        if not self.restore:
            return
        with torch.no_grad():
            for k, v in self.module.state_dict().items():
                v.copy_(saved[k])
            if self.fused:
                self.opt.reset_state()
            else:
                for st in self.opt.state.values():  # fresh Adam moments and step counters
                    for t in st.values():
                        if torch.is_tensor(t):
                            t.zero_()

    def close(self):
        """Release the captured step graph, then the trainer's RCCL communicator
        — in that order, so no graph that captured the communicator's all-reduce
        outlives it.  A sweep that builds a trainer per grid point
        (utils/final_vaesimca.py:312-351) closes each one; the trainer cannot
        step afterwards.  Idempotent; also the context-manager exit."""
        if getattr(self, "_closed", False):
            return
        dev = self.x.device
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)  # no replay may still be running on the graph or the communicator
        if self.graph is not None:
            self.graph.reset()
            self.graph = None
            self.out = None
        if self._comm is not None:
            self._comm.close()
            self._comm = None
        self._closed = True

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()
        return False

    def step(self, x: torch.Tensor | None = None):
        """Run one training step on ``x`` (copied into the static batch buffer);
        returns device tensors (loss, recon, kl)."""
        if getattr(self, "_closed", False):
            raise RuntimeError("GraphedVAETrainer.step() after close()")
        if x is not None:
            self.x.copy_(x, non_blocking=True)
        if self.graph is not None:
            self.graph.replay()
            return self.out
        self.model.train()
        return self._body()
