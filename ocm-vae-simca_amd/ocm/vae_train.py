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

Multi-GPU (C5): wrap the model in DistributedDataParallel before building the
trainer; the gradient all-reduce (RCCL over xGMI) is captured with the step.
"""
from __future__ import annotations

import os
import warnings

import torch

import vae_model as V

__all__ = ["GraphedVAETrainer"]


class GraphedVAETrainer:
    """One optimizer step per ``step(x)``; ``x`` (B, L) float32 on the device.

    loss: "bce" (beta_vae_bce_loss) or "cosine" (beta_vae_cosine_loss);
    lr / weight_decay as torch.optim.Adam (vae_bce_nut.py:155-159)."""

    def __init__(self, model, batch: int, lr=1e-3, weight_decay=0.0, beta=1.0, loss="bce",
                 dtype=torch.bfloat16, graph=True, warmup=3, restore=True):
        self.model = model
        self.module = getattr(model, "module", model)
        dev = next(self.module.parameters()).device
        self.beta = float(beta)
        self.loss = loss
        self.dtype = dtype
        # torch's fused Adam on the GPU (one multi-tensor kernel per step): 480 vs 437
        # steps/s for the foreach form on MI355X (C4 net, B = 512), losses equal to
        # 1e-4; OCM_VAE_ADAM=foreach for A/B.  Eager CPU steps keep the reference's
        # Adam arithmetic exactly (tests/test_vae_train.py)
        fused = dev.type == "cuda" and os.environ.get("OCM_VAE_ADAM", "fused") == "fused"
        self.opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay, capturable=graph,
                                    **({"fused": True} if fused else {"foreach": True}))
        self.x = torch.zeros((batch, self.module.input_length), dtype=torch.float32, device=dev)
        self.graph = None
        self.restore = restore
        if graph and os.environ.get("DEBUG_CLR_GRAPH_PACKET_CAPTURE") != "0":
            # the runtime's packet-capture replay races (ocm/__init__.py); the
            # flag only takes effect if set before HIP initialises
            warnings.warn("DEBUG_CLR_GRAPH_PACKET_CAPTURE is not 0 (import ocm before torch initialises the GPU): "
                          "HIP-graph VAE steps are unsafe on this runtime, running the step eagerly")
            graph = False
        self.graphed = graph
        if graph:
            self._capture(warmup)

    def _body(self):
        self.opt.zero_grad(set_to_none=False)
        with torch.autocast("cuda", dtype=self.dtype, enabled=self.dtype != torch.float32):
            x_rec, mu, logvar = self.model(self.x)
        x_rec, mu, logvar = x_rec.float(), mu.float(), logvar.float()
        if self.loss == "bce":
            recon = V.bce_recon_term(self.x, x_rec)
        else:
            recon = V.cosine_recon_term(self.x, x_rec)
        kl = V.kl_term(mu, logvar)
        total = recon + self.beta * kl
        total.backward()
        self.opt.step()
        return total.detach(), recon.detach(), kl.detach()

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
        with torch.cuda.graph(self.graph):
            self.out = self._body()
        if not self.restore:
            return
        with torch.no_grad():
            for k, v in self.module.state_dict().items():
                v.copy_(saved[k])
            for st in self.opt.state.values():  # fresh Adam moments and step counters
                for t in st.values():
                    if torch.is_tensor(t):
                        t.zero_()

    def step(self, x: torch.Tensor | None = None):
        """Run one training step on ``x`` (copied into the static batch buffer);
        returns device tensors (loss, recon, kl)."""
        if x is not None:
            self.x.copy_(x, non_blocking=True)
        if self.graph is not None:
            self.graph.replay()
            return self.out
        self.model.train()
        return self._body()
