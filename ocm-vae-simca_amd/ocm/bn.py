"""Training-mode BatchNorm1d on libocm (ocm_bn_fwd_train / ocm_bn_bwd).

``FastBatchNorm1d`` is an ``nn.BatchNorm1d`` (same parameters, buffers and
state_dict keys — vae_model.py:45-47, 75-77 build plain ``nn.BatchNorm1d``)
whose training-mode forward on a HIP device runs the split-reduction kernels
of csrc/ocm_bn.hip instead of MIOpen's spatial BN, which handles the VAE's
3-12-channel × 512-2048-position activations at a few GB/s.  Evaluation mode
(running statistics) and host tensors use the stock module.  The kernels
launch on the current stream, so the module is HIP-graph capturable
(ocm/vae_train.py); their reduction scratch is caller-owned: one zero-filled
buffer per module (``_layer_scratch``), reused by every call — the kernels'
per-channel completion counters live at its end and every call leaves them
zero, so each direction is one reduction launch plus the elementwise pass.

``fuse_elu()`` folds the ELU that follows every batch norm of the VAE
(vae_model.py:45-49, 75-79) into the same kernels: the normalisation pass
writes ELU(z), and the backward passes form the ELU's input gradient from
the saved output on the fly (two elementwise kernels fewer per layer and
direction).  ConvVAE1D then puts an ``nn.Identity`` where the ELU module was,
so parameters and state_dict keys do not move.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

from . import _lib
from ._lib import Context, check, ptr, stream_handle

_DT = {torch.float32: 0, torch.bfloat16: 1}
ACT_NONE, ACT_ELU = 0, 1  # include/ocm.h OCM_ACT_*


def _layer_scratch(mod, C: int, dev) -> torch.Tensor:
    """The module's reduction scratch (include/ocm.h ocm_bn_scratch_bytes):
    zero-filled once, then reused by its forward and backward calls, which
    are stream-ordered.  A plain attribute, not a buffer: state_dict keys do
    not move.  Allocated on the first (eager) call, before any graph capture,
    so a captured replay writes through a pointer that stays put."""
    nbytes = int(_lib.load().ocm_bn_scratch_bytes(C))
    buf = mod.__dict__.get("_ocm_scratch")
    if buf is None or buf.device != dev or buf.numel() * 8 < nbytes:
        buf = torch.zeros((nbytes + 7) // 8, dtype=torch.float64, device=dev)
        mod.__dict__["_ocm_scratch"] = buf
    return buf


class _BNTrain(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, nbt, eps, momentum, act, scratch):
        x = x.contiguous()
        N, C, L = x.shape
        dev = x.device
        y = torch.empty_like(x)
        smean = torch.empty(C, dtype=torch.float32, device=dev)
        sinv = torch.empty(C, dtype=torch.float32, device=dev)
        w = weight.detach().float().contiguous() if weight is not None else None
        b = bias.detach().float().contiguous() if bias is not None else None
        h = Context.get(dev.index).handle
        check(_lib.load().ocm_bn_fwd_train(h, _DT[x.dtype], ptr(x), N, C, L, ptr(w), ptr(b), float(eps),
                                           float(momentum), ptr(running_mean), ptr(running_var), ptr(nbt), act,
                                           ptr(y), ptr(smean), ptr(sinv), ptr(scratch), stream_handle(dev)),
              "ocm_bn_fwd_train")
        ctx.act = act
        ctx.scratch = scratch
        ctx.save_for_backward(x, w, smean, sinv, y if act else None)
        ctx.has_w, ctx.has_b = weight is not None, bias is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w, smean, sinv, y = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        N, C, L = x.shape
        dev = x.device
        dx = torch.empty_like(x)
        dw = torch.empty(C, dtype=torch.float32, device=dev) if ctx.has_w else None
        db = torch.empty(C, dtype=torch.float32, device=dev) if ctx.has_b else None
        h = Context.get(dev.index).handle
        check(_lib.load().ocm_bn_bwd(h, _DT[x.dtype], ptr(x), ptr(dy), N, C, L, ptr(w), ptr(smean), ptr(sinv),
                                     ctx.act, ptr(y), ptr(dx), ptr(dw), ptr(db), ptr(ctx.scratch),
                                     stream_handle(dev)),
              "ocm_bn_bwd")
        return dx, dw, db, None, None, None, None, None, None, None


class FastBatchNorm1d(nn.BatchNorm1d):
    """nn.BatchNorm1d with the libocm training-mode kernels on HIP tensors
    (and, after ``fuse_elu()``, the ELU that follows it)."""

    act = ACT_NONE

    def fuse_elu(self):
        self.act = ACT_ELU
        return self

    def forward(self, x):
        if (not self.training and x.is_cuda and x.dim() == 3 and x.dtype in _DT and self.track_running_stats
                and self.running_mean is not None and self.running_mean.dtype == torch.float32
                and not (torch.is_grad_enabled()
                         and (x.requires_grad or (self.affine and self.weight.requires_grad)))):
            # eval with running statistics and no autograd (the latent encoding):
            # one libocm launch (MIOpen's inference kernel: 3.3 ms per 8192-row batch)
            x = x.contiguous()
            y = torch.empty_like(x)
            N, C, L = x.shape
            w = self.weight if self.affine else None
            b = self.bias if self.affine else None
            check(_lib.load().ocm_bn_fwd_eval(Context.get(x.device.index).handle, _DT[x.dtype], ptr(x), N, C, L,
                                              ptr(self.running_mean), ptr(self.running_var), float(self.eps),
                                              ptr(w) if w is not None else None, ptr(b) if b is not None else None,
                                              self.act, ptr(y), stream_handle(x.device)), "ocm_bn_fwd_eval")
            return y
        if not (self.training and x.is_cuda and x.dim() == 3 and x.dtype in _DT) or self.momentum is None:
            # eval (running statistics), host tensors, cumulative-average momentum: the stock module
            y = super().forward(x)
            return F.elu(y) if self.act == ACT_ELU else y
        # the batch count is incremented by the statistics kernel (one launch fewer)
        nbt = (self.num_batches_tracked if self.track_running_stats and self.num_batches_tracked is not None
               and self.num_batches_tracked.dtype == torch.int64 and self.num_batches_tracked.is_cuda else None)
        if self.track_running_stats and self.num_batches_tracked is not None and nbt is None:
            self.num_batches_tracked.add_(1)
        momentum = self.momentum
        track = self.track_running_stats and self.running_mean is not None
        scratch = _layer_scratch(self, x.shape[1], x.device)
        return _BNTrain.apply(x, self.weight, self.bias, self.running_mean if track else None,
                              self.running_var if track else None, nbt, self.eps, momentum, self.act, scratch)
