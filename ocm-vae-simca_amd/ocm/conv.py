"""Narrow Conv1d / ConvTranspose1d on libocm (ocm_conv1d / ocm_conv1d_wgrad).

``FastConv1d`` and ``FastConvTranspose1d`` are ``nn.Conv1d`` /
``nn.ConvTranspose1d`` (same parameters and state_dict keys — vae_model.py:
37-81 builds the stock modules) whose forward on a HIP device, for the VAE's
shapes (≤ 64 channels, kernel ≤ 15, no groups or dilation, zero padding), runs
the direct kernels of csrc/ocm_conv.hip instead of MIOpen's implicit GEMMs and
layout transposes (36 % of the graphed C4 step, profiles/r03g_vae_step_trace.md).
Under bf16 autocast the activations are bf16, as torch's autocast conv would
make them; the weights stay float32 (torch would round them to bf16 first) and
every sum is float32.  Other shapes, host tensors and bf16 weights take the
stock module.  All launches are on the current stream with caller-owned
scratch — one zero-filled buffer per module, reused by every backward call
(the reductions' completion counters live in it and every call leaves them
zero) — so the modules are HIP-graph capturable (ocm/vae_train.py).
"""
from __future__ import annotations

import torch
from torch import nn

from . import _lib
from ._lib import Context, check, ptr, stream_handle

_DT = {torch.float32: 0, torch.bfloat16: 1}
DOWN, UP = 0, 1  # include/ocm.h OCM_CONV_DOWN / OCM_CONV_UP
# ConvTranspose1d's bias gradient inside the weight-gradient launch
# (ocm_conv1d_wgrad_qsum); False: ocm_conv1d_wgrad + ocm_chan_sum (A/B runs,
# scripts/vae_ab.py)
QSUM_FUSED = True


def _layer_scratch(mod, O: int, I: int, K: int, dev) -> torch.Tensor:
    """The module's wgrad / bias-sum scratch (include/ocm.h
    ocm_conv1d_scratch_bytes): zero-filled once, reused by its stream-ordered
    backward calls; a plain attribute (state_dict keys do not move)."""
    nbytes = int(_lib.load().ocm_conv1d_scratch_bytes(O, I, K))
    buf = mod.__dict__.get("_ocm_scratch")
    if buf is None or buf.device != dev or buf.numel() * 4 < nbytes:
        buf = torch.zeros((nbytes + 3) // 4, dtype=torch.float32, device=dev)
        mod.__dict__["_ocm_scratch"] = buf
    return buf


def _launch(mode, x, w, bias, O, Lout, K, stride, pad, out_dtype):
    B, I, Lin = x.shape
    y = torch.empty((B, O, Lout), dtype=out_dtype, device=x.device)
    check(_lib.load().ocm_conv1d(Context.get(x.device.index).handle, mode, _DT[x.dtype], ptr(x), B, I, Lin, ptr(w),
                                 ptr(bias), O, Lout, K, stride, pad, _DT[out_dtype], ptr(y), stream_handle(x.device)),
          "ocm_conv1d")
    return y


class _ConvFn(torch.autograd.Function):
    """y = conv (transposed=False, weight [O][I][K]) or transposed conv
    (transposed=True, weight [I][O][K]) of x (B, I, Lin)."""

    @staticmethod
    def forward(ctx, x, weight, bias, stride, pad, transposed, Lout, out_dtype, scratch):
        x = x.contiguous()
        w = weight.detach().contiguous()
        b = bias.detach().contiguous() if bias is not None else None
        K = w.shape[2]
        O = w.shape[1] if transposed else w.shape[0]
        y = _launch(UP if transposed else DOWN, x, w, b, O, Lout, K, stride, pad, out_dtype)
        ctx.save_for_backward(x, w)
        ctx.conf = (stride, pad, transposed, bias is not None)
        ctx.scratch = scratch
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        stride, pad, transposed, has_bias = ctx.conf
        dy = dy.contiguous()
        if dy.dtype not in _DT:
            dy = dy.float()
        B, I, Lin = x.shape
        _, O, Lout = dy.shape
        K = w.shape[2]
        dev = x.device
        h = Context.get(dev.index).handle
        st = stream_handle(dev)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            # the adjoint pass: Conv1d's input gradient is the "up" form of dy with
            # its [O][I][K] weight; ConvTranspose1d's is the "down" form
            dx = _launch(DOWN if transposed else UP, dy, w, None, I, Lin, K, stride, pad, x.dtype)
        want_db = has_bias and ctx.needs_input_grad[2]
        if ctx.needs_input_grad[1] or want_db:
            scratch = ctx.scratch
            db = torch.empty(O, dtype=torch.float32, device=dev) if want_db else None
            dw = torch.empty_like(w)
            lib = _lib.load()
            if transposed:  # dW[i][o][t] = Σ x[b][i][l] · dy[b][o][l·s + t − pad]; db = Σ dy (a ones row of P
                # in the same matrix-core launch when the taps cover dy once, else ocm_chan_sum after it)
                args = (_DT[x.dtype], ptr(x), I, Lin, _DT[dy.dtype], ptr(dy), O, Lout, B, K, stride, pad, ptr(dw))
                if want_db and QSUM_FUSED:
                    check(lib.ocm_conv1d_wgrad_qsum(h, *args, ptr(db), ptr(scratch), st), "ocm_conv1d_wgrad_qsum")
                else:
                    check(lib.ocm_conv1d_wgrad(h, *args, None, ptr(scratch), st), "ocm_conv1d_wgrad")
                    if want_db:
                        check(lib.ocm_chan_sum(h, _DT[dy.dtype], ptr(dy), B, O, Lout, ptr(db), ptr(scratch), st),
                              "ocm_chan_sum")
            else:  # dW[o][i][t] = Σ dy[b][o][l] · x[b][i][l·s + t − pad], db = Σ dy in the same pass
                args = (_DT[dy.dtype], ptr(dy), O, Lout, _DT[x.dtype], ptr(x), I, Lin, B, K, stride, pad, ptr(dw),
                        ptr(db))
                check(lib.ocm_conv1d_wgrad(h, *args, ptr(scratch), st), "ocm_conv1d_wgrad")
            if not ctx.needs_input_grad[1]:
                dw = None
        return dx, dw, db, None, None, None, None, None, None


def _fast_ok(mod, x) -> bool:
    return (x.is_cuda and x.dim() == 3 and x.dtype in _DT and mod.weight.dtype == torch.float32
            and (mod.bias is None or mod.bias.dtype == torch.float32) and mod.groups == 1
            and mod.dilation == (1,) and mod.padding_mode == "zeros" and not isinstance(mod.padding, str)
            and max(mod.in_channels, mod.out_channels) <= 64 and mod.kernel_size[0] <= 15)


def _act_dtype(x):
    if torch.is_autocast_enabled("cuda"):
        dt = torch.get_autocast_dtype("cuda")
        return dt if dt in _DT else x.dtype
    return x.dtype


class FastConv1d(nn.Conv1d):
    """nn.Conv1d with libocm's direct kernels for the VAE's narrow shapes."""

    def forward(self, x):
        if not _fast_ok(self, x):
            return super().forward(x)
        K, s, pad = self.kernel_size[0], self.stride[0], self.padding[0]
        Lout = (x.shape[-1] + 2 * pad - K) // s + 1
        scratch = _layer_scratch(self, self.out_channels, self.in_channels, K, x.device)
        return _ConvFn.apply(x, self.weight, self.bias, s, pad, False, Lout, _act_dtype(x), scratch)


class FastConvTranspose1d(nn.ConvTranspose1d):
    """nn.ConvTranspose1d with libocm's direct kernels for the VAE's narrow shapes."""

    def forward(self, x, output_size=None):
        if output_size is not None or not _fast_ok(self, x):
            return super().forward(x, output_size)
        K, s, pad, op = self.kernel_size[0], self.stride[0], self.padding[0], self.output_padding[0]
        Lout = (x.shape[-1] - 1) * s - 2 * pad + K + op
        scratch = _layer_scratch(self, self.in_channels, self.out_channels, K, x.device)
        return _ConvFn.apply(x, self.weight, self.bias, s, pad, True, Lout, _act_dtype(x), scratch)
