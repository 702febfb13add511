"""The VAE training step's small tensors on libocm (csrc/ocm_vaestep.hip).

The graphed C4 step (ocm/vae_train.py) is bound by its kernel count: every
torch elementwise / reduction kernel costs ≈ 4.5 µs of the replay however
small its tensor (profiles/r03n_vae_step_trace_by_grid.md: 192 kernels, ≈ 80
of them torch's).  The reference's step (vae_bce_nut.py:178-203 with
vae_model.py:124-158) is restated here as three autograd functions and one
optimizer kernel:

* ``bottleneck(mu, logvar, eps)`` → (z, kl): z = μ + ε·exp(½logσ²)
  (reparameterize, vae_model.py:124-126) and the KL term (vae_model.py:150-152)
  in one launch, their backward in one launch;
* ``recon_total(x, xs, kl, ...)`` → (total, recon): the de-standardisation
  x̂ = xs·std + mean (forward, vae_model.py:130-134), the reconstruction term
  (BCE-with-logits against the per-sample min–max scaled input,
  vae_model.py:153-156, or the MSE of utils/final_vaesimca.py:208-209) and
  total = recon + β·kl in one launch; the backward is one launch;
* ``FusedAdam``: torch.optim.Adam (L2 weight decay) over every parameter in
  one launch (ocm_adam_step), with its moments and step counter on the device.

* ``cast_bf16(*params)``: the Linear layers' float32 weights and biases to
  bfloat16 in one launch per step (autocast would cast each one, and cast each
  bfloat16 gradient back, in a kernel of its own: 20 launches per step), and
  their bfloat16 gradients back to float32 in one launch (ocm_cast_multi);
* ``standardise(x, mean, std)``: the encoder's input (x − mean)/std in bf16,
  one launch (vae_model.py:128-129).

ε is drawn with torch.randn_like on the graph-safe generator, exactly as the
model's reparameterize draws it.  Sums are fp64 with fixed-order partials.
"""
from __future__ import annotations

import ctypes

import torch

from . import _lib
from ._lib import Context, check, ptr, stream_handle

_DT = {torch.float32: 0, torch.bfloat16: 1}
LOSS_KINDS = {"bce": 0, "euclidean": 1}  # include/ocm.h OCM_VAE_LOSS_*


def _h(dev):
    return Context.get(dev.index).handle


_BSCRATCH = {}


def _bottleneck_scratch(dev) -> torch.Tensor:
    """The KL reduction's scratch (ocm_vae_bottleneck_scratch_bytes), one per
    device, zero-filled once (its completion counters are left zero; the
    step's launches are stream-ordered).  Allocated by the first, eager, call."""
    key = dev.index
    if key not in _BSCRATCH:
        nb = int(_lib.load().ocm_vae_bottleneck_scratch_bytes())
        _BSCRATCH[key] = torch.zeros((nb + 7) // 8, dtype=torch.float64, device=dev)
    return _BSCRATCH[key]


class _Bottleneck(torch.autograd.Function):
    @staticmethod
    def forward(ctx, mu, logvar, eps):
        mu, logvar, eps = mu.contiguous(), logvar.contiguous(), eps.contiguous()
        B, d = mu.shape
        z = torch.empty_like(mu)
        kl = torch.empty((), dtype=torch.float32, device=mu.device)
        check(_lib.load().ocm_vae_bottleneck_fwd(_h(mu.device), _DT[mu.dtype], ptr(mu), ptr(logvar), ptr(eps), B, d,
                                                 ptr(z), ptr(kl), ptr(_bottleneck_scratch(mu.device)),
                                                 stream_handle(mu.device)), "ocm_vae_bottleneck_fwd")
        ctx.save_for_backward(mu, logvar, eps)
        ctx.set_materialize_grads(False)
        return z, kl

    @staticmethod
    def backward(ctx, dz, dkl):
        mu, logvar, eps = ctx.saved_tensors
        B, d = mu.shape
        dmu, dlv = torch.empty_like(mu), torch.empty_like(logvar)
        if dz is not None:
            dz = dz.to(mu.dtype).contiguous()
        if dkl is not None:
            dkl = dkl.to(torch.float32).contiguous()
        check(_lib.load().ocm_vae_bottleneck_bwd(_h(mu.device), _DT[mu.dtype], ptr(dz), ptr(dkl), ptr(mu),
                                                 ptr(logvar), ptr(eps), B, d, ptr(dmu), ptr(dlv),
                                                 stream_handle(mu.device)), "ocm_vae_bottleneck_bwd")
        return dmu, dlv, None


class _BottleneckPacked(torch.autograd.Function):
    """_Bottleneck on the packed B×2d output of one [fc_mu; fc_logvar] product
    (μ = ml[:, :d], logσ² = ml[:, d:], read in place: no copies), whose
    gradient is written packed the same way (ocm_vae_bottleneck_*_ld)."""

    @staticmethod
    def forward(ctx, ml, eps):
        ml, eps = ml.contiguous(), eps.contiguous()
        B, d2 = ml.shape
        d = d2 // 2
        z = torch.empty((B, d), dtype=ml.dtype, device=ml.device)
        kl = torch.empty((), dtype=torch.float32, device=ml.device)
        off = d * ml.element_size()
        check(_lib.load().ocm_vae_bottleneck_fwd_ld(_h(ml.device), _DT[ml.dtype], ptr(ml), ptr(ml) + off, d2, ptr(eps),
                                                    B, d, ptr(z), ptr(kl), ptr(_bottleneck_scratch(ml.device)),
                                                    stream_handle(ml.device)), "ocm_vae_bottleneck_fwd_ld")
        ctx.save_for_backward(ml, eps)
        ctx.set_materialize_grads(False)
        return z, kl

    @staticmethod
    def backward(ctx, dz, dkl):
        ml, eps = ctx.saved_tensors
        B, d2 = ml.shape
        d = d2 // 2
        dml = torch.empty_like(ml)
        if dz is not None:
            dz = dz.to(ml.dtype).contiguous()
        if dkl is not None:
            dkl = dkl.to(torch.float32).contiguous()
        off = d * ml.element_size()
        check(_lib.load().ocm_vae_bottleneck_bwd_ld(_h(ml.device), _DT[ml.dtype], ptr(dz), ptr(dkl), ptr(ml),
                                                    ptr(ml) + off, d2, ptr(eps), B, d, ptr(dml), ptr(dml) + off,
                                                    stream_handle(ml.device)), "ocm_vae_bottleneck_bwd_ld")
        return dml, None


class _ReconTotal(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, xs, kl, bufs, kind, beta, eps):
        xs = xs.contiguous()
        B, L = xs.shape
        gxs, out2, scratch, mean, std = bufs.get(B, L, x.device)
        check(_lib.load().ocm_vae_recon_fwd(_h(x.device), kind, ptr(x), _DT[xs.dtype], ptr(xs), B, L, ptr(mean),
                                            ptr(std), float(eps), ptr(kl), float(beta), ptr(gxs), ptr(out2),
                                            ptr(scratch), stream_handle(x.device)), "ocm_vae_recon_fwd")
        ctx.xs_dtype = xs.dtype
        ctx.beta = float(beta)
        ctx.gxs = gxs
        ctx.has_kl = kl is not None
        ctx.set_materialize_grads(False)
        return out2[0]  # total; recon stays in bufs (out2[1])

    @staticmethod
    def backward(ctx, dtotal):
        gxs = ctx.gxs
        B, L = gxs.shape
        if dtotal is None:
            return None, None, None, None, None, None, None
        dtotal = dtotal.to(torch.float32).contiguous()
        dxs = torch.empty((B, L), dtype=ctx.xs_dtype, device=gxs.device)
        dkl = torch.empty((), dtype=torch.float32, device=gxs.device) if ctx.has_kl else None
        check(_lib.load().ocm_vae_recon_bwd(_h(gxs.device), ptr(dtotal), ptr(gxs), B * L, _DT[ctx.xs_dtype], ptr(dxs),
                                            ctx.beta, ptr(dkl), stream_handle(gxs.device)), "ocm_vae_recon_bwd")
        return None, dxs, dkl, None, None, None, None


class ReconBuffers:
    """Persistent device buffers of the fused reconstruction term (graph
    replays reuse them): the gradient d recon / d xs, {total, recon}, the
    ticket scratch (zeroed once), and the model's mean / std."""

    def __init__(self, spec_mean: torch.Tensor, spec_std: torch.Tensor):
        self.mean = spec_mean.detach().to(torch.float32).contiguous()
        self.std = spec_std.detach().to(torch.float32).contiguous()
        self._b = {}

    def get(self, B, L, dev):
        key = (B, L)
        if key not in self._b:
            nb = int(_lib.load().ocm_vae_scratch_bytes(B))
            self._b[key] = (torch.empty((B, L), dtype=torch.float32, device=dev),
                            torch.empty(2, dtype=torch.float32, device=dev),
                            torch.zeros((nb + 7) // 8, dtype=torch.float64, device=dev))
        gxs, out2, scratch = self._b[key]
        return gxs, out2, scratch, self.mean, self.std


def bottleneck(mu, logvar, eps):
    return _Bottleneck.apply(mu, logvar, eps)


def bottleneck_packed(ml, eps):
    """(z, kl) from the packed [μ | logσ²] rows of ``ml`` (B×2d)."""
    return _BottleneckPacked.apply(ml, eps)


def recon_total(x, xs, kl, bufs: ReconBuffers, loss: str, beta: float, eps: float = 1e-8):
    """(total, recon): total carries the gradient; recon is the term's value."""
    total = _ReconTotal.apply(x, xs, kl, bufs, LOSS_KINDS[loss], float(beta), float(eps))
    return total, bufs.get(xs.shape[0], xs.shape[1], xs.device)[1][1]


class FusedAdam:
    """torch.optim.Adam (L2 weight decay, no amsgrad) over ``params`` in one
    launch per step (ocm_adam_step).  The table of (param, grad, moments)
    pointers is written when the gradients' addresses change (eager steps);
    a step captured into a HIP graph keeps the table of its capture."""

    _FIELDS = [("param", ctypes.c_void_p), ("grad", ctypes.c_void_p), ("exp_avg", ctypes.c_void_p),
               ("exp_avg_sq", ctypes.c_void_p), ("offset", ctypes.c_int64), ("numel", ctypes.c_int64)]

    class _Entry(ctypes.Structure):
        pass

    _Entry._fields_ = _FIELDS

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0):
        self.params = [p for p in params if p.requires_grad]
        dev = self.params[0].device
        self.lr, self.b1, self.b2, self.eps, self.wd = float(lr), float(betas[0]), float(betas[1]), float(eps), \
            float(weight_decay)
        self.exp_avg = [torch.zeros_like(p, memory_format=torch.contiguous_format) for p in self.params]
        self.exp_avg_sq = [torch.zeros_like(p, memory_format=torch.contiguous_format) for p in self.params]
        self.step_t = torch.zeros((), dtype=torch.float32, device=dev)
        self.total = sum(p.numel() for p in self.params)
        n = len(self.params)
        self.table = torch.empty(n * ctypes.sizeof(self._Entry), dtype=torch.uint8, device=dev)
        # completion counters of the two-level last-arrival (ocm_adam_step)
        self.scratch = torch.zeros((int(_lib.load().ocm_vae_scratch_bytes(4096)) + 3) // 4, dtype=torch.int32,
                                   device=dev)
        self._key = None

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def _write_table(self, capturing: bool):
        """Entries for the parameters that have a gradient this step; like
        torch.optim.Adam, a parameter whose .grad is None is skipped (its
        moments are left alone).  The step counter is shared, so a parameter
        skipped on some steps sees the optimizer's step count in its bias
        correction, not its own (torch keeps one per parameter)."""
        key = tuple(p.grad.data_ptr() if p.grad is not None else None for p in self.params)
        if key == self._key:
            return
        live = [i for i, p in enumerate(self.params) if p.grad is not None]
        arr = (self._Entry * max(len(live), 1))()
        o = 0
        for j, i in enumerate(live):
            p = self.params[i]
            if not (p.is_contiguous() and p.grad.is_contiguous() and p.grad.dtype == torch.float32):
                raise RuntimeError("FusedAdam: contiguous float32 parameters and gradients only")
            arr[j] = self._Entry(p.data_ptr(), p.grad.data_ptr(), self.exp_avg[i].data_ptr(),
                                 self.exp_avg_sq[i].data_ptr(), o, p.numel())
            o += p.numel()
        self._n_live, self._total_live = len(live), o
        raw = torch.frombuffer(bytearray(arr), dtype=torch.uint8)
        if capturing:  # written once after the capture (the graph replays the capture's addresses)
            self._pending = raw.clone()
        else:  # eager steps: a synchronous copy (the host staging is reused next step)
            self.table[:raw.numel()].copy_(raw.to(self.table.device))
        self._key = key

    def flush_pending(self):
        """After a graph capture: the table of the captured step's gradients."""
        if getattr(self, "_pending", None) is not None:
            self.table[:self._pending.numel()].copy_(self._pending.to(self.table.device))
            torch.cuda.synchronize(self.table.device)
            self._pending = None

    def step(self):
        capturing = torch.cuda.is_current_stream_capturing()
        self._write_table(capturing)
        if self._n_live == 0:
            return
        dev = self.table.device
        check(_lib.load().ocm_adam_step(_h(dev), ptr(self.table), self._n_live, self._total_live, ptr(self.step_t),
                                        self.lr, self.b1, self.b2, self.eps, self.wd, ptr(self.scratch),
                                        stream_handle(dev)), "ocm_adam_step")

    def reset_state(self):
        for t in self.exp_avg + self.exp_avg_sq:
            t.zero_()
        self.step_t.zero_()


def _cast_multi(srcs, dsts, sdt, ddt, dev):
    n = len(srcs)
    src = (ctypes.c_void_p * n)(*[t.data_ptr() for t in srcs])
    dst = (ctypes.c_void_p * n)(*[t.data_ptr() for t in dsts])
    numel = (ctypes.c_int64 * n)(*[t.numel() for t in srcs])
    check(_lib.load().ocm_cast_multi(_h(dev), n, src, sdt, dst, ddt, numel, stream_handle(dev)), "ocm_cast_multi")


class _CastBF16(torch.autograd.Function):
    """float32 parameters → bfloat16 copies (one launch); the backward turns
    their bfloat16 gradients into float32 ones (one launch) and returns them,
    so autograd accumulates them into .grad like any gradient.  Only when the
    caller says every .grad is a freshly zeroed view (``into_zeroed_grads``:
    the data-parallel step zeroes its flat all-reduce buffer first) are they
    written straight into the views instead (no accumulate kernel); that
    equals accumulation because the views hold zeros."""

    @staticmethod
    def forward(ctx, into_zeroed_grads, *params):
        # one flat bf16 buffer: the matrices first, then the vectors, each in
        # the given order and 16-B aligned, so the weights (and the biases) of
        # consecutive layers sit back to back (linear_cat reads [fc_mu; fc_logvar]
        # as one operand without a copy)
        order = [i for i, p in enumerate(params) if p.dim() > 1] + [i for i, p in enumerate(params) if p.dim() <= 1]
        offs, o = [0] * len(params), 0
        for i in order:
            offs[i] = o
            o += (params[i].numel() + 7) // 8 * 8
        flat = torch.empty(max(o, 1), dtype=torch.bfloat16, device=params[0].device)
        outs = [flat[offs[i]:offs[i] + p.numel()].view(p.shape) for i, p in enumerate(params)]
        _cast_multi([p.detach().contiguous() for p in params], outs, _DT[torch.float32], _DT[torch.bfloat16],
                    params[0].device)
        ctx.params = params
        ctx.into_zeroed = bool(into_zeroed_grads)
        ctx.set_materialize_grads(False)
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        params = ctx.params
        live = [(p, g) for p, g in zip(params, grads) if g is not None]
        if not live:
            return (None,) * (len(params) + 1)
        into_views = ctx.into_zeroed and all(p.grad is not None and p.grad.is_contiguous() for p, _ in live)
        outs = [p.grad if into_views else torch.empty_like(p, memory_format=torch.contiguous_format)
                for p, _ in live]
        _cast_multi([g.contiguous() for _, g in live], outs, _DT[torch.bfloat16], _DT[torch.float32],
                    params[0].device)
        if into_views:
            return (None,) * (len(params) + 1)
        res, k = [None], 0
        for g in grads:
            if g is None:
                res.append(None)
            else:
                res.append(outs[k])
                k += 1
        return tuple(res)


def cast_bf16(*params, into_zeroed_grads: bool = False):
    """bf16 copies of ``params``; see _CastBF16 for ``into_zeroed_grads``."""
    return _CastBF16.apply(into_zeroed_grads, *params)


_SKSCRATCH = {}
# _LinearAct's forward for K ≤ 256 with its ELU through ocm_vae_linear_act
# (False: hipBLASLt + torch's elu; A/B runs, scripts/vae_ab.py)
LINEAR_ACT_FUSED = True
SK_MIN_K = 2048  # the split-K GEMM takes products at least this deep (hipBLASLt: the rest)


def _sk_ok(M, N, K, *ts) -> bool:
    return (M % 64 == 0 and N % 64 == 0 and K % 256 == 0 and K >= SK_MIN_K
            and all(t.dtype == torch.bfloat16 and t.is_contiguous() for t in ts))


def gemm_sk(A: torch.Tensor, B: torch.Tensor, b_nk: bool, bias: torch.Tensor | None = None) -> torch.Tensor:
    """A·Bᵀ (``b_nk``: B is N×K, a Linear weight) or A·B (B is K×N), + bias, in
    bf16 with float32 accumulation, split over K (ocm_gemm_bf16_sk).  The float32
    partials live in a per-shape scratch buffer that is never freed (a captured
    step graph keeps its pointer)."""
    M, K = A.shape
    N = B.shape[0] if b_nk else B.shape[1]
    key = (A.device.index, M, N, K)
    buf = _SKSCRATCH.get(key)
    if buf is None:
        nb = int(_lib.load().ocm_gemm_bf16_sk_scratch_bytes(M, N, K))
        buf = _SKSCRATCH[key] = torch.empty((nb + 3) // 4, dtype=torch.float32, device=A.device)
    C = torch.empty((M, N), dtype=torch.bfloat16, device=A.device)
    check(_lib.load().ocm_gemm_bf16_sk(_h(A.device), 1 if b_nk else 0, ptr(A), ptr(B), ptr(bias), M, N, K, ptr(C),
                                       ptr(buf), stream_handle(A.device)), "ocm_gemm_bf16_sk")
    return C


class _LinearAct(torch.autograd.Function):
    """y = x·Wᵀ + b (→ ELU when ``act``) on bf16 tensors, for the bottleneck's
    Linear layers (vae_model.py:80-84: fc, fc_mu, fc_logvar, fc_dec).  The
    forward is hipBLASLt with its bias epilogue and torch's ELU; the backward
    forms gy = g·elu'(y) and the bias gradient in one libocm launch
    (ocm_vae_act_bias_bwd) instead of torch's elu_backward and column-sum
    kernels, then the weight gradient (hipBLASLt) and the input gradient
    (gemm_sk for fc_dec[3]'s K = 6144, else hipBLASLt)."""

    @staticmethod
    def forward(ctx, x, W, b, act):
        ctx.act = bool(act)
        M, K = x.shape
        N = W.shape[0]
        if (act and LINEAR_ACT_FUSED and x.dtype == W.dtype == torch.bfloat16 and K in (32, 64, 128, 256)
                and M % 64 == 0 and N % 64 == 0 and x.is_contiguous() and W.is_contiguous()
                and (b is None or (b.dtype == torch.bfloat16 and b.is_contiguous()))
                and x.data_ptr() % 16 == 0 and W.data_ptr() % 16 == 0):
            # fc_dec's short-K layers: GEMM + bias + ELU in one launch (ocm_vae_linear_act)
            y = torch.empty((M, N), dtype=x.dtype, device=x.device)
            a = torch.empty_like(y)
            check(_lib.load().ocm_vae_linear_act(_h(x.device), ptr(x), ptr(W), ptr(b), M, N, K, ptr(y), ptr(a),
                                                 stream_handle(x.device)), "ocm_vae_linear_act")
            ctx.save_for_backward(x, W, y)
            return a
        # (fc[0]'s K = 6144 forward through gemm_sk measured 7.7 + 9.1 µs against
        # hipBLASLt's 8.5: hipBLASLt keeps the forward, profiles/r06zg_vae_step_trace.md)
        y = torch.addmm(b, x, W.t()) if b is not None else x.mm(W.t())
        ctx.save_for_backward(x, W, y if act else None)
        return torch.nn.functional.elu(y) if act else y

    @staticmethod
    def backward(ctx, ga):
        x, W, y = ctx.saved_tensors
        ga = ga.contiguous()
        B, N = ga.shape
        if ga.dtype == torch.bfloat16 and N % 8 == 0:
            gb = torch.empty(N, dtype=ga.dtype, device=ga.device)
            gy = torch.empty_like(ga) if ctx.act else ga
            check(_lib.load().ocm_vae_act_bias_bwd(_h(ga.device), 1 if ctx.act else 0, ptr(ga),
                                                   ptr(y) if ctx.act else None, B, N, ptr(gy) if ctx.act else None,
                                                   ptr(gb), stream_handle(ga.device)), "ocm_vae_act_bias_bwd")
        else:  # (other dtypes / widths: torch's kernels, the same arithmetic)
            gy = torch.ops.aten.elu_backward(ga, 1.0, 1.0, 1.0, False, y) if ctx.act else ga
            gb = gy.sum(0)
        gx = None
        if ctx.needs_input_grad[0]:  # fc_dec[3]: K = 6144 (vae_model.py:83)
            gx = gemm_sk(gy, W, False) if _sk_ok(B, W.shape[1], N, gy, W) else gy.mm(W)
        gW = gy.t().mm(x) if ctx.needs_input_grad[1] else None
        return gx, gW, gb if ctx.needs_input_grad[2] else None, None


def _bias_grad(g: torch.Tensor) -> torch.Tensor:
    """Σ_rows g (ocm_vae_act_bias_bwd with act 0) for a bf16 B×N gradient."""
    g = g.contiguous()
    B, N = g.shape
    if g.dtype != torch.bfloat16 or N % 8:
        return g.sum(0)
    gb = torch.empty(N, dtype=g.dtype, device=g.device)
    check(_lib.load().ocm_vae_act_bias_bwd(_h(g.device), 0, ptr(g), None, B, N, None, ptr(gb),
                                           stream_handle(g.device)), "ocm_vae_act_bias_bwd")
    return gb


class _LinearPair(torch.autograd.Function):
    """(x·W1ᵀ + b1, x·W2ᵀ + b2) for two Linear layers on one input (fc_mu and
    fc_logvar on h, vae_model.py:81-82): the input gradient is one GEMM plus
    one accumulating GEMM (addmm, β = 1) instead of two GEMMs and autograd's
    add kernel."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2):
        ctx.save_for_backward(x, W1, W2)
        return torch.addmm(b1, x, W1.t()), torch.addmm(b2, x, W2.t())

    @staticmethod
    def backward(ctx, g1, g2):
        x, W1, W2 = ctx.saved_tensors
        g1 = x.new_zeros((x.shape[0], W1.shape[0])) if g1 is None else g1.contiguous()
        g2 = x.new_zeros((x.shape[0], W2.shape[0])) if g2 is None else g2.contiguous()
        gx = g1.mm(W1).addmm_(g2, W2) if ctx.needs_input_grad[0] else None  # (in place: no copy of the first)
        return gx, g1.t().mm(x), _bias_grad(g1), g2.t().mm(x), _bias_grad(g2)


def _adjacent(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """[a; b] along dim 0: a view when b follows a in memory, else torch.cat."""
    if (a.is_contiguous() and b.is_contiguous() and a.dtype == b.dtype and a.shape[1:] == b.shape[1:]
            and b.data_ptr() == a.data_ptr() + a.numel() * a.element_size()):
        return torch.as_strided(a, (a.shape[0] + b.shape[0],) + tuple(a.shape[1:]), a.stride())
    return torch.cat([a, b])


class _LinearCat(torch.autograd.Function):
    """x·[W1; W2]ᵀ + [b1; b2] as ONE product (fc_mu and fc_logvar on one input,
    vae_model.py:81-82): one GEMM forward; backward one input-gradient GEMM,
    one weight-gradient GEMM and one bias sum for both layers (_LinearPair
    needs 2 + 4 launches).  The output is the packed B×(n1 + n2) [μ | logσ²]
    that bottleneck_packed reads in place."""

    @staticmethod
    def forward(ctx, x, W1, b1, W2, b2):
        Wc, bc = _adjacent(W1, W2), _adjacent(b1, b2)
        ctx.save_for_backward(x, Wc)
        ctx.n1 = W1.shape[0]
        return torch.addmm(bc, x, Wc.t())

    @staticmethod
    def backward(ctx, G):
        x, Wc = ctx.saved_tensors
        n1 = ctx.n1
        G = G.contiguous()
        gx = G.mm(Wc) if ctx.needs_input_grad[0] else None
        gW = G.t().mm(x)
        gb = _bias_grad(G)
        return gx, gW[:n1], gb[:n1], gW[n1:], gb[n1:]


def linear_cat(x: torch.Tensor, lin1: torch.nn.Linear, lin2: torch.nn.Linear) -> torch.Tensor:
    """``torch.cat([lin1(x), lin2(x)], 1)`` through _LinearCat."""
    x = x.to(lin1.weight.dtype)
    return _LinearCat.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias)


def linear_pair(x: torch.Tensor, lin1: torch.nn.Linear, lin2: torch.nn.Linear):
    """``(lin1(x), lin2(x))`` through _LinearPair."""
    x = x.to(lin1.weight.dtype)
    return _LinearPair.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias)


def linear_act(x: torch.Tensor, lin: torch.nn.Linear, act: bool) -> torch.Tensor:
    """``lin(x)`` (→ ELU) through _LinearAct, on ``lin``'s (possibly substituted,
    bf16) weight and bias."""
    return _LinearAct.apply(x.to(lin.weight.dtype), lin.weight, lin.bias, act)


def standardise(x: torch.Tensor, mean: torch.Tensor, std: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    """(x − mean) / std per column of a B×L float32 batch, in ``dtype``."""
    B, L = x.shape
    out = torch.empty((B, L), dtype=dtype, device=x.device)
    check(_lib.load().ocm_vae_standardise(_h(x.device), ptr(x), B, L, ptr(mean), ptr(std), _DT[dtype], ptr(out),
                                          stream_handle(x.device)), "ocm_vae_standardise")
    return out
