"""libocm's narrow convolutions (ocm/conv.py, csrc/ocm_conv.hip) against an
fp64 host reference of torch.nn.functional.conv1d / conv_transpose1d:
forward, input gradient, weight and bias gradients, for the C4 network's layers
(vae_model.py:37-81: 1→3 s1, 3→6 s2, 6→12 s2, transposed 12→6 / 6→3 s2 with
output padding, 3→3 s1, the 1×1 head), the reference default kernel 9, odd
lengths, float32 and bf16 autocast."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"

# (transposed, I, O, K, stride, pad, output_padding, L)
SHAPES = [
    (False, 1, 3, 7, 1, 3, 0, 2048),
    (False, 3, 6, 7, 2, 3, 0, 2048),
    (False, 6, 12, 7, 2, 3, 0, 1024),
    (True, 12, 6, 7, 2, 3, 1, 512),
    (True, 6, 3, 7, 2, 3, 1, 1024),
    (True, 3, 3, 7, 1, 3, 0, 2048),
    (False, 3, 1, 1, 1, 0, 0, 2048),
    (False, 5, 7, 9, 2, 4, 0, 301),
    (True, 7, 5, 9, 2, 4, 1, 151),
    (False, 2, 17, 5, 3, 1, 0, 257),
]


def _mods(transposed, I, O, K, s, pad, op):
    from ocm.conv import FastConv1d, FastConvTranspose1d

    torch.manual_seed(1)
    if transposed:
        fast = FastConvTranspose1d(I, O, K, stride=s, padding=pad, output_padding=op)
        ref = torch.nn.ConvTranspose1d(I, O, K, stride=s, padding=pad, output_padding=op)
    else:
        fast = FastConv1d(I, O, K, stride=s, padding=pad)
        ref = torch.nn.Conv1d(I, O, K, stride=s, padding=pad)
    ref.load_state_dict(fast.state_dict())
    return fast.to(DEV), ref.double()


@pytest.mark.parametrize("shape", SHAPES)
def test_conv_fp32_forward_and_grads(shape):
    transposed, I, O, K, s, pad, op, L = shape
    fast, ref = _mods(transposed, I, O, K, s, pad, op)
    B = 6
    g = torch.Generator().manual_seed(2)
    x = torch.randn(B, I, L, generator=g)
    xd = x.to(DEV).requires_grad_(True)
    y = fast(xd)
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    assert y.shape == yr.shape and y.dtype == torch.float32
    np.testing.assert_allclose(y.detach().cpu().numpy(), yr.detach().numpy(), rtol=1e-5, atol=1e-5)
    gy = torch.randn(yr.shape, generator=g)
    y.backward(gy.to(DEV))
    yr.backward(gy.double())
    np.testing.assert_allclose(xd.grad.cpu().numpy(), xr.grad.numpy(), rtol=1e-5, atol=1e-5)
    scale = np.abs(ref.weight.grad.numpy()).max()
    np.testing.assert_allclose(fast.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4,
                               atol=1e-5 * scale)
    np.testing.assert_allclose(fast.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4,
                               atol=1e-5 * np.abs(ref.bias.grad.numpy()).max())


@pytest.mark.parametrize("shape", SHAPES[:7])
def test_conv_bf16_autocast(shape):
    """bf16 activations under autocast: the reference is the fp64 convolution of
    the bf16-rounded input with the float32 weights; outputs and input
    gradients carry one bf16 rounding (2⁻⁸ relative)."""
    transposed, I, O, K, s, pad, op, L = shape
    fast, ref = _mods(transposed, I, O, K, s, pad, op)
    B = 4
    g = torch.Generator().manual_seed(3)
    x = torch.randn(B, I, L, generator=g).bfloat16()
    xd = x.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = fast(xd)
    assert y.dtype == torch.bfloat16
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    tol = 2.0 ** -8 * np.abs(yr.detach().numpy()).max()
    np.testing.assert_allclose(y.float().detach().cpu().numpy(), yr.detach().numpy(), rtol=2 ** -7, atol=tol)
    gy = torch.randn(yr.shape, generator=g).bfloat16()
    y.backward(gy.to(DEV))
    yr.backward(gy.double())
    assert xd.grad.dtype == torch.bfloat16
    tol = 2.0 ** -8 * np.abs(xr.grad.numpy()).max()
    np.testing.assert_allclose(xd.grad.float().cpu().numpy(), xr.grad.numpy(), rtol=2 ** -7, atol=tol)
    scale = np.abs(ref.weight.grad.numpy()).max()
    np.testing.assert_allclose(fast.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4,
                               atol=1e-5 * scale)
    # ConvTranspose1d: the bias gradient from the wgrad launch's ones row (one
    # level of partial sums at B = 4)
    bscale = np.abs(ref.bias.grad.numpy()).max()
    np.testing.assert_allclose(fast.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4, atol=1e-5 * bscale)


@pytest.mark.parametrize("shape", [SHAPES[0], SHAPES[2], SHAPES[3], SHAPES[5]])
def test_conv_bf16_wgrad_full_batch(shape):
    """The C4 batch (B = 512): the matrix-core weight gradient at its full
    workgroup count (1024 workgroups for the 1M-position layers, three levels of
    partial sums) against the fp64 host gradient of the same bf16 operands."""
    transposed, I, O, K, s, pad, op, L = shape
    fast, ref = _mods(transposed, I, O, K, s, pad, op)
    B = 512
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, I, L, generator=g).bfloat16()
    xd = x.to(DEV).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = fast(xd)
    xr = x.double().requires_grad_(True)
    yr = ref(xr)
    gy = torch.randn(yr.shape, generator=g).bfloat16()
    y.backward(gy.to(DEV))
    yr.backward(gy.double())
    scale = np.abs(ref.weight.grad.numpy()).max()
    np.testing.assert_allclose(fast.weight.grad.cpu().numpy(), ref.weight.grad.numpy(), rtol=1e-4,
                               atol=1e-5 * scale)
    bscale = np.abs(ref.bias.grad.numpy()).max()
    np.testing.assert_allclose(fast.bias.grad.cpu().numpy(), ref.bias.grad.numpy(), rtol=1e-4, atol=1e-5 * bscale)


def test_conv_stock_fallback_for_unsupported():
    """Shapes outside the direct kernels' range take the stock module."""
    from ocm.conv import FastConv1d

    m = FastConv1d(2, 3, 3, dilation=2).to(DEV)
    x = torch.randn(2, 2, 50, device=DEV)
    ref = torch.nn.functional.conv1d(x, m.weight, m.bias, dilation=2)
    torch.testing.assert_close(m(x), ref)
