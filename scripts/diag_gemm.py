"""Diagnostic: fp32 torch GEMM accuracy on gfx950 for the VAE's Linear shapes
under the available BLAS backends / precision flags (vs fp64 on the CPU)."""
import torch

torch.manual_seed(0)
shapes = [(300, 288, 32), (300, 208, 24), (300, 32, 8), (512, 6144, 64), (512, 64, 6144), (300, 288, 33)]
print("matmul.allow_tf32", torch.backends.cuda.matmul.allow_tf32, "precision", torch.get_float32_matmul_precision())
for backend in ("default", "cublas", "cublaslt"):
    if backend != "default":
        try:
            torch.backends.cuda.preferred_blas_library(backend)
        except Exception as e:
            print(backend, "unavailable", e)
            continue
    for (m, k, n) in shapes:
        a = torch.randn(m, k)
        w = torch.randn(n, k)
        ref = (a.double() @ w.double().T)
        got = torch.nn.functional.linear(a.cuda(), w.cuda()).cpu().double()
        err = ((got - ref).abs().max() / ref.abs().max()).item()
        print(f"{backend:9s} M={m:4d} K={k:5d} N={n:5d} rel err {err:.3e}")
