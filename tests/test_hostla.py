"""Host-side fp64 linear algebra of the wide-block eigensolver (csrc/ocm_hostla.h).

When n_components needs a subspace block wider than 64 columns, ocm_eig_topk
solves the block's b×b Cholesky (CholQR) and Rayleigh–Ritz eigenproblem on the
host.  Those routines are plain C++: this test compiles them alone with g++
under AddressSanitizer + UBSan (host sanitizers only) and checks them against
NumPy on random, graded and degenerate spectra.  CPU only.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(REPO, "ocm-vae-simca_amd", "csrc")

DRIVER = r"""
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "ocm_hostla.h"
int main(int argc, char** argv) {
  const char* mode = argv[1];
  FILE* f = std::fopen(argv[2], "rb");
  int n = 0;
  if (std::fread(&n, 4, 1, f) != 1) return 2;
  std::vector<double> A((size_t)n * n), out((size_t)n * n + n);
  if (std::fread(A.data(), 8, A.size(), f) != A.size()) return 2;
  std::fclose(f);
  if (mode[0] == 'e') {
    if (!ocm::host_sym_eig(A.data(), n, out.data() + (size_t)n * n, out.data())) return 3;  // QL cap hit
  } else if (mode[0] == 't') {  // tridiagonal: eigenvalues by QL, the top k vectors by inverse iteration
    std::vector<double> d(n), e(n > 1 ? n - 1 : 1);
    for (int i = 0; i < n; ++i) d[i] = A[(size_t)i * n + i];
    for (int i = 0; i + 1 < n; ++i) e[i] = A[(size_t)(i + 1) * n + i];
    if (!ocm::host_tridiag_eigvals(d.data(), e.data(), n, out.data() + (size_t)n * n)) return 3;
    const int k = n < 12 ? n : 12;
    ocm::host_tridiag_invit(d.data(), e.data(), n, out.data() + (size_t)n * n, k, out.data());
  } else {
    ocm::host_chol_inv_t(A.data(), n, out.data());
  }
  FILE* g = std::fopen(argv[3], "wb");
  std::fwrite(out.data(), 8, out.size(), g);
  std::fclose(g);
  return 0;
}
"""


@pytest.fixture(scope="module")
def driver(tmp_path_factory):
    if shutil.which("g++") is None:
        pytest.skip("g++ not available")
    d = tmp_path_factory.mktemp("hostla")
    src = d / "drv.cpp"
    src.write_text(DRIVER)
    exe = d / "drv"
    subprocess.run(["g++", "-O1", "-g", "-std=c++17", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                    "-I", CSRC, str(src), "-o", str(exe)], check=True)
    return d, exe


def _run(driver, mode, A):
    d, exe = driver
    n = A.shape[0]
    inp, outp = d / "in.bin", d / "out.bin"
    with open(inp, "wb") as f:
        f.write(np.int32(n).tobytes())
        f.write(np.ascontiguousarray(A, dtype=np.float64).tobytes())
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1")
    subprocess.run([str(exe), mode, str(inp), str(outp)], check=True, env=env)
    out = np.fromfile(outp, dtype=np.float64)
    return out[: n * n].reshape(n, n), out[n * n:]


def _spd(n, cond, seed):
    rng = np.random.default_rng(seed)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    lam = np.logspace(0, -np.log10(cond), n)
    return (Q * lam) @ Q.T, lam


@pytest.mark.parametrize("n,cond,seed", [(72, 1e3, 0), (144, 1e8, 1), (96, 1.0, 2), (130, 1e12, 3)])
def test_sym_eig_matches_numpy(driver, n, cond, seed):
    A, lam = _spd(n, cond, seed)
    Z, ev = _run(driver, "e", A)
    ref = np.sort(np.linalg.eigvalsh(A))[::-1]
    np.testing.assert_allclose(ev, ref, rtol=0, atol=1e-13 * lam.max() * n)
    assert np.all(np.diff(ev) <= 0)
    np.testing.assert_allclose(Z.T @ Z, np.eye(n), atol=1e-12 * n)
    np.testing.assert_allclose(A @ Z, Z * ev, atol=1e-12 * n * lam.max())


def test_sym_eig_repeated_and_zero_eigenvalues(driver):
    n = 80
    rng = np.random.default_rng(7)
    Q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    lam = np.concatenate([np.full(20, 3.0), np.full(30, 1.0), np.zeros(30)])
    A = (Q * lam) @ Q.T
    Z, ev = _run(driver, "e", A)
    np.testing.assert_allclose(ev, np.sort(lam)[::-1], atol=1e-12)
    np.testing.assert_allclose(A @ Z, Z * ev, atol=1e-11)


def test_sym_eig_indefinite_and_diagonal(driver):
    rng = np.random.default_rng(8)
    A = rng.standard_normal((70, 70))
    A = A + A.T
    Z, ev = _run(driver, "e", A)
    np.testing.assert_allclose(ev, np.sort(np.linalg.eigvalsh(A))[::-1], atol=1e-11)
    D = np.diag(np.arange(66, dtype=float))
    Z, ev = _run(driver, "e", D)
    np.testing.assert_allclose(ev, np.arange(66)[::-1], atol=0)


@pytest.mark.parametrize("n,cond", [(96, 1e4), (160, 1e10)])
def test_chol_inverse_transpose(driver, n, cond):
    S, _ = _spd(n, cond, 11)
    M, _ = _run(driver, "c", S)
    L = np.linalg.cholesky(S)
    np.testing.assert_allclose(M, np.linalg.inv(L).T, rtol=1e-6 * max(1.0, np.sqrt(cond) / 100), atol=1e-9 * np.abs(np.linalg.inv(L)).max())
    assert np.allclose(np.tril(M, -1), 0.0)
    # CholQR identity: (W M)ᵀ (W M) = I for S = WᵀW
    W = np.linalg.cholesky(S).T  # any W with WᵀW = S
    np.testing.assert_allclose((W @ M).T @ (W @ M), np.eye(n), atol=1e-5 if cond > 1e8 else 1e-10)


def _tridiag(d, e):
    return np.diag(d) + np.diag(e, 1) + np.diag(e, -1)


@pytest.mark.parametrize("case", ["random", "graded", "clustered", "split"])
def test_tridiag_eigvals_and_inverse_iteration(driver, case):
    """The dense fallback / eigs_all path (ocm_eigh_f64): QL eigenvalues of the
    Householder tridiagonal and inverse-iteration vectors for the top 12,
    including exactly repeated eigenvalues (a split tridiagonal)."""
    rng = np.random.default_rng(3)
    n = 300
    if case == "random":
        d, e = rng.standard_normal(n), rng.standard_normal(n - 1)
    elif case == "graded":
        d, e = np.logspace(2, -6, n), 1e-3 * rng.standard_normal(n - 1)
    elif case == "clustered":
        d, e = 1.0 + 1e-9 * rng.standard_normal(n), 1e-10 * rng.standard_normal(n - 1)
        d[:5] += 3.0
    else:  # three equal blocks: every eigenvalue three times
        b = 100
        db, eb = rng.standard_normal(b), rng.standard_normal(b - 1)
        d = np.tile(db, 3)
        e = np.concatenate([eb, [0.0], eb, [0.0], eb])
    T = _tridiag(d, e)
    X, ev = _run(driver, "t", T)
    ref = np.sort(np.linalg.eigvalsh(T))[::-1]
    scale = np.abs(ref).max()
    np.testing.assert_allclose(ev, ref, rtol=0, atol=1e-13 * scale * n)
    k = 12
    V = X.reshape(-1)[: n * k].reshape(n, k)
    np.testing.assert_allclose(V.T @ V, np.eye(k), atol=1e-9)
    np.testing.assert_allclose(T @ V, V * ev[:k], atol=1e-10 * scale)
