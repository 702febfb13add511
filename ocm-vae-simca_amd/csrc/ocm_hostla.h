// Host-side fp64 linear algebra for the small b×b steps of the eigensolver
// when the subspace block is wider than one 64-column device block
// (ocm_linalg.hip, n_components > ~42).  Plain C++ (no HIP): also compiled
// alone by tests/test_hostla.py under the host sanitizers.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <cstdint>
#include <limits>
#include <vector>

namespace ocm {

// implicit QL sweeps per eigenvalue before it counts as not converged (LAPACK
// dsteqr allows 30·n in total; one eigenvalue takes 2-3 on average)
constexpr int QL_MAX_ITER = 90;

// S = L Lᵀ with the device kernels' pivot clamp (1e-14·max diag); M = L⁻ᵀ.
inline void host_chol_inv_t(const double* S, int b, double* M) {
  std::vector<double> L((size_t)b * b, 0.0), Li((size_t)b * b, 0.0);
  double dmax = 0.0;
  for (int i = 0; i < b; ++i) dmax = std::max(dmax, S[(size_t)i * b + i]);
  if (!(dmax > 0.0)) dmax = 1.0;
  for (int j = 0; j < b; ++j) {
    double d = S[(size_t)j * b + j];
    for (int l = 0; l < j; ++l) d -= L[(size_t)j * b + l] * L[(size_t)j * b + l];
    const double djj = std::sqrt(std::max(d, 1e-14 * dmax));
    L[(size_t)j * b + j] = djj;
    for (int i = j + 1; i < b; ++i) {
      double v = S[(size_t)i * b + j];
      for (int l = 0; l < j; ++l) v -= L[(size_t)i * b + l] * L[(size_t)j * b + l];
      L[(size_t)i * b + j] = v / djj;
    }
  }
  // Li = L⁻¹ (lower), column by column
  for (int c = 0; c < b; ++c) {
    for (int i = c; i < b; ++i) {
      double v = i == c ? 1.0 : 0.0;
      for (int l = c; l < i; ++l) v -= L[(size_t)i * b + l] * Li[(size_t)l * b + c];
      Li[(size_t)i * b + c] = v / L[(size_t)i * b + i];
    }
  }
  for (int i = 0; i < b; ++i)
    for (int j = 0; j < b; ++j) M[(size_t)i * b + j] = Li[(size_t)j * b + i];
}

// Symmetric eigen-decomposition of n×n A (row-major; the symmetric part is
// used): eigenvalues descending into ev, Z[i·n + j] = component i of
// eigenvector j.
// Returns false if some eigenvalue did not converge within QL_MAX_ITER implicit
// QL sweeps (its value and vectors are then unreliable).
// √(a² + b²) without std::hypot's cost (its overflow care is needed only far
// from the magnitudes of a covariance's projections; those take the slow path)
inline double fast_hypot(double a, double b) {
  const double m = std::fmax(std::fabs(a), std::fabs(b));
  if (m > 1e150 || (m < 1e-150 && m > 0.0)) return std::hypot(a, b);
  return std::sqrt(a * a + b * b);
}

inline bool host_sym_eig(const double* A, int n, double* ev, double* Z) {
  // flat work arrays; zt[j·n + i] = component i of (eventually) eigenvector j,
  // so reflectors and QL rotations update contiguous rows
  std::vector<double> a((size_t)n * n), d(n), e(n, 0.0), v(n), pv(n), zt((size_t)n * n, 0.0), hw((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) a[(size_t)i * n + j] = 0.5 * (A[(size_t)i * n + j] + A[(size_t)j * n + i]);
  // A ← H A H, H = I − 2 w wᵀ, zeroing column k below the subdiagonal;
  // w_k (entries k+1..n-1) kept in row k of hw (zero row: no reflection)
  const int nref = std::max(0, n - 2);
  for (int k = 0; k < nref; ++k) {
    double* w = &hw[(size_t)k * n];
    double nrm = 0.0;
    for (int i = k + 1; i < n; ++i) nrm += a[(size_t)i * n + k] * a[(size_t)i * n + k];
    nrm = std::sqrt(nrm);
    if (nrm == 0.0) continue;
    const double x0 = a[(size_t)(k + 1) * n + k];
    const double alpha = x0 > 0 ? -nrm : nrm;
    for (int i = k + 1; i < n; ++i) w[i] = a[(size_t)i * n + k];
    w[k + 1] -= alpha;
    double wn = 0.0;
    for (int i = k + 1; i < n; ++i) wn += w[i] * w[i];
    wn = std::sqrt(wn);
    if (wn == 0.0) {
      for (int i = k + 1; i < n; ++i) w[i] = 0.0;
      continue;
    }
    for (int i = k + 1; i < n; ++i) w[i] /= wn;
    // p = A w (trailing block), K = wᵀp, q = p − K w, A −= 2(w qᵀ + q wᵀ)
    double K = 0.0;
    for (int i = k + 1; i < n; ++i) {
      double s = 0.0;
      const double* ar = &a[(size_t)i * n];
      for (int j = k + 1; j < n; ++j) s += ar[j] * w[j];
      pv[i] = s;
      K += w[i] * s;
    }
    for (int i = k + 1; i < n; ++i) v[i] = pv[i] - K * w[i];
    for (int i = k + 1; i < n; ++i) {
      double* ar = &a[(size_t)i * n];
      const double wi = w[i], vi = v[i];
      for (int j = k + 1; j < n; ++j) ar[j] -= 2.0 * (wi * v[j] + vi * w[j]);
    }
    a[(size_t)(k + 1) * n + k] = a[(size_t)k * n + k + 1] = alpha;
    for (int i = k + 2; i < n; ++i) a[(size_t)i * n + k] = a[(size_t)k * n + i] = 0.0;
  }
  for (int i = 0; i < n; ++i) d[i] = a[(size_t)i * n + i];
  for (int i = 0; i + 1 < n; ++i) e[i] = a[(size_t)(i + 1) * n + i];
  // Q = H_0 H_1 … H_{n-3}: applied to the identity from the last reflector back
  for (int i = 0; i < n; ++i) zt[(size_t)i * n + i] = 1.0;
  for (int k = nref - 1; k >= 0; --k) {
    const double* w = &hw[(size_t)k * n];
    for (int j = 0; j < n; ++j) {  // column j of Q (row j of zt): z_j −= 2 w (wᵀ z_j)
      double* zr = &zt[(size_t)j * n];
      double s = 0.0;
      for (int i = k + 1; i < n; ++i) s += w[i] * zr[i];
      if (s == 0.0) continue;
      for (int i = k + 1; i < n; ++i) zr[i] -= 2.0 * s * w[i];
    }
  }
  // implicit QL on (d, e), rotations accumulated into the rows of zt
  const double eps = std::numeric_limits<double>::epsilon();
  bool converged = true;
  for (int l = 0; l < n; ++l) {
    for (int iter = 0;; ++iter) {
      if (iter == QL_MAX_ITER) {
        converged = false;
        break;
      }
      int m = l;
      for (; m + 1 < n; ++m) {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= eps * dd) break;
      }
      if (m == l) break;
      double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
      double r = fast_hypot(g, 1.0);
      g = d[m] - d[l] + e[l] / (g + (g >= 0 ? r : -r));
      double s = 1.0, c = 1.0, p = 0.0;
      int i = m - 1;
      bool underflow = false;
      for (; i >= l; --i) {
        double f = s * e[i], bb = c * e[i];
        r = fast_hypot(f, g);
        e[i + 1] = r;
        if (r == 0.0) {
          d[i + 1] -= p;
          e[m] = 0.0;
          underflow = true;
          break;
        }
        s = f / r;
        c = g / r;
        g = d[i + 1] - p;
        r = (d[i] - g) * s + 2.0 * c * bb;
        p = s * r;
        d[i + 1] = g + p;
        g = c * r - bb;
        double* z0 = &zt[(size_t)i * n];
        double* z1 = &zt[(size_t)(i + 1) * n];
        for (int q = 0; q < n; ++q) {
          const double zf = z1[q];
          z1[q] = s * z0[q] + c * zf;
          z0[q] = c * z0[q] - s * zf;
        }
      }
      if (underflow) continue;
      d[l] -= p;
      e[l] = g;
      e[m] = 0.0;
    }
  }
  std::vector<int> ord(n);
  for (int i = 0; i < n; ++i) ord[i] = i;
  std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return d[x] > d[y]; });
  for (int j = 0; j < n; ++j) {
    ev[j] = d[ord[j]];
    const double* zr = &zt[(size_t)ord[j] * n];
    for (int i = 0; i < n; ++i) Z[(size_t)i * n + j] = zr[i];
  }
  return converged;
}

// Eigenvalues of the symmetric tridiagonal matrix (d[0..n-1] diagonal,
// e[0..n-2] off-diagonal) by implicit QL without vectors; descending into ev.
// Returns false if some eigenvalue did not converge within QL_MAX_ITER sweeps.
inline bool host_tridiag_eigvals(const double* d_in, const double* e_in, int n, double* ev) {
  std::vector<double> d(d_in, d_in + n), e(n, 0.0);
  for (int i = 0; i + 1 < n; ++i) e[i] = e_in[i];
  const double eps = std::numeric_limits<double>::epsilon();
  bool converged = true;
  for (int l = 0; l < n; ++l) {
    for (int iter = 0;; ++iter) {
      if (iter == QL_MAX_ITER) {
        converged = false;
        break;
      }
      int m = l;
      for (; m + 1 < n; ++m) {
        const double dd = std::fabs(d[m]) + std::fabs(d[m + 1]);
        if (std::fabs(e[m]) <= eps * dd) break;
      }
      if (m == l) break;
      double g = (d[l + 1] - d[l]) / (2.0 * e[l]);
      double r = std::hypot(g, 1.0);
      g = d[m] - d[l] + e[l] / (g + (g >= 0 ? r : -r));
      double s = 1.0, c = 1.0, p = 0.0;
      int i = m - 1;
      bool underflow = false;
      for (; i >= l; --i) {
        double f = s * e[i], bb = c * e[i];
        r = std::hypot(f, g);
        e[i + 1] = r;
        if (r == 0.0) {
          d[i + 1] -= p;
          e[m] = 0.0;
          underflow = true;
          break;
        }
        s = f / r;
        c = g / r;
        g = d[i + 1] - p;
        r = (d[i] - g) * s + 2.0 * c * bb;
        p = s * r;
        d[i + 1] = g + p;
        g = c * r - bb;
      }
      if (underflow) continue;
      d[l] -= p;
      e[l] = g;
      e[m] = 0.0;
    }
  }
  std::sort(d.begin(), d.end(), [](double a, double b) { return a > b; });
  for (int i = 0; i < n; ++i) ev[i] = d[i];
  return converged;
}

// Eigenvectors of the tridiagonal matrix for the k eigenvalues lam[0..k-1]
// (descending) by inverse iteration (LAPACK dstein's scheme: LU with partial
// pivoting of T − λI, perturbed when λ repeats, and modified Gram–Schmidt
// against the vectors of the same cluster, |λ_i − λ_j| ≤ 1e-3·‖T‖₁).
// X[i·k + j] = component i of vector j (unit norm).
inline void host_tridiag_invit(const double* d, const double* e, int n, const double* lam, int k, double* X) {
  const double eps = std::numeric_limits<double>::epsilon();
  double tnorm = 0.0;
  for (int i = 0; i < n; ++i)
    tnorm = std::max(tnorm, std::fabs(d[i]) + (i > 0 ? std::fabs(e[i - 1]) : 0.0) + (i + 1 < n ? std::fabs(e[i]) : 0.0));
  if (!(tnorm > 0.0)) tnorm = 1.0;
  const double ortol = 1e-3 * tnorm, pert = 10.0 * eps * tnorm;
  std::vector<double> dl(n), dd(n), du(n), du2(n), b(n), x(n);
  std::vector<int> piv(n);
  double xprev = 0.0;
  int cluster0 = 0;
  uint64_t seed = 0x9E3779B97F4A7C15ull;
  for (int j = 0; j < k; ++j) {
    double xj = lam[j];
    if (j > 0 && lam[j - 1] - lam[j] > ortol) cluster0 = j;
    if (j > 0 && xj >= xprev - pert) xj = xprev - pert;  // separate repeated eigenvalues
    xprev = xj;
    // T − xj·I = L·U (partial pivoting)
    for (int i = 0; i < n; ++i) {
      dd[i] = d[i] - xj;
      dl[i] = i + 1 < n ? e[i] : 0.0;
      du[i] = i + 1 < n ? e[i] : 0.0;
      du2[i] = 0.0;
      piv[i] = i;
    }
    for (int i = 0; i + 1 < n; ++i) {
      if (std::fabs(dd[i]) >= std::fabs(dl[i])) {
        if (dd[i] == 0.0) dd[i] = pert;
        const double f = dl[i] / dd[i];
        dl[i] = f;
        dd[i + 1] -= f * du[i];
      } else {
        const double f = dd[i] / dl[i];
        dd[i] = dl[i];
        dl[i] = f;
        const double t = du[i];
        du[i] = dd[i + 1];
        dd[i + 1] = t - f * dd[i + 1];
        if (i + 2 < n) {
          du2[i] = du[i + 1];
          du[i + 1] = -f * du[i + 1];
        }
        piv[i] = i + 1;
      }
    }
    for (int i = 0; i < n; ++i)
      if (dd[i] == 0.0) dd[i] = pert;
    for (int i = 0; i < n; ++i) {  // a deterministic pseudo-random start
      seed = seed * 6364136223846793005ull + 1442695040888963407ull;
      b[i] = (double)((seed >> 11) & ((1ull << 52) - 1)) / (double)(1ull << 52) - 0.5;
    }
    for (int it = 0; it < 5; ++it) {
      // solve L U x = b
      for (int i = 0; i + 1 < n; ++i) {
        if (piv[i] != i) std::swap(b[i], b[i + 1]);
        b[i + 1] -= dl[i] * b[i];
      }
      x[n - 1] = b[n - 1] / dd[n - 1];
      if (n > 1) x[n - 2] = (b[n - 2] - du[n - 2] * x[n - 1]) / dd[n - 2];
      for (int i = n - 3; i >= 0; --i) x[i] = (b[i] - du[i] * x[i + 1] - du2[i] * x[i + 2]) / dd[i];
      // against the earlier vectors of this cluster
      for (int q = cluster0; q < j; ++q) {
        double s = 0.0;
        for (int i = 0; i < n; ++i) s += X[(size_t)i * k + q] * x[i];
        for (int i = 0; i < n; ++i) x[i] -= s * X[(size_t)i * k + q];
      }
      double nrm = 0.0;
      for (int i = 0; i < n; ++i) nrm += x[i] * x[i];
      nrm = std::sqrt(nrm);
      if (!(nrm > 0.0)) nrm = 1.0;
      for (int i = 0; i < n; ++i) b[i] = x[i] / nrm;
    }
    for (int i = 0; i < n; ++i) X[(size_t)i * k + j] = b[i];
  }
}

}  // namespace ocm
