// Host-side fp64 linear algebra for the small b×b steps of the eigensolver
// when the subspace block is wider than one 64-column device block
// (ocm_linalg.hip, n_components > ~42).  Plain C++ (no HIP): also compiled
// alone by tests/test_hostla.py under the host sanitizers.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <limits>
#include <vector>

namespace ocm {

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
inline void host_sym_eig(const double* A, int n, double* ev, double* Z) {
  std::vector<double> a((size_t)n * n), d(n), e(n, 0.0), v(n), pv(n), z((size_t)n * n, 0.0);
  for (int i = 0; i < n; ++i)
    for (int j = 0; j < n; ++j) a[(size_t)i * n + j] = 0.5 * (A[(size_t)i * n + j] + A[(size_t)j * n + i]);
  std::vector<std::vector<double>> hv;  // Householder vectors (index k: entries k+1..n-1)
  // A ← H A H, H = I − 2 w wᵀ, zeroing column k below the subdiagonal
  for (int k = 0; k + 2 < n; ++k) {
    double nrm = 0.0;
    for (int i = k + 1; i < n; ++i) nrm += a[(size_t)i * n + k] * a[(size_t)i * n + k];
    nrm = std::sqrt(nrm);
    std::vector<double> w(n, 0.0);
    if (nrm == 0.0) {
      hv.push_back(w);
      continue;
    }
    const double x0 = a[(size_t)(k + 1) * n + k];
    const double alpha = x0 > 0 ? -nrm : nrm;
    for (int i = k + 1; i < n; ++i) w[i] = a[(size_t)i * n + k];
    w[k + 1] -= alpha;
    double wn = 0.0;
    for (int i = k + 1; i < n; ++i) wn += w[i] * w[i];
    wn = std::sqrt(wn);
    if (wn == 0.0) {
      hv.push_back(std::vector<double>(n, 0.0));
      continue;
    }
    for (int i = k + 1; i < n; ++i) w[i] /= wn;
    // p = A w (trailing block), K = wᵀp, q = p − K w, A −= 2(w qᵀ + q wᵀ)
    double K = 0.0;
    for (int i = k + 1; i < n; ++i) {
      double s = 0.0;
      for (int j = k + 1; j < n; ++j) s += a[(size_t)i * n + j] * w[j];
      pv[i] = s;
      K += w[i] * s;
    }
    for (int i = k + 1; i < n; ++i) v[i] = pv[i] - K * w[i];
    for (int i = k + 1; i < n; ++i)
      for (int j = k + 1; j < n; ++j) a[(size_t)i * n + j] -= 2.0 * (w[i] * v[j] + v[i] * w[j]);
    a[(size_t)(k + 1) * n + k] = a[(size_t)k * n + k + 1] = alpha;
    for (int i = k + 2; i < n; ++i) a[(size_t)i * n + k] = a[(size_t)k * n + i] = 0.0;
    hv.push_back(w);
  }
  for (int i = 0; i < n; ++i) d[i] = a[(size_t)i * n + i];
  for (int i = 0; i + 1 < n; ++i) e[i] = a[(size_t)(i + 1) * n + i];
  // Q = H_0 H_1 … H_{n-3}: apply to the identity from the last reflector back
  for (int i = 0; i < n; ++i) z[(size_t)i * n + i] = 1.0;
  for (int k = (int)hv.size() - 1; k >= 0; --k) {
    const std::vector<double>& w = hv[k];
    for (int j = 0; j < n; ++j) {  // column j: z_j −= 2 w (wᵀ z_j)
      double s = 0.0;
      for (int i = k + 1; i < n; ++i) s += w[i] * z[(size_t)i * n + j];
      if (s == 0.0) continue;
      for (int i = k + 1; i < n; ++i) z[(size_t)i * n + j] -= 2.0 * s * w[i];
    }
  }
  // implicit QL on (d, e), rotations accumulated into the columns of z
  const double eps = std::numeric_limits<double>::epsilon();
  for (int l = 0; l < n; ++l) {
    for (int iter = 0; iter < 60; ++iter) {
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
        for (int q = 0; q < n; ++q) {
          const double zf = z[(size_t)q * n + i + 1];
          z[(size_t)q * n + i + 1] = s * z[(size_t)q * n + i] + c * zf;
          z[(size_t)q * n + i] = c * z[(size_t)q * n + i] - s * zf;
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
    for (int i = 0; i < n; ++i) Z[(size_t)i * n + j] = z[(size_t)i * n + ord[j]];
  }
}

}  // namespace ocm
