// Row-sharded fit: the one data-path exchange of a SIMCA fit
// spread over GPUs is the sum of every rank's second moments.
//
// Each rank's Gram is accumulated about its OWN shift s_r (a sample mean of
// its rows: the i8×3 digits and the f32 chunk sums need values centred to
// O(σ)), so the ranks need no collective before the Gram.  ocm_gram_pack then
// re-expresses the rank's moments about zero in fp64,
//     M_r = G_r + s_r·c_rᵀ + c_r·s_rᵀ + n_r·s_r·s_rᵀ      (Σ x xᵀ of its rows)
//     m_r = c_r + n_r·s_r                                 (Σ x)
// and writes the upper triangle of M_r, m_r and n_r into ONE flat buffer:
// p(p+1)/2 + p + 1 doubles (16.8 MB at p = 2048 instead of 33.5 MB for the
// full G plus two more collectives for Σy and n).  One all-reduce (sum) of
// that buffer gives M, m, n of all rows, and ocm_cov_from_packed forms
//     μ = m/n,  C = (M − n·μ·μᵀ)/(n − 1)
// i.e. np.cov / explained_variance_ (utils/SIMCA.py:64-66 → sklearn
// _pca.py:584) of the whole class.  The re-centring about zero costs
// |μ|²/λ_tail of relative precision in fp64 (≈ 1e-13 on the bench spectra),
// far below the float32 SVD the reference runs.
#include <cmath>

#include "ocm_internal.h"

namespace {

__host__ __device__ inline int64_t tri_off(int64_t i, int64_t p) { return i * p - i * (i - 1) / 2; }

// blockIdx.y = row i; threads cover columns j ≥ i
__global__ __launch_bounds__(256) void k_gram_pack(const double* __restrict__ G, const double* __restrict__ cs,
                                                   const float* __restrict__ shift, double n, int p,
                                                   double* __restrict__ packed) {
  const int i = blockIdx.y;
  const int j = i + blockIdx.x * 256 + threadIdx.x;
  const double si = (double)shift[i], ci = cs[i];
  if (j < p) {
    const double sj = (double)shift[j], cj = cs[j];
    packed[tri_off(i, p) + (j - i)] = G[(int64_t)i * p + j] + si * cj + ci * sj + n * si * sj;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    const int64_t tri = (int64_t)p * (p + 1) / 2;
    packed[tri + i] = ci + n * si;
    if (i == 0) packed[tri + p] = n;
  }
}

__global__ __launch_bounds__(256) void k_cov_packed_mean(const double* __restrict__ packed, int p,
                                                         double* __restrict__ mean) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  if (i < p) mean[i] = packed[tri + i] / packed[tri + p];
}

__global__ __launch_bounds__(256) void k_cov_packed(const double* __restrict__ packed, const double* __restrict__ mean,
                                                    int p, double* __restrict__ C) {
  const int i = blockIdx.y;
  const int j = blockIdx.x * 256 + threadIdx.x;
  if (j >= p) return;
  const int64_t tri = (int64_t)p * (p + 1) / 2;
  const double n = packed[tri + p];
  const int a = min(i, j), b = max(i, j);
  const double m = packed[tri_off(a, p) + (b - a)];
  C[(int64_t)i * p + j] = (m - n * mean[i] * mean[j]) / (n - 1.0);
}

}  // namespace

extern "C" {

int ocm_gram_pack(ocm_ctx* ctx, const double* G, const double* colsum, const float* shift, int64_t n, int32_t p,
                  double* packed_out, void* stream) {
  OCM_REQUIRE(ctx && G && colsum && shift && packed_out, "ocm_gram_pack: NULL argument");
  OCM_REQUIRE(p > 0 && p <= 65535 && n >= 0, "ocm_gram_pack: bad shape");
  hipStream_t st = (hipStream_t)stream;
  dim3 g((unsigned)((p + 255) / 256), (unsigned)p);
  hipLaunchKernelGGL(k_gram_pack, g, dim3(256), 0, st, G, colsum, shift, (double)n, p, packed_out);
  OCM_CHECK_LAUNCH("k_gram_pack");
  return OCM_OK;
}

int ocm_cov_from_packed(ocm_ctx* ctx, const double* packed, int32_t p, double* C_out, double* mean_out,
                        void* stream) {
  OCM_REQUIRE(ctx && packed && C_out && mean_out, "ocm_cov_from_packed: NULL argument");
  OCM_REQUIRE(p > 0 && p <= 65535, "ocm_cov_from_packed: bad shape");
  hipStream_t st = (hipStream_t)stream;
  hipLaunchKernelGGL(k_cov_packed_mean, dim3((unsigned)((p + 255) / 256)), dim3(256), 0, st, packed, p, mean_out);
  OCM_CHECK_LAUNCH("k_cov_packed_mean");
  dim3 g((unsigned)((p + 255) / 256), (unsigned)p);
  hipLaunchKernelGGL(k_cov_packed, g, dim3(256), 0, st, packed, mean_out, p, C_out);
  OCM_CHECK_LAUNCH("k_cov_packed");
  return OCM_OK;
}

}  // extern "C"
