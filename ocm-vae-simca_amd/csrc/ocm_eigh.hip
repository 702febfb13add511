// Dense symmetric eigensolver (fp64): every eigenvalue of C and, optionally,
// the leading k eigenvectors.
//
// Two callers, both off the timed path:
//   * `_model[cls]['eigs_all']` (utils/SIMCA.py:88 keeps all min(n, p)
//     explained variances of the full SVD, sklearn _pca.py:584-598);
//   * the fallback of ocm_eig_topk when the subspace iteration does not
//     converge (no spectral gap after component k): the reference's full SVD
//     always returns, so the drop-in takes the dense route instead of failing.
//
// Householder tridiagonalisation Q ᵀ C Q = T on the GPU (LAPACK dsytd2's
// reflectors, one per column, on the HBM-resident full symmetric matrix: a
// symv launch and a rank-2 update launch per column, the next reflector formed
// by the rank-2 update's last workgroup), the eigenvalues of T by implicit QL
// on the host (O(p²) on two p-vectors), the top k eigenvectors of T by inverse
// iteration on the host (dstein's scheme), and their back-transformation by
// the stored reflectors on the GPU.  Sign convention of sklearn svd_flip
// (u_based_decision=False): each vector's largest |entry| positive.
#include <algorithm>
#include <cmath>
#include <vector>

#include "ocm_hostla.h"
#include "ocm_internal.h"

namespace {

constexpr int TR_T = 256;

__device__ __forceinline__ double block_sum(double v, double* red) {
  v = wave_sum_f64(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];  // fixed order
  return s;
}

// Reflector of row j (dlarfg): x = A[j][j+1 ..]; v (v₀ = 1) replaces x in
// row j, d[j] = A[j][j], e[j] = β, tau[j] = τ.  One workgroup.
__device__ void house_row(double* __restrict__ A, int p, int j, double* __restrict__ d, double* __restrict__ e,
                          double* __restrict__ tau) {
  __shared__ double red[TR_T / 64];
  __shared__ double sc[2];
  double* x = A + (int64_t)j * p + j + 1;
  const int n = p - j - 1;
  double s = 0.0;
  for (int i = 1 + (int)threadIdx.x; i < n; i += blockDim.x) s += x[i] * x[i];
  const double xn2 = block_sum(s, red);
  if (threadIdx.x == 0) {
    const double alpha = x[0];
    if (xn2 == 0.0) {
      sc[0] = 0.0;  // τ = 0: H = I
      sc[1] = 0.0;
      tau[j] = 0.0;
      e[j] = alpha;
    } else {
      const double beta = -copysign(sqrt(alpha * alpha + xn2), alpha);
      tau[j] = (beta - alpha) / beta;
      e[j] = beta;
      sc[0] = 1.0 / (alpha - beta);
      sc[1] = 1.0;
    }
    d[j] = A[(int64_t)j * p + j];
  }
  __syncthreads();
  const double scale = sc[0];
  const bool nz = sc[1] != 0.0;
  for (int i = 1 + (int)threadIdx.x; i < n; i += blockDim.x) x[i] = nz ? x[i] * scale : 0.0;
  if (threadIdx.x == 0) x[0] = 1.0;
}

__global__ __launch_bounds__(TR_T) void k_tri_house0(double* A, int p, double* d, double* e, double* tau) {
  house_row(A, p, 0, d, e, tau);
}

// w_i = τ Σ_l A[i][l] v_l over the trailing block (one wave per row), and
// α = −½ τ wᵀv by the last workgroup (partials summed in order).
__global__ __launch_bounds__(TR_T) void k_tri_symv(const double* __restrict__ A, int p, int j,
                                                    const double* __restrict__ tau, double* __restrict__ w,
                                                    double* __restrict__ part, unsigned* __restrict__ ticket,
                                                    double* __restrict__ alpha) {
  __shared__ double red[TR_T / 64];
  __shared__ bool last;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i0 = j + 1, n = p - i0;
  const double* v = A + (int64_t)j * p + i0;
  const double t = tau[j];
  const int i = i0 + blockIdx.x * (TR_T / 64) + wv;
  double wi = 0.0, pv = 0.0;
  if (i < p) {
    const double* row = A + (int64_t)i * p + i0;
    double s = 0.0;
    for (int l = lane; l < n; l += 64) s += row[l] * v[l];
    wi = t * wave_sum_f64(s);
    if (lane == 0) w[i - i0] = wi;
    pv = wi * v[i - i0];
  }
  if (lane != 0) pv = 0.0;
  const double ps = block_sum(pv, red);
  if (threadIdx.x == 0) {
    part[blockIdx.x] = ps;
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  double s = 0.0;
  for (int b = threadIdx.x; b < (int)gridDim.x; b += TR_T) s += part[b];
  // in order: each thread's strided partials, then the block sum in wave order
  const double tot = block_sum(s, red);
  if (threadIdx.x == 0) {
    *alpha = -0.5 * t * tot;
    *ticket = 0u;
  }
}

// A₂₂ −= v w'ᵀ + w' vᵀ, w' = w + α v; the last workgroup then forms the
// reflector of row j + 1.
__global__ __launch_bounds__(TR_T) void k_tri_rank2(double* __restrict__ A, int p, int j,
                                                     const double* __restrict__ w, const double* __restrict__ alpha,
                                                     double* __restrict__ d, double* __restrict__ e,
                                                     double* __restrict__ tau, unsigned* __restrict__ ticket) {
  __shared__ bool last;
  const int i0 = j + 1, n = p - i0;
  const double* v = A + (int64_t)j * p + i0;
  const double al = *alpha;
  const int r = blockIdx.y;  // row of the trailing block
  const int c = blockIdx.x * TR_T + threadIdx.x;
  if (c < n) {
    const double vr = v[r], vc = v[c];
    const double wr = w[r] + al * vr, wc = w[c] + al * vc;
    double* a = A + (int64_t)(i0 + r) * p + i0 + c;
    *a -= vr * wc + wr * vc;
  }
  if (j + 4 > p) return;  // row j + 1 starts the last 2×2 block: no reflector (k_tri_tail reads it)
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    last = atomicAdd(ticket, 1u) == gridDim.x * gridDim.y - 1;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  house_row(A, p, j + 1, d, e, tau);
  if (threadIdx.x == 0) *ticket = 0u;
}

// the trailing 2×2 (or 1×1) block of T
__global__ void k_tri_tail(const double* __restrict__ A, int p, double* __restrict__ d, double* __restrict__ e) {
  if (threadIdx.x != 0) return;
  if (p >= 2) {
    d[p - 2] = A[(int64_t)(p - 2) * p + p - 2];
    e[p - 2] = A[(int64_t)(p - 2) * p + p - 1];
  }
  d[p - 1] = A[(int64_t)(p - 1) * p + p - 1];
}

// Eigenvector c of C = Q x_c, Q = H₀ H₁ … H_{p−3} (reflector j in row j of A
// from column j + 1); one workgroup per vector, x in LDS.  X: p×k (row i,
// column c); out: k×p rows.
__global__ __launch_bounds__(TR_T) void k_tri_backtransform(const double* __restrict__ A, int p,
                                                             const double* __restrict__ tau,
                                                             const double* __restrict__ X, int k,
                                                             double* __restrict__ out) {
  extern __shared__ double xs[];
  __shared__ double red[TR_T / 64];
  const int c = blockIdx.x;
  for (int i = threadIdx.x; i < p; i += TR_T) xs[i] = X[(int64_t)i * k + c];
  __syncthreads();
  for (int j = p - 3; j >= 0; --j) {
    const double t = tau[j];
    if (t == 0.0) continue;  // uniform
    const double* v = A + (int64_t)j * p + j + 1;
    const int n = p - j - 1;
    double s = 0.0;
    for (int i = threadIdx.x; i < n; i += TR_T) s += v[i] * xs[j + 1 + i];
    const double f = t * block_sum(s, red);
    for (int i = threadIdx.x; i < n; i += TR_T) xs[j + 1 + i] -= f * v[i];
    __syncthreads();
  }
  for (int i = threadIdx.x; i < p; i += TR_T) out[(int64_t)c * p + i] = xs[i];
}

// rows of `ev` (k×p): max-|entry| positive (sklearn svd_flip, first index on ties)
__global__ __launch_bounds__(TR_T) void k_rows_signfix(double* __restrict__ ev, int p) {
  __shared__ double bv[TR_T];
  __shared__ int bi[TR_T];
  double* row = ev + (int64_t)blockIdx.x * p;
  double best = -1.0;
  int bidx = 0x7fffffff;
  for (int j = threadIdx.x; j < p; j += TR_T) {
    const double a = fabs(row[j]);
    if (a > best || (a == best && j < bidx)) {
      best = a;
      bidx = j;
    }
  }
  bv[threadIdx.x] = best;
  bi[threadIdx.x] = bidx;
  __syncthreads();
  for (int o = TR_T / 2; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) {
      const double a = bv[threadIdx.x + o];
      const int ai = bi[threadIdx.x + o];
      if (a > bv[threadIdx.x] || (a == bv[threadIdx.x] && ai < bi[threadIdx.x])) {
        bv[threadIdx.x] = a;
        bi[threadIdx.x] = ai;
      }
    }
    __syncthreads();
  }
  const double sg = row[bi[0]] < 0.0 ? -1.0 : 1.0;
  __syncthreads();
  for (int j = threadIdx.x; j < p; j += TR_T) row[j] *= sg;
}

}  // namespace

namespace ocm {

constexpr int EIGH_VEC_MAXP = 96 * 1024 / (int)sizeof(double);  // 12288

int eigh_dense(ocm_ctx* ctx, const double* C, int p, double* evals_out, int k, double* evecs_out, hipStream_t st) {
  const size_t pp = (size_t)p * p;
  const int nblk_max = (p + TR_T / 64 - 1) / (TR_T / 64);
  const size_t need = (pp + 4 * (size_t)p + (size_t)nblk_max + (size_t)p * std::max(k, 1) + 64) * sizeof(double) +
                      8 * 256;
  void* wsp = workspace(ctx, need, st);
  if (!wsp) return OCM_ERR_NOMEM;
  Carve cv{static_cast<char*>(wsp)};
  double* A = cv.take<double>(pp);
  double* d = cv.take<double>(p);
  double* e = cv.take<double>(p);
  double* tau = cv.take<double>(p);
  double* w = cv.take<double>(p);
  double* part = cv.take<double>(nblk_max);
  double* X = cv.take<double>((size_t)p * std::max(k, 1));
  double* alpha = cv.take<double>(8);
  unsigned* ticket = cv.take<unsigned>(4);
  OCM_HIP(hipMemcpyAsync(A, C, pp * sizeof(double), hipMemcpyDeviceToDevice, st));
  OCM_HIP(hipMemsetAsync(ticket, 0, 16, st));
  OCM_HIP(hipMemsetAsync(e, 0, (size_t)p * sizeof(double), st));
  OCM_HIP(hipMemsetAsync(tau, 0, (size_t)p * sizeof(double), st));
  if (p >= 3) {
    hipLaunchKernelGGL(k_tri_house0, dim3(1), dim3(TR_T), 0, st, A, p, d, e, tau);
    for (int j = 0; j + 2 < p; ++j) {
      const int n = p - j - 1;
      const int nb = (n + TR_T / 64 - 1) / (TR_T / 64);
      hipLaunchKernelGGL(k_tri_symv, dim3(nb), dim3(TR_T), 0, st, A, p, j, tau, w, part, ticket, alpha);
      hipLaunchKernelGGL(k_tri_rank2, dim3((n + TR_T - 1) / TR_T, n), dim3(TR_T), 0, st, A, p, j, w, alpha, d, e,
                         tau, ticket + 1);
    }
    OCM_CHECK_LAUNCH("k_tri_rank2");
  }
  hipLaunchKernelGGL(k_tri_tail, dim3(1), dim3(64), 0, st, A, p, d, e);
  OCM_CHECK_LAUNCH("k_tri_tail");
  std::vector<double> hd(p), he(std::max(p, 1)), hev(p);
  OCM_HIP(hipMemcpyAsync(hd.data(), d, (size_t)p * sizeof(double), hipMemcpyDeviceToHost, st));
  OCM_HIP(hipMemcpyAsync(he.data(), e, (size_t)p * sizeof(double), hipMemcpyDeviceToHost, st));
  OCM_HIP(hipStreamSynchronize(st));
  if (!host_tridiag_eigvals(hd.data(), he.data(), p, hev.data())) {
    ocm::set_error("ocm_eigh_f64: implicit QL did not converge");
    return OCM_ERR_NOCONV;
  }
  OCM_HIP(hipMemcpyAsync(evals_out, hev.data(), (size_t)p * sizeof(double), hipMemcpyHostToDevice, st));
  if (k > 0 && evecs_out) {
    std::vector<double> hx((size_t)p * k);
    host_tridiag_invit(hd.data(), he.data(), p, hev.data(), k, hx.data());
    OCM_HIP(hipMemcpyAsync(X, hx.data(), hx.size() * sizeof(double), hipMemcpyHostToDevice, st));
    const size_t lds = (size_t)p * sizeof(double);
    hipLaunchKernelGGL(k_tri_backtransform, dim3(k), dim3(TR_T), lds, st, A, p, tau, X, k, evecs_out);
    hipLaunchKernelGGL(k_rows_signfix, dim3(k), dim3(TR_T), 0, st, evecs_out, p);
    OCM_CHECK_LAUNCH("k_tri_backtransform");
  }
  // the host vectors must outlive the copies
  OCM_HIP(hipStreamSynchronize(st));
  return OCM_OK;
}

}  // namespace ocm

extern "C" {

int ocm_eigh_f64(ocm_ctx* ctx, const double* C, int32_t p, double* evals_out, int32_t k, double* evecs_out,
                 void* stream) {
  OCM_REQUIRE(ctx && C && evals_out, "ocm_eigh_f64: NULL argument");
  OCM_REQUIRE(p >= 1 && p <= 16384, "ocm_eigh_f64: 1 <= p <= 16384");
  OCM_REQUIRE(k >= 0 && k <= p && (k == 0 || evecs_out), "ocm_eigh_f64: 0 <= k <= p (evecs_out for k > 0)");
  // the back-transformation stages one p-vector in LDS (96 KiB): checked
  // before any work starts
  OCM_REQUIRE(k == 0 || p <= ocm::EIGH_VEC_MAXP, "ocm_eigh_f64: eigenvectors (k > 0) need p <= 12288");
  return ocm::eigh_dense(ctx, C, p, evals_out, k, evecs_out, (hipStream_t)stream);
}

}  // extern "C"
