// K6 — percentiles by radix select (np.percentile, method 'linear').
// Reference sites: utils/SIMCA.py:160,187 (perc limits), VAE_SIMCA.py:285,
// 305, utils/final_vaesimca.py:436-437 (latent thresholds).
//
// Values map to order-preserving unsigned keys (IEEE sign trick); each pass
// histograms one 8-bit digit of the keys that match the prefix found so far
// (LDS histogram per workgroup, one global atomic per bin per workgroup).
// The k-th smallest key is fixed after 8 passes (f64) or 4 (f32).  The pass
// kernel is exported (ocm_radix_hist) so multi-rank callers can all-reduce
// the 256-bin histogram between passes.
#include <cmath>
#include <cstring>

#include "ocm_internal.h"

namespace {

__device__ __forceinline__ uint64_t okey64(uint64_t u) {
  return (u >> 63) ? ~u : (u | 0x8000000000000000ull);
}
__device__ __forceinline__ uint64_t okey32(uint32_t u) {
  return (u >> 31) ? (uint64_t)(~u) : (uint64_t)(u | 0x80000000u);
}

__global__ __launch_bounds__(256) void k_radix_hist(const void* __restrict__ v, int dtype, int64_t n,
                                                    uint64_t prefix, uint64_t himask, int shift,
                                                    unsigned long long* __restrict__ hist) {
  __shared__ unsigned int lh[256];
  lh[threadIdx.x] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) {
    uint64_t key;
    if (dtype == 0)
      key = okey64(reinterpret_cast<const uint64_t*>(v)[i]);
    else
      key = okey32(reinterpret_cast<const uint32_t*>(v)[i]);
    if (((key ^ prefix) & himask) == 0) atomicAdd(&lh[(key >> shift) & 255u], 1u);
  }
  __syncthreads();
  const unsigned c = lh[threadIdx.x];
  if (c) atomicAdd(&hist[threadIdx.x], (unsigned long long)c);
}

double key_to_value(uint64_t key, int dtype) {
  if (dtype == 0) {
    const uint64_t u = (key >> 63) ? (key & 0x7FFFFFFFFFFFFFFFull) : ~key;
    double d;
    memcpy(&d, &u, 8);
    return d;
  }
  const uint32_t k32 = (uint32_t)key;
  const uint32_t u = (k32 >> 31) ? (k32 & 0x7FFFFFFFu) : ~k32;
  float f;
  memcpy(&f, &u, 4);
  return (double)f;
}

int hist_pass(ocm_ctx* ctx, const void* v, int dtype, int64_t n, uint64_t prefix, int shift, uint64_t* hist,
              hipStream_t st) {
  const int nbits = dtype == 0 ? 64 : 32;
  const uint64_t himask = (shift + 8 >= nbits) ? 0ull : (~0ull << (shift + 8)) & (nbits == 64 ? ~0ull : 0xFFFFFFFFull);
  OCM_HIP(hipMemsetAsync(hist, 0, 256 * sizeof(uint64_t), st));
  int nblk = (int)std::min<int64_t>((n + 255) / 256, (int64_t)ctx->num_cus * 8);
  if (nblk < 1) nblk = 1;
  hipLaunchKernelGGL(k_radix_hist, dim3(nblk), dim3(256), 0, st, v, dtype, n, prefix, himask, shift,
                     reinterpret_cast<unsigned long long*>(hist));
  OCM_CHECK_LAUNCH("k_radix_hist");
  return OCM_OK;
}

// k-th smallest (0-based) value
int select_kth(ocm_ctx* ctx, const void* v, int dtype, int64_t n, int64_t kth, double* out, hipStream_t st) {
  auto* hist = static_cast<uint64_t*>(ocm::workspace(ctx, 256 * sizeof(uint64_t), st));
  auto* hh = static_cast<uint64_t*>(ocm::host_staging(ctx, 256 * sizeof(uint64_t)));
  if (!hist || !hh) return OCM_ERR_NOMEM;
  const int nbits = dtype == 0 ? 64 : 32;
  uint64_t prefix = 0;
  int64_t rank = kth;
  for (int shift = nbits - 8; shift >= 0; shift -= 8) {
    int rc = hist_pass(ctx, v, dtype, n, prefix, shift, hist, st);
    if (rc) return rc;
    OCM_HIP(hipMemcpyAsync(hh, hist, 256 * sizeof(uint64_t), hipMemcpyDeviceToHost, st));
    OCM_HIP(hipStreamSynchronize(st));
    int d = 0;
    for (; d < 256; ++d) {
      if (rank < (int64_t)hh[d]) break;
      rank -= (int64_t)hh[d];
    }
    if (d == 256) return ocm::fail(OCM_ERR_ARG, "radix select: rank out of range");
    prefix |= (uint64_t)d << shift;
  }
  *out = key_to_value(prefix, dtype);
  return OCM_OK;
}

}  // namespace

extern "C" {

int ocm_radix_hist(ocm_ctx* ctx, const void* v, int32_t dtype, int64_t n, uint64_t prefix, int32_t shift,
                   uint64_t* hist_out, void* stream) {
  OCM_REQUIRE(ctx && v && hist_out, "ocm_radix_hist: NULL argument");
  OCM_REQUIRE(dtype == 0 || dtype == 1, "ocm_radix_hist: dtype 0 (f64) or 1 (f32)");
  OCM_REQUIRE(shift >= 0 && shift % 8 == 0 && shift < (dtype == 0 ? 64 : 32), "ocm_radix_hist: bad shift");
  return hist_pass(ctx, v, dtype, n, prefix, shift, hist_out, (hipStream_t)stream);
}

int ocm_percentile(ocm_ctx* ctx, const void* v, int32_t dtype, int64_t n, double pct, double* out, void* stream) {
  OCM_REQUIRE(ctx && v && out, "ocm_percentile: NULL argument");
  OCM_REQUIRE(n >= 1, "ocm_percentile: empty input");
  OCM_REQUIRE(dtype == 0 || dtype == 1, "ocm_percentile: dtype 0 (f64) or 1 (f32)");
  OCM_REQUIRE(pct >= 0.0 && pct <= 100.0, "ocm_percentile: pct in [0, 100]");
  hipStream_t st = (hipStream_t)stream;
  // numpy 2.2 np.percentile(method='linear') evaluates everything in the
  // array's dtype (numpy/lib/_function_base_impl.py: q = pct / dtype(100),
  // virtual index (n-1)·q, gamma = vi - floor(vi), _lerp with the b-side
  // form for gamma >= 0.5); vi >= n-1 takes the last order statistic.
  if (dtype == 1) {
    const float q = (float)pct / 100.0f;
    const float vi = (float)(n - 1) * q;
    const float lo_f = std::floor(vi);
    const bool top = vi >= (float)(n - 1);
    const int64_t lo = top ? n - 1 : (int64_t)lo_f;
    const float g = vi - lo_f;
    double a = 0.0, b = 0.0;
    int rc = select_kth(ctx, v, dtype, n, lo, &a, st);
    if (rc) return rc;
    if (!top) {
      rc = select_kth(ctx, v, dtype, n, lo + 1, &b, st);
      if (rc) return rc;
    } else {
      b = a;
    }
    const float fa = (float)a, fb = (float)b, diff = fb - fa;
    *out = (double)((g >= 0.5f) ? fb - diff * (1.0f - g) : fa + diff * g);
    return OCM_OK;
  }
  const double q = pct / 100.0;
  const double vi = (double)(n - 1) * q;
  const double lo_d = std::floor(vi);
  const bool top = vi >= (double)(n - 1);
  const int64_t lo = top ? n - 1 : (int64_t)lo_d;
  const double g = vi - lo_d;
  double a = 0.0, b = 0.0;
  int rc = select_kth(ctx, v, dtype, n, lo, &a, st);
  if (rc) return rc;
  if (!top) {
    rc = select_kth(ctx, v, dtype, n, lo + 1, &b, st);
    if (rc) return rc;
  } else {
    b = a;
  }
  const double diff = b - a;
  *out = (g >= 0.5) ? b - diff * (1.0 - g) : a + diff * g;
  return OCM_OK;
}

}  // extern "C"
