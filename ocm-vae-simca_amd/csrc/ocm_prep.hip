// Spectral preprocessing of the drivers:
//   SNV   x ← (x − mean_row) / (std_row + 1e-8)     (simca_nuts.py:47-49,
//         utils/data_utils.py:57; np.std with ddof 0)
//   Savitzky–Golay  scipy.signal.savgol_filter(x, w, polyorder, deriv, axis=1,
//         mode='interp')                            (simca_nuts.py:51,
//         simca_new_cheese.py:37-38, utils/data_utils.py:59)
// as one HBM pass per row (read p floats, write p floats).  mode='interp'
// is linear in the samples: interior points use the w-tap convolution
// coefficients, the first / last w/2 points the least-squares polynomial fit
// of the first / last w samples evaluated (and differentiated) there.  The
// host builds those coefficient tables (taps) once per (w, polyorder, deriv,
// delta); the kernel applies them from LDS.
#include <algorithm>

#include "ocm_internal.h"

namespace {

constexpr int PREP_MAXW = 63;

// One workgroup per row.  taps layout: [w] interior, then [half][w] left edge,
// then [half][w] right edge (edge row j applies to output j / p−half+j).
__global__ __launch_bounds__(256) void k_snv_savgol(const float* __restrict__ X, int64_t ldx, int64_t m, int p,
                                                    int snv, int w, const double* __restrict__ taps,
                                                    float* __restrict__ out, int64_t ldo) {
  extern __shared__ double srow[];  // p doubles
  __shared__ double stap[PREP_MAXW * (PREP_MAXW + 2)];
  __shared__ double red[8];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t r = blockIdx.x;
  const int half = w / 2;
  const int ntap = w > 0 ? w + 2 * half * w : 0;
  for (int i = tid; i < ntap; i += 256) stap[i] = taps[i];
  const float* xr = X + r * ldx;
  double s = 0.0;
  for (int j = tid; j < p; j += 256) {
    const double v = (double)xr[j];
    srow[j] = v;
    s += v;
  }
  if (snv) {
    // two-pass moments in fp64: mean, then Σ(x − mean)²
    s = wave_sum_f64(s);
    if (lane == 0) red[wave] = s;
    __syncthreads();
    const double mean = ((red[0] + red[1]) + (red[2] + red[3])) / p;
    __syncthreads();
    double ss = 0.0;
    for (int j = tid; j < p; j += 256) {
      const double d = srow[j] - mean;
      ss += d * d;
    }
    ss = wave_sum_f64(ss);
    if (lane == 0) red[4 + wave] = ss;
    __syncthreads();
    // the reference works in the array dtype: mean / std rounded to float32
    const float meanf = (float)mean;
    const float sdf = (float)sqrt(((red[4] + red[5]) + (red[6] + red[7])) / p);
    const float den = sdf + 1e-8f;
    for (int j = tid; j < p; j += 256) srow[j] = (double)(((float)srow[j] - meanf) / den);
  }
  __syncthreads();
  float* orow = out + r * ldo;
  if (w <= 0) {
    for (int j = tid; j < p; j += 256) orow[j] = (float)srow[j];
    return;
  }
  for (int j = tid; j < p; j += 256) {
    const double* c;
    int start;
    if (j < half) {
      c = stap + w + j * w;
      start = 0;
    } else if (j >= p - half) {
      c = stap + w + half * w + (j - (p - half)) * w;
      start = p - w;
    } else {
      c = stap;
      start = j - half;
    }
    double acc = 0.0;
    for (int t = 0; t < w; ++t) acc += c[t] * srow[start + t];
    orow[j] = (float)acc;
  }
}

// Fast path (p % 4 == 0, p ≤ 4096, window ∈ {none, 5, 15}: the drivers'
// filters): one wave per row, four rows per workgroup.  Each lane holds the
// float4 pieces at columns 256k + 4·lane (coalesced 1-KiB wave loads and
// stores); the row moments are wave reductions (no LDS, no block barrier);
// for Savitzky–Golay the SNV row goes to a wave-private LDS row and each lane
// forms its four outputs from a (W + 3)-sample window with the interior taps
// in registers.  Same arithmetic as k_snv_savgol: fp64 moments rounded to
// float32, the f32 SNV division, fp64 filter sums rounded to float32.
constexpr int PREP_SEGS_MAX = 16;  // p ≤ 4096 (the register tile holds p / 256 float4 per lane)
template <int W, int PREP_MAXSEG>
__global__ __launch_bounds__(256) void k_snv_sg4(const float* __restrict__ X, int64_t ldx, int64_t m, int p, int snv,
                                                 const double* __restrict__ taps, float* __restrict__ out,
                                                 int64_t ldo) {
  extern __shared__ float srow4[];  // [4][p] (W > 0)
  constexpr int H = W / 2;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  const bool valid = r < m;
  const int nseg = (p + 255) / 256;
  const float* xr = X + (valid ? r : 0) * ldx;
  f32x4 x[PREP_MAXSEG];
#pragma unroll
  for (int k = 0; k < PREP_MAXSEG; ++k) {
    const int c0 = 256 * k + 4 * lane;
    x[k] = (k < nseg && c0 < p) ? *reinterpret_cast<const f32x4*>(xr + c0) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if (snv) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < PREP_MAXSEG; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += (double)x[k][e];
    const double mean = wave_sum_f64(s) / p;
    double ss = 0.0;
#pragma unroll
    for (int k = 0; k < PREP_MAXSEG; ++k) {
      const int c0 = 256 * k + 4 * lane;
      if (k < nseg && c0 < p)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double d = (double)x[k][e] - mean;
          ss += d * d;
        }
    }
    const float meanf = (float)mean;
    const float sdf = (float)sqrt(wave_sum_f64(ss) / p);
    const float den = sdf + 1e-8f;
#pragma unroll
    for (int k = 0; k < PREP_MAXSEG; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) x[k][e] = (x[k][e] - meanf) / den;
  }
  float* orow = out + (valid ? r : 0) * ldo;
  if constexpr (W == 0) {
    if (valid)
#pragma unroll
      for (int k = 0; k < PREP_MAXSEG; ++k) {
        const int c0 = 256 * k + 4 * lane;
        if (k < nseg && c0 < p) *reinterpret_cast<f32x4*>(orow + c0) = x[k];
      }
    return;
  } else {
    float* row = srow4 + (size_t)wave * p;
    // all taps (interior + both edge tables) once per workgroup, after the rows
    double* stp = reinterpret_cast<double*>(srow4 + (size_t)4 * p + ((4 * p) & 1));
    for (int i = threadIdx.x; i < W + 2 * H * W; i += 256) stp[i] = taps[i];
#pragma unroll
    for (int k = 0; k < PREP_MAXSEG; ++k) {
      const int c0 = 256 * k + 4 * lane;
      if (k < nseg && c0 < p) *reinterpret_cast<f32x4*>(row + c0) = x[k];
    }
    __syncthreads();
    double ct[W];
#pragma unroll
    for (int t = 0; t < W; ++t) ct[t] = taps[t];  // interior taps (wave-uniform)
    if (!valid) return;
#pragma unroll
    for (int k = 0; k < PREP_MAXSEG; ++k) {
      const int j0 = 256 * k + 4 * lane;
      if (!(k < nseg && j0 < p)) continue;
      f32x4 o;
      if (j0 - H >= 0 && j0 + 3 + H < p) {
        double win[W + 3];
#pragma unroll
        for (int t = 0; t < W + 3; ++t) win[t] = (double)row[j0 - H + t];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          double acc = 0.0;
#pragma unroll
          for (int t = 0; t < W; ++t) acc += ct[t] * win[i + t];
          o[i] = (float)acc;
        }
      } else {  // the first / last H outputs: the least-squares edge fits
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int j = j0 + i;
          const double* c;
          int start;
          if (j < H) {
            c = stp + W + j * W;
            start = 0;
          } else if (j >= p - H) {
            c = stp + W + H * W + (j - (p - H)) * W;
            start = p - W;
          } else {
            c = stp;
            start = j - H;
          }
          double acc = 0.0;
#pragma unroll
          for (int t = 0; t < W; ++t) acc += c[t] * (double)row[start + t];
          o[i] = (float)acc;
        }
      }
      *reinterpret_cast<f32x4*>(orow + j0) = o;
    }
  }
}


// ---- lazy-view support (include/ocm.h ocm_prep) ---------------------------
// Row statistics of the SNV, the one read-only pre-pass of the fused path:
// (m_r, s_r) = (mean_r, 1/(std_r + 1e-8)), fp64 moments rounded to float32 as
// k_snv_sg4 forms them.  One wave per row, four rows per workgroup; p ≤ 4096
// keeps the row in registers (two-pass moments without a second read).
template <int MAXSEG>
__global__ __launch_bounds__(256) void k_prep_rowstats(const float* __restrict__ X, int64_t ldx, int64_t m, int p,
                                                       float* __restrict__ out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * 4 + wave;
  if (r >= m) return;
  const float* xr = X + r * ldx;
  double mean, ss = 0.0;
  if constexpr (MAXSEG > 0) {
    const int nseg = (p + 255) / 256;
    f32x4 x[MAXSEG];
#pragma unroll
    for (int k = 0; k < MAXSEG; ++k) {
      const int c0 = 256 * k + 4 * lane;
      x[k] = (k < nseg && c0 < p) ? *reinterpret_cast<const f32x4*>(xr + c0) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < MAXSEG; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) s += (double)x[k][e];
    mean = wave_sum_f64(s) / p;
#pragma unroll
    for (int k = 0; k < MAXSEG; ++k) {
      const int c0 = 256 * k + 4 * lane;
      if (k < nseg && c0 < p)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const double d = (double)x[k][e] - mean;
          ss += d * d;
        }
    }
  } else {  // any p: two passes over the row (the second from cache)
    double s = 0.0;
    for (int c = lane; c < p; c += 64) s += (double)xr[c];
    mean = wave_sum_f64(s) / p;
    for (int c = lane; c < p; c += 64) {
      const double d = (double)xr[c] - mean;
      ss += d * d;
    }
  }
  const float sdf = (float)sqrt(wave_sum_f64(ss) / p);
  if (lane == 0) {
    out[2 * r] = (float)mean;
    out[2 * r + 1] = 1.f / (sdf + 1e-8f);
  }
}

// The materialised view (fallback shapes, tests): one thread per output
// element, the scalar formula (its window loads hit the L1).
__global__ __launch_bounds__(256) void k_prep_apply(const float* __restrict__ X, int64_t ldx,
                                                    const int64_t* __restrict__ rows, int p, PrepArgs pa,
                                                    float* __restrict__ out, int64_t ldo, int64_t i0) {
  const int j = blockIdx.x * 256 + threadIdx.x;
  const int64_t i = i0 + blockIdx.y;
  if (j >= p) return;
  const int64_t r = rows ? rows[i] : i;
  float mr = 0.f, sr = 1.f;
  if (pa.snv) {
    mr = pa.rowstat[2 * r];
    sr = pa.rowstat[2 * r + 1];
  }
  out[i * ldo + j] = ocm::prep_elem(X + r * ldx, p, j, pa, mr, sr);
}

}  // namespace

namespace ocm {

// Checks shared by every *_prep entry point.
int check_prep(const ocm_prep* prep, int p, const char* who) {
  OCM_REQUIRE(prep, std::string(who) + ": NULL prep");
  const int w = prep->window;
  OCM_REQUIRE(w == 0 || (w % 2 == 1 && w >= 3 && w <= 31 && w <= p), std::string(who) +
              ": prep window must be 0 or odd in [3, 31] and <= p");
  OCM_REQUIRE(w == 0 || prep->taps, std::string(who) + ": prep taps required");
  OCM_REQUIRE(!prep->snv || prep->rowstat, std::string(who) + ": SNV needs rowstat");
  OCM_REQUIRE(prep->deriv >= 0 && (w > 0 || prep->deriv == 0), std::string(who) + ": bad deriv");
  OCM_REQUIRE(w > 0 || prep->snv, std::string(who) + ": empty prep (no SNV, no filter)");
  return OCM_OK;
}

int prep_apply(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int p, const PrepArgs& pa,
               float* out, int64_t ldo, hipStream_t st) {
  for (int64_t i0 = 0; i0 < m; i0 += 65535) {  // grid y ≤ 65535 rows per launch
    const unsigned cnt = (unsigned)std::min<int64_t>(65535, m - i0);
    hipLaunchKernelGGL(k_prep_apply, dim3((unsigned)((p + 255) / 256), cnt), dim3(256), 0, st, X, ldx, rows, p, pa,
                       out, ldo, i0);
  }
  OCM_CHECK_LAUNCH("k_prep_apply");
  return OCM_OK;
}

}  // namespace ocm

namespace {
}  // namespace

extern "C" {

int ocm_snv_savgol_f32(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t m, int32_t p, int32_t snv,
                       int32_t window, const double* taps, float* out, int64_t ldo, void* stream) {
  OCM_REQUIRE(ctx && X && out, "ocm_snv_savgol_f32: NULL argument");
  OCM_REQUIRE(m >= 0 && p >= 1 && ldx >= p && ldo >= p, "ocm_snv_savgol_f32: bad shape");
  OCM_REQUIRE(window == 0 || (window % 2 == 1 && window >= 1 && window <= PREP_MAXW && window <= p && taps),
              "ocm_snv_savgol_f32: window must be odd, <= 63 and <= p (taps required)");
  OCM_REQUIRE((size_t)p * sizeof(double) <= 96 * 1024, "ocm_snv_savgol_f32: p > 12288 not supported");
  if (m == 0) return OCM_OK;
  hipStream_t st = (hipStream_t)stream;
  const double* dtaps = nullptr;
  if (window > 0) {
    const int ntap = window + 2 * (window / 2) * window;
    auto* w = static_cast<double*>(ocm::workspace(ctx, (size_t)ntap * sizeof(double) + 256, st));
    if (!w) return OCM_ERR_NOMEM;
    OCM_HIP(hipMemcpyAsync(w, taps, (size_t)ntap * sizeof(double), hipMemcpyHostToDevice, st));
    dtaps = w;
  }
  OCM_REQUIRE(m < (1LL << 31), "ocm_snv_savgol_f32: too many rows per call");
  bool fast = p % 4 == 0 && p <= 256 * PREP_SEGS_MAX && ldx % 4 == 0 && ldo % 4 == 0 &&
                    (reinterpret_cast<uintptr_t>(X) & 15) == 0 && (reinterpret_cast<uintptr_t>(out) & 15) == 0 &&
                    (window == 0 || window == 5 || window == 15) && p >= window + 3;
  const size_t lds = window > 0 ? (size_t)(4 * p + 2) * sizeof(float) +
                                      (size_t)(window + 2 * (window / 2) * window) * sizeof(double)
                                : 0;
  int max_lds = 0;  // the wave-private rows must fit the device's LDS (160 KiB on gfx950)
  OCM_HIP(hipDeviceGetAttribute(&max_lds, hipDeviceAttributeMaxSharedMemoryPerBlock, ctx->device));
  if (fast && lds > (size_t)max_lds) fast = false;
  if (fast) {
    const dim3 g((unsigned)((m + 3) / 4));
#define OCM_SG4(W_, S_) hipLaunchKernelGGL((k_snv_sg4<W_, S_>), g, dim3(256), lds, st, X, ldx, m, p, snv, dtaps, out, ldo)
#define OCM_SG4_S(W_) \
  if (p <= 1024)      \
    OCM_SG4(W_, 4);   \
  else if (p <= 2048) \
    OCM_SG4(W_, 8);   \
  else                \
    OCM_SG4(W_, 16);
    if (window == 0) {
      OCM_SG4_S(0)
    } else if (window == 5) {
      OCM_SG4_S(5)
    } else {
      OCM_SG4_S(15)
    }
#undef OCM_SG4_S
#undef OCM_SG4
    OCM_CHECK_LAUNCH("k_snv_sg4");
    return OCM_OK;
  }
  hipLaunchKernelGGL(k_snv_savgol, dim3((unsigned)m), dim3(256), (size_t)p * sizeof(double), st, X, ldx, m, p, snv,
                     window, dtaps, out, ldo);
  OCM_CHECK_LAUNCH("k_snv_savgol");
  return OCM_OK;
}

int ocm_prep_rowstats_f32(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t m, int32_t p, float* rowstat_out,
                          void* stream) {
  OCM_REQUIRE(ctx && X && rowstat_out, "ocm_prep_rowstats_f32: NULL argument");
  OCM_REQUIRE(m >= 0 && p >= 1 && ldx >= p, "ocm_prep_rowstats_f32: bad shape");
  if (m == 0) return OCM_OK;
  hipStream_t st = (hipStream_t)stream;
  const dim3 g((unsigned)((m + 3) / 4));
  const bool vec = p % 4 == 0 && ldx % 4 == 0 && (reinterpret_cast<uintptr_t>(X) & 15) == 0;
  if (vec && p <= 1024)
    hipLaunchKernelGGL(k_prep_rowstats<4>, g, dim3(256), 0, st, X, ldx, m, p, rowstat_out);
  else if (vec && p <= 2048)
    hipLaunchKernelGGL(k_prep_rowstats<8>, g, dim3(256), 0, st, X, ldx, m, p, rowstat_out);
  else if (vec && p <= 4096)
    hipLaunchKernelGGL(k_prep_rowstats<16>, g, dim3(256), 0, st, X, ldx, m, p, rowstat_out);
  else
    hipLaunchKernelGGL(k_prep_rowstats<0>, g, dim3(256), 0, st, X, ldx, m, p, rowstat_out);
  OCM_CHECK_LAUNCH("k_prep_rowstats");
  return OCM_OK;
}

int ocm_eig_test_reruns(ocm_ctx* ctx, int64_t* count_out) {
  OCM_REQUIRE(ctx && count_out, "ocm_eig_test_reruns: NULL argument");
  *count_out = ctx->eig_test_reruns;
  return OCM_OK;
}

int ocm_prep_materialised(ocm_ctx* ctx, int64_t* count_out) {
  OCM_REQUIRE(ctx && count_out, "ocm_prep_materialised: NULL argument");
  *count_out = ctx->prep_materialised;
  return OCM_OK;
}

int ocm_prep_apply_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                       const ocm_prep* prep, float* out, int64_t ldo, void* stream) {
  OCM_REQUIRE(ctx && X && out, "ocm_prep_apply_f32: NULL argument");
  OCM_REQUIRE(m >= 0 && p >= 1 && ldx >= p && ldo >= p, "ocm_prep_apply_f32: bad shape");
  if (int rc = ocm::check_prep(prep, p, "ocm_prep_apply_f32")) return rc;
  return ocm::prep_apply(ctx, X, ldx, rows, m, p, ocm::prep_args(prep), out, ldo, (hipStream_t)stream);
}

}  // extern "C"
