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
  hipLaunchKernelGGL(k_snv_savgol, dim3((unsigned)m), dim3(256), (size_t)p * sizeof(double), st, X, ldx, m, p, snv,
                     window, dtaps, out, ldo);
  OCM_CHECK_LAUNCH("k_snv_savgol");
  return OCM_OK;
}

}  // extern "C"
