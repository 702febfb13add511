// K4 / K7 / K9 — per-spectrum projection, Q (orthogonal) and Hotelling T²
// distances, fused decision; reconstruction residual norms for the VAE.
//
// Reference math: utils/SIMCA.py:65-71 (fit), 104-107 (transform), 127-145
// (predict + decision), sklearn/decomposition/_base.py:147-153,197
// (transform / inverse_transform), vae_model.py:164.
//
// Layout: a wave owns 32 spectra; a workgroup (4 waves) 128 spectra.  The
// row tile streams through LDS in 64-wavelength chunks (coalesced 256-B row
// segments, mean subtracted on the way in) next to the matching 64-column
// slice of the loadings P.  Two sweeps over the chunks:
//   sweep 1  Tᵀ (comps × rows) += P_chunk · D_chunkᵀ        v_mfma_f32_32x32x2_f32
//   sweep 2  Rᵀ (cols × rows)   = P_chunkᵀ · Tᵀ → r = d − R, q += r²
// Sweep 2 feeds the sweep-1 accumulator registers straight back as the B
// operand (its column is already on the lane), so T never leaves registers.
// Q is the explicit residual (first-order insensitive to error in t, unlike
// the ‖d‖² − ‖t‖² identity).  T is flushed to f64 every chunk.  The second
// sweep re-reads the tile, served from L2/Infinity Cache.
#include "ocm_internal.h"

namespace {

constexpr int SW = 4;   // waves per workgroup
constexpr int SR = 32;  // spectra per wave
constexpr int SC = 64;  // wavelengths per chunk
constexpr int SROWS = SW * SR;

struct DecArgs {
  int32_t enabled;
  int32_t type;
  double t2_scale, q_scale, dlim;
};

__device__ __forceinline__ double dred_of(int type, double t, double q) {
  switch (type) {
    case OCM_TYPE_SIM: return fmax(t, q);
    case OCM_TYPE_ALT: return sqrt(t * t + q * q);
    default: return t + q;  // ci, dd
  }
}

template <int KT, bool VEC>
__global__ __launch_bounds__(256) void k_score(const float* __restrict__ X, int64_t ldx,
                                               const int64_t* __restrict__ rows, int64_t m, int p,
                                               const float* __restrict__ P, const float* __restrict__ mu,
                                               const double* __restrict__ A, int k, int a_diag,
                                               float* __restrict__ T_out, double* __restrict__ T2_out,
                                               float* __restrict__ Q_out, DecArgs dec, double* __restrict__ acc_out,
                                               int64_t acc_stride, double* __restrict__ stat_part) {
  constexpr int KP = KT * 32;
  constexpr int D_FLOATS = SW * SR * (SC + 1);
  constexpr int P_FLOATS = KP * (SC + 1);
  constexpr int MAIN_BYTES = (D_FLOATS + P_FLOATS) * 4;
  constexpr int EPI_BYTES = SW * SR * (KP + 1) * 8;
  constexpr int LDS_BYTES = MAIN_BYTES > EPI_BYTES ? MAIN_BYTES : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];
  __shared__ double sred[SW][4];
  float* Ds = reinterpret_cast<float*>(smem);
  float* Ps = Ds + D_FLOATS;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * SROWS + wave * SR;
  float* Dw = Ds + wave * SR * (SC + 1);

  // loaders: D chunk — lane → (row = 4j + lane/16, col4 = (lane%16)*4), j < 8
  const int dcol = (lane & 15) * 4, drow = lane >> 4;
  int64_t srow[8];
  unsigned rmask = 0;  // bit j: row j of this lane's loader set is real
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t g = row0 + 4 * j + drow;
    const bool ok = g < m;
    rmask |= ok ? (1u << j) : 0u;
    const int64_t gc = ok ? g : m - 1;  // clamp: always a valid address
    srow[j] = rows ? rows[gc] : gc;
  }
  // P chunk — thread → (comp = e/16, col4 = (e%16)*4), e = tid + 256·i
  constexpr int PV = KP * SC / 4 / 256;  // float4 per thread (2 or 4)

  // Branch-free prefetch (clamped addresses, loads left in flight); the mean
  // subtraction and the row / column / component masks are applied in
  // sstore, after the MFMAs that hide the loads.
  f32x4 rd[8], rp[PV], rmu;
  auto ld4 = [&](const float* base, int col) -> f32x4 {
    if (VEC) return *reinterpret_cast<const f32x4*>(base + (col < p ? col : 0));
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = base[min(col + e, p - 1)];
    return v;
  };
  auto gload = [&](int c0) {
    rmu = ld4(mu, c0 + dcol);
#pragma unroll
    for (int j = 0; j < 8; ++j) rd[j] = ld4(X + srow[j] * ldx, c0 + dcol);
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = tid + 256 * i;
      const int comp = e >> 4, col = (e & 15) * 4;
      rp[i] = ld4(P + (int64_t)min(comp, k - 1) * p, c0 + col);
    }
  };
  auto sstore = [&](int c0) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float* d = Dw + (4 * j + drow) * (SC + 1) + dcol;
      const bool rv = (rmask >> j) & 1u;
#pragma unroll
      for (int e = 0; e < 4; ++e) d[e] = (rv && c0 + dcol + e < p) ? rd[j][e] - rmu[e] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < PV; ++i) {
      const int e = tid + 256 * i;
      const int comp = e >> 4, col = (e & 15) * 4;
      float* d = Ps + comp * (SC + 1) + col;
#pragma unroll
      for (int q = 0; q < 4; ++q) d[q] = (comp < k && c0 + col + q < p) ? rp[i][q] : 0.f;
    }
  };

  const int nchunk = (p + SC - 1) / SC;
  f32x16 accT[KT];
  double accT64[KT][16];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      accT[t][r] = 0.f;
      accT64[t][r] = 0.0;
    }

  // ---- sweep 1: projection ------------------------------------------------
  gload(0);
  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();  // previous chunk's LDS reads are done
    sstore(c * SC);
    __syncthreads();
    if (c + 1 < nchunk) gload((c + 1) * SC);
#pragma unroll
    for (int s = 0; s < SC / 2; ++s) {
      const float b = Dw[l31 * (SC + 1) + 2 * s + h];
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const float a = Ps[(t * 32 + l31) * (SC + 1) + 2 * s + h];
        accT[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, accT[t], 0, 0, 0);
      }
    }
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        accT64[t][r] += (double)accT[t][r];
        accT[t][r] = 0.f;
      }
  }

  // T back to f32 as the sweep-2 B operand
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) accT[t][r] = (float)accT64[t][r];

  // ---- sweep 2: reconstruction residual ------------------------------------
  double q64 = 0.0;
  gload(0);
  for (int c = 0; c < nchunk; ++c) {
    __syncthreads();
    sstore(c * SC);
    __syncthreads();
    if (c + 1 < nchunk) gload((c + 1) * SC);
    float qc = 0.f;
#pragma unroll
    for (int cb = 0; cb < SC / 32; ++cb) {
      f32x16 accR;
#pragma unroll
      for (int r = 0; r < 16; ++r) accR[r] = 0.f;
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int comp = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
          const float a = Ps[comp * (SC + 1) + cb * 32 + l31];
          accR = __builtin_amdgcn_mfma_f32_32x32x2f32(a, accT[t][r], accR, 0, 0, 0);
        }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int col = cb * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const float d = Dw[l31 * (SC + 1) + col] - accR[r];
        qc += d * d;
      }
    }
    q64 += (double)qc;
  }
  q64 += __shfl_xor(q64, 32, 64);

  // ---- epilogue: gather T rows through LDS (f64), T², decision, stats ------
  __syncthreads();
  double* Tt = reinterpret_cast<double*>(smem) + wave * SR * (KP + 1);
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int comp = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
      Tt[l31 * (KP + 1) + comp] = accT64[t][r];
    }
  __syncthreads();
  const int64_t grow = row0 + l31;
  const bool own = (h == 0) && (grow < m);
  double T2 = 0.0, Q = q64;
  if (own) {
    const double* trow = Tt + l31 * (KP + 1);
    if (a_diag) {
      for (int a = 0; a < k; ++a) T2 += trow[a] * trow[a] * A[a * k + a];
    } else {
      for (int a = 0; a < k; ++a) {
        double s = 0.0;
        for (int b = 0; b < k; ++b) s += A[a * k + b] * trow[b];
        T2 += trow[a] * s;
      }
    }
    if (T_out)
      for (int a = 0; a < k; ++a) T_out[grow * k + a] = (float)trow[a];
    if (T2_out) T2_out[grow] = T2;
    if (Q_out) Q_out[grow] = (float)Q;
    if (dec.enabled) {
      const double dr = dred_of(dec.type, T2 * dec.t2_scale, (double)(float)Q * dec.q_scale);
      acc_out[grow * acc_stride] = dr < dec.dlim ? 1.0 : 0.0;
    }
  }
  if (stat_part) {
    const double qf = (double)(float)Q;
    double s0 = own ? T2 : 0.0, s1 = own ? T2 * T2 : 0.0, s2 = own ? qf : 0.0, s3 = own ? qf * qf : 0.0;
    s0 = wave_sum_f64(s0);
    s1 = wave_sum_f64(s1);
    s2 = wave_sum_f64(s2);
    s3 = wave_sum_f64(s3);
    if (lane == 0) {
      sred[wave][0] = s0;
      sred[wave][1] = s1;
      sred[wave][2] = s2;
      sred[wave][3] = s3;
    }
    __syncthreads();
    if (tid < 4) {
      double v = 0.0;
      for (int w = 0; w < SW; ++w) v += sred[w][tid];
      stat_part[(int64_t)blockIdx.x * 4 + tid] = v;
    }
  }
}

__global__ void k_stats_reduce(const double* __restrict__ part, int64_t nblk, double* __restrict__ out) {
  // 4 waves, wave w sums column w in a fixed order (deterministic)
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double v = 0.0;
  for (int64_t i = lane; i < nblk; i += 64) v += part[i * 4 + w];
  v = wave_sum_f64(v);
  if (lane == 0) out[w] = v;
}

__global__ void k_decide(const double* __restrict__ T2, const float* __restrict__ Q, int64_t m, DecArgs dec,
                         double* __restrict__ t2red, double* __restrict__ qred, double* __restrict__ dred,
                         double* __restrict__ acc, int64_t acc_stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const double t = T2[i] * dec.t2_scale;
  const double q = (double)Q[i] * dec.q_scale;
  if (t2red) t2red[i] = t;
  if (qred) qred[i] = q;
  const double d = dred_of(dec.type, t, q);
  if (dred) dred[i] = d;
  if (acc) acc[i * acc_stride] = d < dec.dlim ? 1.0 : 0.0;
}

// q_i = Σ_j (x_ij − x̂_ij)², one wave per row, f64 accumulation
__global__ __launch_bounds__(256) void k_rowsq(const float* __restrict__ x, const float* __restrict__ xh, int64_t m,
                                               int p, int64_t ld, float* __restrict__ q) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= m) return;
  double s = 0.0;
  for (int j = lane; j < p; j += 64) {
    const float d = x[r * ld + j] - xh[r * ld + j];
    s += (double)d * d;
  }
  s = wave_sum_f64(s);
  if (lane == 0) q[r] = (float)s;
}

__global__ void k_cast_f64_f32(const double* __restrict__ a, int64_t n, float* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (float)a[i];
}

}  // namespace

extern "C" {

int ocm_score_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                  const float* P, const float* mu, const double* A, int32_t k, float* T_out, double* T2_out,
                  float* Q_out, const ocm_decision* dec, double* accept_out, int64_t accept_stride,
                  double* stats_out, void* stream) {
  OCM_REQUIRE(ctx && X && P && mu && A, "ocm_score_f32: NULL argument");
  OCM_REQUIRE(m >= 0 && p > 0 && ldx >= p, "ocm_score_f32: bad shape");
  OCM_REQUIRE(k >= 1 && k <= 64, "ocm_score_f32: 1 <= k <= 64");
  OCM_REQUIRE(!dec || accept_out, "ocm_score_f32: decision requires accept_out");
  hipStream_t st = (hipStream_t)stream;
  if (m == 0) {
    if (stats_out) OCM_HIP(hipMemsetAsync(stats_out, 0, 4 * sizeof(double), st));
    return OCM_OK;
  }
  const int64_t nblk = (m + SROWS - 1) / SROWS;
  OCM_REQUIRE(nblk < (1LL << 31), "ocm_score_f32: too many rows");
  double* part = nullptr;
  if (stats_out) {
    part = static_cast<double*>(ocm::workspace(ctx, (size_t)nblk * 4 * sizeof(double), st));
    if (!part) return OCM_ERR_NOMEM;
  }
  const int a_diag = 0;  // general k×k quadratic form (k² FMAs per row are negligible)
  DecArgs d{};
  if (dec) {
    d.enabled = 1;
    d.type = dec->type;
    d.t2_scale = dec->t2_scale;
    d.q_scale = dec->q_scale;
    d.dlim = dec->dlim;
  }
  const bool vec = (ldx % 4 == 0) && (p % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0) &&
                   ((reinterpret_cast<uintptr_t>(P) & 15) == 0);
  dim3 g((unsigned)nblk);
  {
    ocm::TimedRegion tr(ctx, OCM_KERNEL_SCORE, st);
#define OCM_SCORE_LAUNCH(KT_, V_)                                                                              \
  hipLaunchKernelGGL((k_score<KT_, V_>), g, dim3(256), 0, st, X, ldx, rows, m, p, P, mu, A, k, a_diag, T_out, \
                     T2_out, Q_out, d, accept_out, accept_stride, part)
    if (k <= 32) {
      if (vec) OCM_SCORE_LAUNCH(1, true); else OCM_SCORE_LAUNCH(1, false);
    } else {
      if (vec) OCM_SCORE_LAUNCH(2, true); else OCM_SCORE_LAUNCH(2, false);
    }
#undef OCM_SCORE_LAUNCH
  }
  OCM_CHECK_LAUNCH("k_score");
  if (stats_out) {
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(256), 0, st, part, nblk, stats_out);
    OCM_CHECK_LAUNCH("k_stats_reduce");
  }
  return OCM_OK;
}

int ocm_decide(ocm_ctx* ctx, const double* T2, const float* Q, int64_t m, const ocm_decision* dec, double* t2red_out,
               double* qred_out, double* dred_out, double* accept_out, int64_t accept_stride, void* stream) {
  OCM_REQUIRE(ctx && T2 && Q && dec, "ocm_decide: NULL argument");
  if (m <= 0) return OCM_OK;
  DecArgs d{1, dec->type, dec->t2_scale, dec->q_scale, dec->dlim};
  hipLaunchKernelGGL(k_decide, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, T2, Q, m, d,
                     t2red_out, qred_out, dred_out, accept_out, accept_stride);
  OCM_CHECK_LAUNCH("k_decide");
  return OCM_OK;
}

int ocm_rowsq_residual_f32(ocm_ctx* ctx, const float* x, const float* xhat, int64_t m, int32_t p, int64_t ld,
                           float* q_out, void* stream) {
  OCM_REQUIRE(ctx && x && xhat && q_out, "ocm_rowsq_residual_f32: NULL argument");
  OCM_REQUIRE(p > 0 && ld >= p, "ocm_rowsq_residual_f32: bad shape");
  if (m <= 0) return OCM_OK;
  hipLaunchKernelGGL(k_rowsq, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, xhat, m, p, ld,
                     q_out);
  OCM_CHECK_LAUNCH("k_rowsq");
  return OCM_OK;
}

int ocm_cast_f64_f32(ocm_ctx* ctx, const double* a, int64_t n, float* b, void* stream) {
  OCM_REQUIRE(ctx && a && b, "ocm_cast_f64_f32: NULL argument");
  if (n <= 0) return OCM_OK;
  hipLaunchKernelGGL(k_cast_f64_f32, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, a, n, b);
  OCM_CHECK_LAUNCH("k_cast_f64_f32");
  return OCM_OK;
}

}  // extern "C"
