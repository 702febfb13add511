// K4 / K7 / K9 — per-spectrum projection, Q (orthogonal) and Hotelling T²
// distances, fused decision; reconstruction residual norms for the VAE.
//
// Reference math: utils/SIMCA.py:65-71 (fit), 104-107 (transform), 127-145
// (predict + decision), sklearn/decomposition/_base.py:147-153,197
// (transform / inverse_transform), vae_model.py:164.
//
// k_score_direct: f32 MFMA, each wave streams its 32 rows from HBM straight
// into operand registers; loadings / mean in LDS blocks.  Two sweeps over the
// row's columns:
//   sweep 1  Tᵀ (comps × rows) += P_chunk · D_chunkᵀ        v_mfma_f32_32x32x2_f32
//   sweep 2  Rᵀ (cols × rows)   = P_chunkᵀ · Tᵀ → r = d − R, q += r²
// Sweep 2 feeds the sweep-1 accumulator registers straight back as the B
// operand (its column is already on the lane), so T never leaves registers.
// Q is the explicit residual (first-order insensitive to error in t, unlike
// the ‖d‖² − ‖t‖² identity, which f32 accumulation cannot afford).  T is
// flushed to f64 every chunk.
#include "ocm_internal.h"

namespace {

constexpr int SW = 4;   // waves per workgroup
constexpr int SR = 32;  // spectra per wave
constexpr int SROWS = SW * SR;

struct DecArgs {
  int32_t enabled;
  int32_t type;
  double t2_scale, q_scale, dlim;
};

using ocm::dred_of;

// Shared epilogue: T rows gathered through LDS (f64), T² = tᵀ A t, Q, fused
// decision, per-workgroup moment partials.  accT64 holds Tᵀ in the 32×32 MFMA
// accumulator layout: comp = 32t + (r&3) + 8(r>>2) + 4h, row = lane & 31.
template <int KT, int NW>
__device__ __forceinline__ void score_epilogue(double* tls, double* sred, const double (&accT64)[KT][16], double q64,
                                               int64_t row0, int64_t m, int k, int a_diag,
                                               const double* __restrict__ A, float* __restrict__ T_out,
                                               double* __restrict__ T2_out, float* __restrict__ Q_out, DecArgs dec,
                                               double* __restrict__ acc_out, int64_t acc_stride,
                                               double* __restrict__ stat_part) {
  constexpr int KP = KT * 32;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  __syncthreads();
  double* Tt = tls + wave * 32 * (KP + 1);
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
      sred[wave * 4 + 0] = s0;
      sred[wave * 4 + 1] = s1;
      sred[wave * 4 + 2] = s2;
      sred[wave * 4 + 3] = s3;
    }
    __syncthreads();
    if (tid < 4) {
      double v = 0.0;
      for (int w = 0; w < NW; ++w) v += sred[w * 4 + tid];
      stat_part[(int64_t)blockIdx.x * 4 + tid] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// k_score_direct — the default scoring kernel.  Every wave streams its own
// 32 rows from HBM straight into MFMA operand registers (double-buffered,
// two named register sets, loop unrolled by 2); the loadings and the mean
// are staged per workgroup in LDS in 256-column blocks (one barrier pair per
// block, i.e. per 8 MFMA chunks), so waves never wait on each other inside a
// block.  The K order is permuted so that lane (row = lane&31, half h) reads
// contiguous 16-B pieces of its row: in a 32-column chunk, MFMA step 4i+e
// uses column 8i + 4h + e (i, e < 4) for the data (B) and loadings (A) alike.
// ---------------------------------------------------------------------------
constexpr int PB = 256;  // columns per LDS loadings block

template <int KT, bool VEC>
__global__ __launch_bounds__(256, 2) void k_score_direct(const float* __restrict__ X, int64_t ldx,
                                                         const int64_t* __restrict__ rows, int64_t m, int p,
                                                         const float* __restrict__ P, const float* __restrict__ mu,
                                                         const double* __restrict__ A, int k, int a_diag,
                                                         float* __restrict__ T_out, double* __restrict__ T2_out,
                                                         float* __restrict__ Q_out, DecArgs dec,
                                                         double* __restrict__ acc_out, int64_t acc_stride,
                                                         double* __restrict__ stat_part) {
  constexpr int KP = KT * 32;
  constexpr int PS = PB + 4;  // padded LDS row: conflict-free ds_read_b128 across comps
  constexpr int MAIN_F = KP * PS + PB;
  constexpr int EPI_F = SW * SR * (KP + 1) * 2;
  __shared__ __attribute__((aligned(16))) float smem[MAIN_F > EPI_F ? MAIN_F : EPI_F];
  __shared__ double sred[SW * 4];
  float* Pl = smem;             // [KP][PS]
  float* Ml = smem + KP * PS;   // [PB]
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l31 = lane & 31, h = lane >> 5;
  const int64_t row0 = (int64_t)blockIdx.x * SROWS + wave * SR;
  const int64_t grow = row0 + l31;
  const float rowmask = grow < m ? 1.f : 0.f;
  const int64_t gcl = grow < m ? grow : m - 1;
  const float* xrow = X + (rows ? rows[gcl] : gcl) * ldx;

  auto ld4 = [&](const float* base, int col) -> f32x4 {
    if (VEC) return *reinterpret_cast<const f32x4*>(base + (col < p ? col : 0));
    f32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e) v[e] = base[min(col + e, p - 1)];
    return v;
  };
  // stage loadings / mean columns [b0, b0+PB) into LDS (zero outside k, p)
  auto stage = [&](int b0) {
    __syncthreads();  // previous block fully consumed
    for (int e = tid; e < KP * (PB / 4); e += 256) {
      const int comp = e / (PB / 4), c4 = (e % (PB / 4)) * 4;
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      if (comp < k) v = ld4(P + (int64_t)comp * p, b0 + c4);
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (b0 + c4 + q >= p) v[q] = 0.f;
      *reinterpret_cast<f32x4*>(&Pl[comp * PS + c4]) = v;
    }
    for (int c = tid; c < PB; c += 256) Ml[c] = b0 + c < p ? mu[b0 + c] : 0.f;
    __syncthreads();
  };

  f32x16 accT[KT];
  double accT64[KT][16];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      accT[t][r] = 0.f;
      accT64[t][r] = 0.0;
    }

  // ---- sweep 1: Tᵀ = P · Dᵀ, 32-column chunks ---------------------------------
  // data set for one chunk: d[i] = x[8i + 4h .. +3]
  struct S1 {
    f32x4 d[4];
  };
  auto load1 = [&](S1& S, int c0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) S.d[i] = ld4(xrow, c0 + 8 * i + 4 * h);
  };
  auto comp1 = [&](const S1& S, int c0, int b0) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int lc = c0 - b0 + 8 * i + 4 * h;  // column within the LDS block
      const f32x4 u = *reinterpret_cast<const f32x4*>(&Ml[lc]);
      f32x4 w[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) w[t] = *reinterpret_cast<const f32x4*>(&Pl[(t * 32 + l31) * PS + lc]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        // padded columns have u = 0 and w = 0, so only the row mask is needed
        const float b = (S.d[i][e] - u[e]) * rowmask;
#pragma unroll
        for (int t = 0; t < KT; ++t) accT[t] = __builtin_amdgcn_mfma_f32_32x32x2f32(w[t][e], b, accT[t], 0, 0, 0);
      }
    }
  };
  for (int b0 = 0; b0 < p; b0 += PB) {
    stage(b0);
    const int bend = min(b0 + PB, p);
    S1 SA, SB;
    load1(SA, b0);
    for (int c0 = b0; c0 < bend; c0 += 64) {
      load1(SB, c0 + 32);
      comp1(SA, c0, b0);
      if (c0 + 64 < bend) load1(SA, c0 + 64);
      if (c0 + 32 < bend) comp1(SB, c0 + 32, b0);
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
  f32x16 accTf[KT];
#pragma unroll
  for (int t = 0; t < KT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) accTf[t][r] = (float)accT64[t][r];

  // ---- sweep 2: Rᵀ = Pᵀ · Tᵀ per 32-column chunk, Q = Σ (d − R)² -------------
  // step r consumes comps κ_r + 4h (κ_r = (r&3) + 8(r>>2)); for k ≤ 24 the
  // trailing steps hold only zero loadings and are skipped.
  const int nsteps = KT == 1 ? (k > 24 ? 16 : (k > 16 ? 12 : (k > 8 ? 8 : 4))) : 16;
  double q64 = 0.0;
  auto comp2 = [&](const S1& S, int c0, int b0) {
    f32x16 accR;
#pragma unroll
    for (int r = 0; r < 16; ++r) accR[r] = 0.f;
    const int lcol = c0 - b0 + l31;
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        if (KT == 1 && r >= nsteps) break;
        const int comp = t * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        accR = __builtin_amdgcn_mfma_f32_32x32x2f32(Pl[comp * PS + lcol], accTf[t][r], accR, 0, 0, 0);
      }
    float qc = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      // accR register 4g+e holds column 8g + 4h + e of the chunk (row lane&31)
      const int col = c0 + 8 * g + 4 * h;
      const f32x4 u = *reinterpret_cast<const f32x4*>(&Ml[col - b0]);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float cm = col + e < p ? 1.f : 0.f;  // clamped loads beyond p carry data
        const float r = ((S.d[g][e] - u[e]) - accR[4 * g + e]) * cm;
        qc += r * r;
      }
    }
    q64 += (double)(qc * rowmask);
  };
  // same per-lane column pieces as sweep 1 (8g + 4h), so load1 is reused
  for (int b0 = 0; b0 < p; b0 += PB) {
    stage(b0);
    const int bend = min(b0 + PB, p);
    S1 SA, SB;
    load1(SA, b0);
    for (int c0 = b0; c0 < bend; c0 += 64) {
      load1(SB, c0 + 32);
      comp2(SA, c0, b0);
      if (c0 + 64 < bend) load1(SA, c0 + 64);
      if (c0 + 32 < bend) comp2(SB, c0 + 32, b0);
    }
  }
  q64 += __shfl_xor(q64, 32, 64);

  score_epilogue<KT, SW>(reinterpret_cast<double*>(smem), sred, accT64, q64, row0, m, k, a_diag, A, T_out, T2_out,
                         Q_out, dec, acc_out, acc_stride, stat_part);
}

__global__ __launch_bounds__(1024) void k_stats_reduce(const double* __restrict__ part, int64_t nblk,
                                                       double* __restrict__ out) {
  // 16 waves: wave w sums column w & 3 over row slice w >> 2 (4 slices), four
  // independent accumulators per lane; slices combined in a fixed order
  // (deterministic)
  __shared__ double red[16];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = w & 3, sl = w >> 2;
  double v0 = 0.0, v1 = 0.0, v2 = 0.0, v3 = 0.0;
  int64_t i = (int64_t)sl * 64 + lane;
  for (; i + 3 * 256 < nblk; i += 4 * 256) {
    v0 += part[i * 4 + col];
    v1 += part[(i + 256) * 4 + col];
    v2 += part[(i + 512) * 4 + col];
    v3 += part[(i + 768) * 4 + col];
  }
  for (; i < nblk; i += 256) v0 += part[i * 4 + col];
  double v = wave_sum_f64((v0 + v1) + (v2 + v3));
  if (lane == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x < 4) out[threadIdx.x] = (red[threadIdx.x] + red[4 + threadIdx.x]) + (red[8 + threadIdx.x] + red[12 + threadIdx.x]);
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
__global__ __launch_bounds__(256) void k_rowsq(const float* __restrict__ x, int64_t ldx, const float* __restrict__ xh,
                                               int64_t ldxh, int64_t m, int p, float* __restrict__ q) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= m) return;
  double s = 0.0;
  for (int j = lane; j < p; j += 64) {
    const double d = (double)x[r * ldx + j] - (double)xh[r * ldxh + j];
    s += d * d;
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
                  const double* P, const double* mu, const double* A, int32_t k, float* T_out, double* T2_out,
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
  const int64_t rows_per_blk = SROWS;
  const int64_t nblk = (m + rows_per_blk - 1) / rows_per_blk;
  OCM_REQUIRE(nblk < (1LL << 31), "ocm_score_f32: too many rows");
  const size_t part_bytes = stats_out ? (size_t)nblk * 4 * sizeof(double) : 0;
  const size_t cast_bytes = ((size_t)k * p + p) * sizeof(float) + 512;
  void* w = ocm::workspace(ctx, part_bytes + cast_bytes + 1024, st);
  if (!w) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(w)};
  double* part = stats_out ? cv.take<double>((size_t)nblk * 4) : nullptr;
  // the f32 kernel takes f32 loadings / mean
  float* P32 = cv.take<float>((size_t)k * p);
  float* mu32 = cv.take<float>(p);
  hipLaunchKernelGGL(k_cast_f64_f32, dim3((unsigned)(((int64_t)k * p + 255) / 256)), dim3(256), 0, st, P,
                     (int64_t)k * p, P32);
  hipLaunchKernelGGL(k_cast_f64_f32, dim3((p + 255) / 256), dim3(256), 0, st, mu, (int64_t)p, mu32);
  OCM_CHECK_LAUNCH("k_cast_f64_f32");
  const int a_diag = 0;  // general k×k quadratic form (k² FMAs per row are negligible)
  DecArgs d{};
  if (dec) {
    d.enabled = 1;
    d.type = dec->type;
    d.t2_scale = dec->t2_scale;
    d.q_scale = dec->q_scale;
    d.dlim = dec->dlim;
  }
  const bool vec = (ldx % 4 == 0) && (p % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  dim3 g((unsigned)nblk);
  {
    ocm::TimedRegion tr(ctx, OCM_KERNEL_SCORE, st);
#define OCM_SCORE_LAUNCH(KT_, V_)                                                                          \
  hipLaunchKernelGGL((k_score_direct<KT_, V_>), g, dim3(256), 0, st, X, ldx, rows, m, p, P32, mu32, A, k, a_diag, \
                     T_out, T2_out, Q_out, d, accept_out, accept_stride, part)
    if (k <= 32) {
      if (vec) OCM_SCORE_LAUNCH(1, true); else OCM_SCORE_LAUNCH(1, false);
    } else {
      if (vec) OCM_SCORE_LAUNCH(2, true); else OCM_SCORE_LAUNCH(2, false);
    }
#undef OCM_SCORE_LAUNCH
  }
  OCM_CHECK_LAUNCH("k_score");
  if (stats_out) {
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(1024), 0, st, part, nblk, stats_out);
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

int ocm_rowsq_residual_f32(ocm_ctx* ctx, const float* x, int64_t ldx, const float* xhat, int64_t ldxh, int64_t m,
                           int32_t p, float* q_out, void* stream) {
  OCM_REQUIRE(ctx && x && xhat && q_out, "ocm_rowsq_residual_f32: NULL argument");
  OCM_REQUIRE(p > 0 && ldx >= p && (ldxh == 0 || ldxh >= p), "ocm_rowsq_residual_f32: bad shape");
  if (m <= 0) return OCM_OK;
  hipLaunchKernelGGL(k_rowsq, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, ldx, xhat, ldxh, m,
                     p, q_out);
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
