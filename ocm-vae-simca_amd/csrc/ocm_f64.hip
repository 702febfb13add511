// float64 spectra: the PCA precision follows the input dtype, as sklearn does
// for the reference's PCA(svd_solver='full') on float64 X
// (utils/SIMCA.py:64-66 → sklearn/decomposition/_pca.py:544-584: the SVD runs
// in the input dtype) and as its NumPy scoring does (utils/SIMCA.py:65-71,
// 104-107, 127-130: float64 T, X̂, residual and Q).
//
// k_gram_f64   shifted Gram Σ (x − s)(x − s)ᵀ on fp64 MFMA
//              (v_mfma_f64_16x16x4f64): 128×128 upper-triangle tiles, four
//              waves of 64×64 (4×4 blocks of 16×16, 128 accumulator VGPRs),
//              operands loaded straight from L2/HBM four row-steps ahead (16
//              MFMAs of 64 cycles per step hide them; no LDS, no barrier), rows
//              split into chunks whose fp64 partials are summed in a fixed order.
//              MFMA-bound: n·p(p+1) flops at the fp64 matrix rate.
// k_score_f64  t = P·(x − μ) on the same MFMA (M = 16 components, N = 16
//              spectra, K = 4 wavelengths per step) and T² = Σ t²/λ.
// k_qres_f64   Q = ‖(x − μ) − Pᵀt‖² as the reference forms it: the explicit
//              residual X − (T·P + μ) (utils/SIMCA.py:67-68, 71), not the
//              identity ‖y‖² − ‖t‖², which loses eps·‖y‖²/Q of Q's relative
//              accuracy on nearly low-rank data; Pᵀt on the same MFMA (M = 16
//              spectra, N = 16 wavelengths, K = 4 components per step), then the
//              fused decision and the χ² moment partials.  Two reads of X.
#include "ocm_internal.h"

#include <algorithm>

namespace {

typedef double f64x4 __attribute__((ext_vector_type(4)));

struct DecF64 {
  int32_t enabled;
  int32_t type;
  double t2_scale, q_scale, dlim;
};

// ---------------------------------------------------------------------------
// column mean (fp64 rows): per (column, row split) partial sums
// ---------------------------------------------------------------------------
__global__ void k_colsum_part_f64(const double* __restrict__ X, int64_t ldx, const int64_t* __restrict__ rows,
                                  int64_t n, int p, int64_t rows_per_split, double* __restrict__ part) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int sp = blockIdx.y;
  if (col >= p) return;
  const int64_t a = (int64_t)sp * rows_per_split;
  const int64_t e = min(n, a + rows_per_split);
  double v = 0.0;
  for (int64_t r = a; r < e; ++r) v += X[(rows ? rows[r] : r) * ldx + col];
  part[(size_t)sp * p + col] = v;
}

__global__ void k_colsum_final_f64(const double* __restrict__ part, int nsplit, int p, double inv_n,
                                   double* __restrict__ mean) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= p) return;
  double v = 0.0;
  for (int s = 0; s < nsplit; ++s) v += part[(size_t)s * p + col];
  mean[col] = v * inv_n;
}

// ---------------------------------------------------------------------------
// k_gram_f64
// ---------------------------------------------------------------------------
constexpr int GT64 = 128;  // tile edge
constexpr int GD64 = 4;    // row-steps (of 4 rows) loaded ahead

// f64 16x16x4 operand / result map (as k_dgemm): A[i][k] from lane (i = l&15,
// k = l>>4), B[k][j] from lane (k = l>>4, j = l&15), D[i][j] in lane
// (j = l&15) register r with i = (l>>4) + 4r.
__global__ __launch_bounds__(256, 1) void k_gram_f64(const double* __restrict__ X, int64_t ldx,
                                                     const int64_t* __restrict__ rows, int64_t r_begin,
                                                     int64_t r_end, int p, const float* __restrict__ shift,
                                                     int64_t chunk, int nt, double* __restrict__ part,
                                                     double* __restrict__ cpart) {
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int r16 = lane & 15, ks = lane >> 4;
  // linear upper-triangle tile index → (ti ≤ tj)
  int rem = blockIdx.x, ti = 0;
  while (rem >= nt - ti) {
    rem -= nt - ti;
    ++ti;
  }
  const int tj = ti + rem;
  const int ntiles = nt * (nt + 1) / 2;
  const int64_t c_lo = r_begin + (int64_t)blockIdx.y * chunk;
  const int64_t c_hi = min(r_end, c_lo + chunk);

  int ci[4], cj[4];
  double si[4], sj[4], mi[4], mj[4];
#pragma unroll
  for (int a = 0; a < 4; ++a) {
    const int gi = ti * GT64 + wm * 64 + 16 * a + r16;
    const int gj = tj * GT64 + wn * 64 + 16 * a + r16;
    mi[a] = gi < p ? 1.0 : 0.0;
    mj[a] = gj < p ? 1.0 : 0.0;
    ci[a] = gi < p ? gi : p - 1;
    cj[a] = gj < p ? gj : p - 1;
    si[a] = (double)shift[ci[a]];
    sj[a] = (double)shift[cj[a]];
  }
  f64x4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (f64x4){0.0, 0.0, 0.0, 0.0};
  double csum[4] = {0.0, 0.0, 0.0, 0.0};
  const bool want_cs = cpart && ti == tj && wn == 0;

  // ring of GD64 row-steps of operands (raw x and the row's validity)
  double ra[GD64][4], rb[GD64][4], rv[GD64];
  auto load = [&](int slot, int64_t r0) {
    const int64_t r = r0 + ks;
    const bool ok = r < c_hi;
    const int64_t rr = ok ? r : c_lo;  // a valid row, masked below
    const double* xr = X + (rows ? rows[rr] : rr) * ldx;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      ra[slot][a] = xr[ci[a]];
      rb[slot][a] = xr[cj[a]];
    }
    rv[slot] = ok ? 1.0 : 0.0;
  };
  const int64_t nsteps = (c_hi - c_lo + 3) / 4;
#pragma unroll
  for (int s = 0; s < GD64; ++s)
    if (s < nsteps) load(s, c_lo + 4 * s);
  for (int64_t s0 = 0; s0 < nsteps; s0 += GD64) {
#pragma unroll
    for (int s = 0; s < GD64; ++s) {
      if (s0 + s >= nsteps) break;
      double ya[4], yb[4];
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        ya[a] = (ra[s][a] - si[a]) * (rv[s] * mi[a]);
        yb[a] = (rb[s][a] - sj[a]) * (rv[s] * mj[a]);
      }
      if (s0 + s + GD64 < nsteps) load(s, c_lo + 4 * (s0 + s + GD64));
      if (want_cs)
#pragma unroll
        for (int a = 0; a < 4; ++a) csum[a] += ya[a];
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = __builtin_amdgcn_mfma_f64_16x16x4f64(ya[a], yb[b], acc[a][b], 0, 0, 0);
    }
  }
  double* tp = part + ((size_t)blockIdx.y * ntiles + blockIdx.x) * GT64 * GT64;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int il = wm * 64 + 16 * a + ks + 4 * r, jl = wn * 64 + 16 * b + r16;
        tp[il * GT64 + jl] = acc[a][b][r];
      }
  if (want_cs) {
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      double v = csum[a];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      if (ks == 0) cpart[((size_t)blockIdx.y * nt + ti) * GT64 + wm * 64 + 16 * a + r16] = v;
    }
  }
}

// chunk partials → G (both triangles) and column sums, fixed summation order
__global__ __launch_bounds__(256) void k_gram_f64_reduce(const double* __restrict__ part,
                                                         const double* __restrict__ cpart, int nchunks, int nt,
                                                         int p, double* __restrict__ G, double* __restrict__ colsum) {
  const int ntiles = nt * (nt + 1) / 2;
  const int tile = blockIdx.x / 64, sub = blockIdx.x % 64;
  int rem = tile, ti = 0;
  while (rem >= nt - ti) {
    rem -= nt - ti;
    ++ti;
  }
  const int tj = ti + rem;
  const int e = sub * 256 + threadIdx.x;  // element of the 128×128 tile
  const int il = e / GT64, jl = e % GT64;
  double v = 0.0;
  for (int c = 0; c < nchunks; ++c) v += part[((size_t)c * ntiles + tile) * GT64 * GT64 + e];
  const int gi = ti * GT64 + il, gj = tj * GT64 + jl;
  if (gi < p && gj < p) {
    G[(size_t)gi * p + gj] = v;
    G[(size_t)gj * p + gi] = v;
  }
  if (ti == tj && sub == 0 && threadIdx.x < GT64) {
    const int col = ti * GT64 + threadIdx.x;
    double s = 0.0;
    for (int c = 0; c < nchunks; ++c) s += cpart[((size_t)c * nt + ti) * GT64 + threadIdx.x];
    if (col < p) colsum[col] = s;
  }
}

// ---------------------------------------------------------------------------
// k_score_f64<NB, RB>: wave = RB blocks of 16 spectra, NB blocks of 16
// components (kb ≤ 16·NB); lane (row r16, k-slot ks) reads wavelengths
// c0 + 4·ks + e of its row for the four MFMA steps e of a 16-column chunk (the
// K order is permuted identically for P and y).
// T2_in (nullable): T² of earlier component blocks (k > 64); T2_out: the sum
// so far.  T_out (m × ldt, this block's columns) is always written: the
// residual pass reads it.
// ---------------------------------------------------------------------------
template <int NB, int RB>
__global__ __launch_bounds__(256) void k_score_f64(const double* __restrict__ X, int64_t ldx,
                                                   const int64_t* __restrict__ rows, int64_t m, int p,
                                                   const double* __restrict__ P, const double* __restrict__ mu,
                                                   const double* __restrict__ a_diag, int kb,
                                                   double* __restrict__ T_out, int64_t ldt,
                                                   const double* T2_in, double* T2_out) {  // T2_in may alias T2_out
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int r16 = lane & 15, ks = lane >> 4;
  const int64_t rbase = ((int64_t)blockIdx.x * 4 + wave) * (16 * RB);
  const double* xr[RB];
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int64_t g = rbase + 16 * rb + r16;
    const int64_t gc = g < m ? g : m - 1;
    xr[rb] = X + (rows ? rows[gc] : gc) * ldx;
  }
  const double* pr[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) {
    const int c = 16 * nb + r16;
    pr[nb] = P + (int64_t)(c < kb ? c : 0) * p;
  }
  double pmask[NB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb) pmask[nb] = 16 * nb + r16 < kb ? 1.0 : 0.0;

  f64x4 acc[NB][RB];
#pragma unroll
  for (int nb = 0; nb < NB; ++nb)
#pragma unroll
    for (int rb = 0; rb < RB; ++rb) acc[nb][rb] = (f64x4){0.0, 0.0, 0.0, 0.0};

  struct Ld {
    double x[RB][4];
    double w[NB][4];
    double u[4];
  };
  auto load = [&](Ld& L, int c0) {
    const int c = c0 + 4 * ks;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int cc = c + e < p ? c + e : p - 1;
      L.u[e] = c + e < p ? mu[cc] : 0.0;
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) L.x[rb][e] = c + e < p ? xr[rb][cc] : 0.0;
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) L.w[nb][e] = c + e < p ? pr[nb][cc] * pmask[nb] : 0.0;
    }
  };
  auto comp = [&](const Ld& L) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
#pragma unroll
      for (int rb = 0; rb < RB; ++rb) {
        const double y = L.x[rb][e] - L.u[e];
#pragma unroll
        for (int nb = 0; nb < NB; ++nb) acc[nb][rb] = __builtin_amdgcn_mfma_f64_16x16x4f64(L.w[nb][e], y, acc[nb][rb], 0, 0, 0);
      }
    }
  };
  Ld LA, LB;
  load(LA, 0);
  for (int c0 = 0; c0 < p; c0 += 32) {
    if (c0 + 16 < p) load(LB, c0 + 16);
    comp(LA);
    if (c0 + 32 < p) load(LA, c0 + 32);
    if (c0 + 16 < p) comp(LB);
  }

  // lane (r16, ks) holds t for spectrum r16 of each row block, components
  // 16·nb + ks + 4r; the four k-slot lanes of a spectrum combine by shuffles
#pragma unroll
  for (int rb = 0; rb < RB; ++rb) {
    const int64_t g = rbase + 16 * rb + r16;
    double t2 = 0.0;
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = 16 * nb + ks + 4 * r;
        const double t = acc[nb][rb][r];
        if (c < kb) {
          t2 += t * t * a_diag[c];
          if (g < m) T_out[g * ldt + c] = t;
        }
      }
    t2 += __shfl_xor(t2, 16, 64);
    t2 += __shfl_xor(t2, 32, 64);
    if (ks == 0 && g < m) T2_out[g] = T2_in ? T2_in[g] + t2 : t2;
  }
}

// ---------------------------------------------------------------------------
// k_qres_f64: one wave per 16 spectra.  For each 16-wavelength chunk the
// reconstruction (T·P)[i][c] is one 16×16 MFMA tile over the k components
// (A = T rows: lane (i = l&15, kk = l>>4) holds T[i][4s + kk]; B = P: lane
// (kk = l>>4, j = l&15) holds P[4s + kk][c0 + j]; D[i][j] in lane (j = l&15),
// register r, i = (l>>4) + 4r); lane (j, kk) then forms r = (x − μ) − D for
// its four spectra at wavelength c0 + j and accumulates r².  The 16 wavelength
// lanes of a spectrum combine by shuffles.  Q, the fused decision (on the
// final T²) and the χ² moment partials follow.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_qres_f64(const double* __restrict__ X, int64_t ldx,
                                                  const int64_t* __restrict__ rows, int64_t m, int p,
                                                  const double* __restrict__ P, const double* __restrict__ mu, int k,
                                                  const double* __restrict__ T, const double* __restrict__ T2,
                                                  double* __restrict__ Q_out, DecF64 dec,
                                                  double* __restrict__ acc_out, int64_t acc_stride,
                                                  double* __restrict__ stat_part) {
  __shared__ double sred[16];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int j = lane & 15, kk = lane >> 4;
  const int64_t rbase = ((int64_t)blockIdx.x * 4 + wave) * 16;
  // A operand row (spectrum rbase + j) and the four spectra this lane's
  // accumulator registers belong to (rbase + kk + 4r)
  const int64_t ga = rbase + j;
  const double* trow = T + (ga < m ? ga : m - 1) * (int64_t)k;
  const double amask = ga < m ? 1.0 : 0.0;
  const double* xr[4];
  double rmask[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t g = rbase + kk + 4 * r;
    const int64_t gc = g < m ? g : m - 1;
    xr[r] = X + (rows ? rows[gc] : gc) * ldx;
    rmask[r] = g < m ? 1.0 : 0.0;
  }
  const int nsteps = (k + 3) / 4;
  double q[4] = {0.0, 0.0, 0.0, 0.0};
  for (int c0 = 0; c0 < p; c0 += 16) {
    const int c = c0 + j;
    const int cc = c < p ? c : p - 1;
    const double cmask = c < p ? 1.0 : 0.0;
    double y[4];
    const double u = mu[cc];
#pragma unroll
    for (int r = 0; r < 4; ++r) y[r] = xr[r][cc] - u;
    f64x4 d = (f64x4){0.0, 0.0, 0.0, 0.0};
    for (int s = 0; s < nsteps; ++s) {
      const int comp = 4 * s + kk;
      const int ce = comp < k ? comp : k - 1;
      const double okc = comp < k ? 1.0 : 0.0;
      const double a = trow[ce] * (amask * okc);
      const double b = P[(int64_t)ce * p + cc] * (okc * cmask);
      d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, d, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const double res = (y[r] - d[r]) * (cmask * rmask[r]);
      q[r] += res * res;
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    q[r] += __shfl_xor(q[r], 1, 64);
    q[r] += __shfl_xor(q[r], 2, 64);
    q[r] += __shfl_xor(q[r], 4, 64);
    q[r] += __shfl_xor(q[r], 8, 64);
  }
  double st[4] = {0.0, 0.0, 0.0, 0.0};
  if (j == 0) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t g = rbase + kk + 4 * r;
      if (g < m) {
        const double t2 = T2[g];
        Q_out[g] = q[r];
        if (dec.enabled) {
          const double dd = ocm::dred_of(dec.type, t2 * dec.t2_scale, q[r] * dec.q_scale);
          acc_out[g * acc_stride] = dd < dec.dlim ? 1.0 : 0.0;
        }
        st[0] += t2;
        st[1] += t2 * t2;
        st[2] += q[r];
        st[3] += q[r] * q[r];
      }
    }
  }
  if (stat_part) {
#pragma unroll
    for (int i = 0; i < 4; ++i) st[i] = wave_sum_f64(st[i]);
    if (lane == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i) sred[wave * 4 + i] = st[i];
    __syncthreads();
    if (tid < 4)
      stat_part[(int64_t)blockIdx.x * 4 + tid] =
          (sred[tid] + sred[4 + tid]) + (sred[8 + tid] + sred[12 + tid]);
  }
}

__global__ __launch_bounds__(1024) void k_stats_reduce_f64(const double* __restrict__ part, int64_t nblk,
                                                           double* __restrict__ out) {
  __shared__ double red[16];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int col = w & 3, sl = w >> 2;
  double v = 0.0;
  for (int64_t i = (int64_t)sl * 64 + lane; i < nblk; i += 256) v += part[i * 4 + col];
  v = wave_sum_f64(v);
  if (lane == 0) red[w] = v;
  __syncthreads();
  if (threadIdx.x < 4)
    out[threadIdx.x] = (red[threadIdx.x] + red[4 + threadIdx.x]) + (red[8 + threadIdx.x] + red[12 + threadIdx.x]);
}

__global__ void k_decide_f64(const double* __restrict__ T2, const double* __restrict__ Q, int64_t m, DecF64 dec,
                             double* __restrict__ t2red, double* __restrict__ qred, double* __restrict__ dred,
                             double* __restrict__ acc, int64_t acc_stride) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= m) return;
  const double t = T2[i] * dec.t2_scale;
  const double q = Q[i] * dec.q_scale;
  if (t2red) t2red[i] = t;
  if (qred) qred[i] = q;
  const double d = ocm::dred_of(dec.type, t, q);
  if (dred) dred[i] = d;
  if (acc) acc[i * acc_stride] = d < dec.dlim ? 1.0 : 0.0;
}

constexpr int SF_RB = 4;  // row blocks of 16 per wave

template <int NB>
void launch_score_f64(dim3 g, hipStream_t st, const double* X, int64_t ldx, const int64_t* rows, int64_t m, int p,
                      const double* P, const double* mu, const double* a, int kb, double* T, int64_t ldt,
                      const double* T2_in, double* T2_out) {
  hipLaunchKernelGGL((k_score_f64<NB, SF_RB>), g, dim3(256), 0, st, X, ldx, rows, m, p, P, mu, a, kb, T, ldt, T2_in,
                     T2_out);
}

}  // namespace

extern "C" {

int ocm_colmean_f64(ocm_ctx* ctx, const double* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                    double* mean_out, void* stream) {
  OCM_REQUIRE(ctx && X && mean_out, "ocm_colmean_f64: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p, "ocm_colmean_f64: bad shape");
  hipStream_t st = (hipStream_t)stream;
  const int64_t per = 32;
  const int nsplit = (int)std::min<int64_t>((n + per - 1) / per, 4096);
  const int64_t rps = (n + nsplit - 1) / nsplit;
  auto* part = static_cast<double*>(ocm::workspace(ctx, (size_t)nsplit * p * sizeof(double), st));
  if (!part) return OCM_ERR_NOMEM;
  hipLaunchKernelGGL(k_colsum_part_f64, dim3((p + 255) / 256, nsplit), dim3(256), 0, st, X, ldx, rows, n, p, rps, part);
  OCM_CHECK_LAUNCH("k_colsum_part_f64");
  hipLaunchKernelGGL(k_colsum_final_f64, dim3((p + 255) / 256), dim3(256), 0, st, part, nsplit, p, 1.0 / (double)n,
                     mean_out);
  OCM_CHECK_LAUNCH("k_colsum_final_f64");
  return OCM_OK;
}

int ocm_gram_f64(ocm_ctx* ctx, const double* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                 const float* shift, const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out,
                 void* stream) {
  OCM_REQUIRE(ctx && X && shift && seg_offsets && G_out && colsum_out, "ocm_gram_f64: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p && nseg > 0, "ocm_gram_f64: bad shape");
  OCM_REQUIRE(seg_offsets[0] == 0 && seg_offsets[nseg] == n, "ocm_gram_f64: seg_offsets must span [0, n]");
  for (int s = 0; s < nseg; ++s)
    OCM_REQUIRE(seg_offsets[s + 1] >= seg_offsets[s], "ocm_gram_f64: seg_offsets not ascending");
  hipStream_t st = (hipStream_t)stream;
  const int nt = (p + GT64 - 1) / GT64;
  const int ntiles = nt * (nt + 1) / 2;
  int64_t maxseg = 0;
  for (int s = 0; s < nseg; ++s) maxseg = std::max(maxseg, seg_offsets[s + 1] - seg_offsets[s]);
  // ≈ 4 workgroups per CU over all chunks; ≥ 64 rows per chunk
  const int nchunk_max = (int)std::max<int64_t>(1, std::min<int64_t>((4 * ctx->num_cus + ntiles - 1) / ntiles,
                                                                      (maxseg + 63) / 64));
  const size_t part_n = (size_t)nchunk_max * ntiles * GT64 * GT64;
  const size_t cpart_n = (size_t)nchunk_max * nt * GT64;
  void* w = ocm::workspace(ctx, (part_n + cpart_n) * sizeof(double) + 1024, st);
  if (!w) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(w)};
  double* part = cv.take<double>(part_n);
  double* cpart = cv.take<double>(cpart_n);
  for (int s = 0; s < nseg; ++s) {
    const int64_t a = seg_offsets[s], b = seg_offsets[s + 1];
    double* G = G_out + (size_t)s * p * p;
    double* cs = colsum_out + (size_t)s * p;
    if (b == a) {
      OCM_HIP(hipMemsetAsync(G, 0, (size_t)p * p * sizeof(double), st));
      OCM_HIP(hipMemsetAsync(cs, 0, (size_t)p * sizeof(double), st));
      continue;
    }
    const int64_t len = b - a;
    const int nch = (int)std::min<int64_t>(nchunk_max, (len + 63) / 64);
    const int64_t chunk = ((len + nch - 1) / nch + 3) / 4 * 4;
    const int nchunks = (int)((len + chunk - 1) / chunk);
    {
      ocm::TimedRegion tr(ctx, OCM_KERNEL_GRAM, st);
      hipLaunchKernelGGL(k_gram_f64, dim3(ntiles, nchunks), dim3(256), 0, st, X, ldx, rows, a, b, p, shift, chunk, nt,
                         part, cpart);
    }
    OCM_CHECK_LAUNCH("k_gram_f64");
    hipLaunchKernelGGL(k_gram_f64_reduce, dim3(ntiles * 64), dim3(256), 0, st, part, cpart, nchunks, nt, p, G, cs);
    OCM_CHECK_LAUNCH("k_gram_f64_reduce");
  }
  return OCM_OK;
}

int ocm_score_f64_diag(ocm_ctx* ctx, const double* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                       const double* P, const double* mu, const double* a_diag, int32_t k, double* T_out,
                       double* T2_out, double* Q_out, const ocm_decision* dec, double* accept_out,
                       int64_t accept_stride, double* stats_out, void* stream) {
  OCM_REQUIRE(ctx && X && P && mu && a_diag, "ocm_score_f64_diag: NULL argument");
  OCM_REQUIRE(m >= 0 && p > 0 && ldx >= p, "ocm_score_f64_diag: bad shape");
  OCM_REQUIRE(k >= 1 && k <= p, "ocm_score_f64_diag: 1 <= k <= p");
  OCM_REQUIRE(!dec || accept_out, "ocm_score_f64_diag: decision requires accept_out");
  hipStream_t st = (hipStream_t)stream;
  if (m == 0) {
    if (stats_out) OCM_HIP(hipMemsetAsync(stats_out, 0, 4 * sizeof(double), st));
    return OCM_OK;
  }
  const int64_t rows_per_wg = 4 * 16 * SF_RB;
  const int64_t nblk = (m + rows_per_wg - 1) / rows_per_wg;
  const int64_t nblk_q = (m + 63) / 64;  // k_qres_f64: 64 spectra per workgroup
  OCM_REQUIRE(nblk_q < (1LL << 31), "ocm_score_f64_diag: too many rows");
  constexpr int KB = 64;
  const int nkb = (k + KB - 1) / KB;
  const size_t part_n = stats_out ? (size_t)nblk_q * 4 : 0;
  const size_t t_n = T_out ? 0 : (size_t)m * k;  // the residual pass needs T
  const size_t t2_n = T2_out ? 0 : (size_t)m;
  const size_t q_n = Q_out ? 0 : (size_t)m;
  void* w = ocm::workspace(ctx, (part_n + t_n + t2_n + q_n) * sizeof(double) + 1024, st);
  if (!w) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(w)};
  double* part = stats_out ? cv.take<double>(part_n) : nullptr;
  double* Tw = T_out ? T_out : cv.take<double>((size_t)m * k);
  double* T2w = T2_out ? T2_out : cv.take<double>(m);
  double* Qw = Q_out ? Q_out : cv.take<double>(m);
  DecF64 d{};
  if (dec) d = DecF64{1, dec->type, dec->t2_scale, dec->q_scale, dec->dlim};
  const dim3 g((unsigned)nblk);
  for (int bk = 0; bk < nkb; ++bk) {
    const int c0 = bk * KB, kb = std::min(KB, k - c0);
    ocm::TimedRegion tr(ctx, OCM_KERNEL_SCORE, st);
    const double* Pb = P + (size_t)c0 * p;
    const double* ab = a_diag + c0;
    const double* T2i = bk == 0 ? nullptr : T2w;
    if (kb <= 16)
      launch_score_f64<1>(g, st, X, ldx, rows, m, p, Pb, mu, ab, kb, Tw + c0, k, T2i, T2w);
    else if (kb <= 32)
      launch_score_f64<2>(g, st, X, ldx, rows, m, p, Pb, mu, ab, kb, Tw + c0, k, T2i, T2w);
    else
      launch_score_f64<4>(g, st, X, ldx, rows, m, p, Pb, mu, ab, kb, Tw + c0, k, T2i, T2w);
    OCM_CHECK_LAUNCH("k_score_f64");
  }
  if (Q_out || dec || stats_out) {
    hipLaunchKernelGGL(k_qres_f64, dim3((unsigned)nblk_q), dim3(256), 0, st, X, ldx, rows, m, p, P, mu, k, Tw, T2w,
                       Qw, d, accept_out, accept_stride, part);
    OCM_CHECK_LAUNCH("k_qres_f64");
  }
  if (stats_out) {
    hipLaunchKernelGGL(k_stats_reduce_f64, dim3(1), dim3(1024), 0, st, part, nblk_q, stats_out);
    OCM_CHECK_LAUNCH("k_stats_reduce_f64");
  }
  return OCM_OK;
}

int ocm_decide_f64(ocm_ctx* ctx, const double* T2, const double* Q, int64_t m, const ocm_decision* dec,
                   double* t2red_out, double* qred_out, double* dred_out, double* accept_out, int64_t accept_stride,
                   void* stream) {
  OCM_REQUIRE(ctx && T2 && Q && dec, "ocm_decide_f64: NULL argument");
  if (m <= 0) return OCM_OK;
  DecF64 d{1, dec->type, dec->t2_scale, dec->q_scale, dec->dlim};
  hipLaunchKernelGGL(k_decide_f64, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, (hipStream_t)stream, T2, Q, m, d,
                     t2red_out, qred_out, dred_out, accept_out, accept_stride);
  OCM_CHECK_LAUNCH("k_decide_f64");
  return OCM_OK;
}

}  // extern "C"
