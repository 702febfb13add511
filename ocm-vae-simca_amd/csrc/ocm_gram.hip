// K1 — shifted Gram / column sums on FP32 MFMA, and the covariance built
// from it.  Replaces the full SVD of the centred class matrix in
// utils/SIMCA.py:64-66 (sklearn/decomposition/_pca.py:544-584): the SIMCA
// fit needs the eigen-decomposition of C = Σ(x-μ)(x-μ)ᵀ/(n-1), and C is one
// dense contraction over the spectra rows.
//
// Layout: X row-major n×p float32 (spectra × wavelengths).  A workgroup owns
// one GT×GT tile (ti ≤ tj, upper triangle only) of G = Σ yᵀy (y = x − shift)
// over one chunk of rows; it streams BK-row panels of the two column blocks
// through double-buffered LDS (coalesced row segments, shift subtracted on
// the way in) and accumulates with v_mfma_f32_32x32x2_f32 (exact f32 FMA
// chain).  Waves tile the output 2 (M) × GT/64 (N), each wave GT/2 × 64 =
// (GT/64) × 2 MFMA tiles.  Chunk partials (f32, ≤ 8192 rows each ≈ 6e-8·√L
// relative) are summed in f64 by a second kernel.  Diagonal tiles also
// accumulate the column sums (f64).  Workgroup ids are remapped so that
// consecutive tiles of one row chunk land on one XCD and share its L2.
//   GT = 256 (default): 8 waves, BK = 16, 64 KiB LDS, 128 accumulators/lane.
//   GT = 128:           4 waves, BK = 32, 64 KiB LDS,  64 accumulators/lane.
#include <cstring>
#include <string>
#include <vector>

#include "ocm_internal.h"

namespace {

// One value of the (possibly preprocessed) row `r` of X: the sample kernels
// (shift, outlier thresholds) and the exact fix-up read through this.
__device__ __forceinline__ float load_y(const float* __restrict__ X, int64_t ldx, int64_t r, int col, int p,
                                        const PrepArgs& pa) {
  if (pa.w == 0 && !pa.snv) return X[r * ldx + col];
  float m = 0.f, sc = 1.f;
  if (pa.snv) {
    m = pa.rowstat[2 * r];
    sc = pa.rowstat[2 * r + 1];
  }
  return ocm::prep_elem(X + r * ldx, p, col, pa, m, sc);
}


constexpr int MAXSEG = 32;

struct SegTable {
  int64_t begin[MAXSEG + 1];   // processed-row offsets of the segments
  int32_t cprefix[MAXSEG + 1]; // cumulative chunk counts
  int32_t nseg;
  int32_t chunk_rows;
};

__device__ __forceinline__ void tile_coords(int t, int nt, int& ti, int& tj) {
  ti = 0;
  while (t >= nt - ti) {
    t -= nt - ti;
    ++ti;
  }
  tj = ti + t;
}

template <int GT, int BK_>
struct GramCfg {
  static constexpr int BK = BK_;                        // rows per LDS stage
  static constexpr int WN = GT / 64;                    // waves along N
  static constexpr int THREADS = 2 * WN * 64;           // 2 × WN waves
  static constexpr int MT = GT / 64;                    // 32-row MFMA tiles per wave (M = GT/2)
  static constexpr int C4 = GT / 4;                     // float4 per panel row
  static constexpr int RSTEP = THREADS / C4;            // rows per loader pass
  static constexpr int LPP = BK / RSTEP;                // loader passes per panel
};

constexpr int GATHER_MAX_CHUNK = 2048;  // rows per chunk when a row-index list is used

template <int GT, int BK_, bool VEC, bool GATHER>
__global__ __launch_bounds__(GT * 2, 2) void k_gram(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ rows, int p, const float* __restrict__ shift,
    SegTable st, int nt, int ntiles, int total_wg, float* __restrict__ part, double* __restrict__ colpart) {
  using Cfg = GramCfg<GT, BK_>;
  constexpr int BK = Cfg::BK, MT = Cfg::MT, LPP = Cfg::LPP, RSTEP = Cfg::RSTEP;
  __shared__ __attribute__((aligned(16))) float lds[2][2][BK][GT];  // [buf][A/B][row][col]
  __shared__ int64_t ridx[GATHER ? GATHER_MAX_CHUNK : 1];           // chunk's row indices

  // XCD-aware bijective remap: blocks b ≡ x (mod 8) share an XCD; give each
  // XCD a contiguous range of logical ids (chunk-major, tile-minor).
  const int b = blockIdx.x;
  const int q8 = total_wg / 8, r8 = total_wg % 8, x8 = b % 8;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int chunk = wg / ntiles;
  const int tile = wg - chunk * ntiles;
  int ti, tj;
  tile_coords(tile, nt, ti, tj);
  const bool diag = (ti == tj);
  const int I = ti * GT, J = tj * GT;

  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  const int nstage = (int)((r1 - r0 + BK - 1) / BK);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave / Cfg::WN, wn = wave % Cfg::WN;
  if (GATHER) {
    // stage the chunk's row indices in LDS so that X loads never wait on an
    // index load (vmcnt is in-order: it would drain the prefetch as well)
    for (int64_t g = r0 + tid; g < r1; g += Cfg::THREADS) ridx[g - r0] = rows[g];
    __syncthreads();
  }
  const int l31 = lane & 31, h = lane >> 5;

  // loader: C4 float4 per panel row, RSTEP rows per pass, LPP passes
  const int c4 = tid % Cfg::C4, rr = tid / Cfg::C4;
  f32x4 shA, shB;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ca = I + 4 * c4 + e, cb = J + 4 * c4 + e;
    shA[e] = ca < p ? shift[ca] : 0.f;
    shB[e] = cb < p ? shift[cb] : 0.f;
  }

  f32x4 ra[LPP], rb[LPP];
  double csum64[4] = {0.0, 0.0, 0.0, 0.0};

  // Branch-free prefetch: addresses are clamped into valid memory and the
  // loads are left in flight; the shift subtraction and the row / column
  // masks are applied in sstore (after the MFMAs), so no load is waited on
  // before the compute that should hide it.
  const int colA = I + 4 * c4, colB = J + 4 * c4;
  // VEC requires p % 4 == 0: a float4 is then entirely inside or outside [0, p)
  const bool inA = colA < p, inB = colB < p;
  const float* baseA = X + (inA ? colA : 0);
  const float* baseB = X + (inB ? colB : 0);
  auto gload = [&](int stage) {
#pragma unroll
    for (int j = 0; j < LPP; ++j) {
      int64_t g = r0 + (int64_t)stage * BK + rr + RSTEP * j;
      g = g < r1 ? g : r1 - 1;
      const int64_t srow = GATHER ? ridx[g - r0] : g;
      // B is loaded unconditionally (a diagonal tile re-reads A's line from
      // L1): a conditional load would force register moves that wait on it
      if (VEC) {
        ra[j] = *reinterpret_cast<const f32x4*>(baseA + srow * ldx);
        rb[j] = *reinterpret_cast<const f32x4*>(baseB + srow * ldx);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ra[j][e] = X[srow * ldx + min(colA + e, p - 1)];
          rb[j][e] = X[srow * ldx + min(colB + e, p - 1)];
        }
      }
    }
  };
  auto sstore = [&](int stage, int buf) {
#pragma unroll
    for (int j = 0; j < LPP; ++j) {
      const int64_t g = r0 + (int64_t)stage * BK + rr + RSTEP * j;
      const bool rv = g < r1;
      f32x4 va, vb;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        va[e] = (rv && colA + e < p) ? ra[j][e] - shA[e] : 0.f;
        vb[e] = (rv && colB + e < p) ? rb[j][e] - shB[e] : 0.f;
      }
      *reinterpret_cast<f32x4*>(&lds[buf][0][rr + RSTEP * j][4 * c4]) = va;
      if (!diag) *reinterpret_cast<f32x4*>(&lds[buf][1][rr + RSTEP * j][4 * c4]) = vb;
      if (diag) {
#pragma unroll
        for (int e = 0; e < 4; ++e) csum64[e] += (double)va[e];
      }
    }
  };
  (void)inB;

  f32x16 acc[MT][2];
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  if (nstage > 0) {
    gload(0);
    sstore(0, 0);
  }
  __syncthreads();
  const int bsel = diag ? 0 : 1;
  // In a diagonal tile, waves whose whole sub-block lies strictly below the
  // diagonal (row start ≥ col end) only help stage data: G is symmetric and
  // the reduce kernel mirrors the upper half.
  const bool idle = diag && (wm * (GT / 2) >= (wn + 1) * 64);
  int cur = 0;
  for (int stg = 0; stg < nstage; ++stg) {
    if (stg + 1 < nstage) gload(stg + 1);
    const float* As = &lds[cur][0][0][0];
    const float* Bs = &lds[cur][bsel][0][0];
#pragma unroll
    for (int kk = 0; kk < BK / 2; ++kk) {
      if (idle) break;
      const int krow = (2 * kk + h) * GT;
      float av[MT], bv[2];
#pragma unroll
      for (int a = 0; a < MT; ++a) av[a] = As[krow + wm * (GT / 2) + a * 32 + l31];
#pragma unroll
      for (int c = 0; c < 2; ++c) bv[c] = Bs[krow + wn * 64 + c * 32 + l31];
#pragma unroll
      for (int a = 0; a < MT; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) acc[a][c] = __builtin_amdgcn_mfma_f32_32x32x2f32(av[a], bv[c], acc[a][c], 0, 0, 0);
    }
    if (stg + 1 < nstage) sstore(stg + 1, cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // partial tile out: [chunk][tile][GT][GT] float
  float* out = part + ((size_t)chunk * ntiles + tile) * (GT * GT);
#pragma unroll
  for (int a = 0; a < MT; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * (GT / 2) + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wn * 64 + c * 32 + l31;
        out[row * GT + col] = acc[a][c][r];
      }

  if (diag) {
    // reduce the RSTEP row groups of each column through LDS (reuse stage buffer)
    __syncthreads();
    double* red = reinterpret_cast<double*>(&lds[0][0][0][0]);  // [RSTEP][GT]
#pragma unroll
    for (int e = 0; e < 4; ++e) red[rr * GT + 4 * c4 + e] = csum64[e];
    __syncthreads();
    for (int c = tid; c < GT; c += Cfg::THREADS) {
      double v = 0.0;
#pragma unroll
      for (int g = 0; g < RSTEP; ++g) v += red[g * GT + c];
      colpart[((size_t)chunk * nt + ti) * GT + c] = v;
    }
  }
}

// ---------------------------------------------------------------------------
// bf16×3 split Gram on bf16 MFMA (v_mfma_f32_32x32x16_bf16, 16× the FP32-MFMA
// rate).  Every y = x − shift (f32) is split exactly into three bf16 levels
// y = y1 + y2 + y3 (each RNE; an f32 has 24 significant bits = 3 × 8, so the
// split is exact); the tile accumulates the six products with
// level(a) + level(b) ≤ 4 (y1y1, y1y2, y2y1, y1y3, y2y2, y3y1) in f32.  The
// dropped y2y3 + y3y2 + y3y3 are ≤ ~2⁻²⁴·|y_i||y_j| per term — the size of
// the f32 rounding of a single product.  The MFMA's internal sum truncates
// (below), so each K-step's six products start from a zero accumulator and
// are added to the running f32 sum by the VALU (round to nearest); 16/6 ≈
// 2.7× the FP32-MFMA peak rate remains available.
// Same work decomposition and partial layout as k_gram<256, ·> (so the same
// reduce); 16 rows per LDS stage, stored K-major per column (16 bf16 = 32 B
// per column and level) with the two 16-B halves swapped on bit 3 of the
// column: the ds_read_b128 fragment reads (lane = column, half = k-octet) and
// the ds_write_b128 stores are then bank-conflict-free.
// ---------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
constexpr int G3T = 256, G3K = 16, G3THREADS = 512;

__device__ __forceinline__ int g3_off(int panel, int lvl, int col, int half) {
  // bytes within one stage buffer: [panel][lvl][col][32 B], half swizzled
  return (((panel * 3 + lvl) * G3T + col) << 5) + ((half ^ ((col >> 3) & 1)) << 4);
}

template <bool GATHER>
__global__ __launch_bounds__(G3THREADS, 1) void k_gram3(
    const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ rows, int p, const float* __restrict__ shift,
    SegTable st, int nt, int ntiles, int total_wg, float* __restrict__ part, double* __restrict__ colpart) {
  constexpr int STAGE_BYTES = 2 * 3 * G3T * 32;  // 48 KiB per stage (both panels)
  __shared__ __attribute__((aligned(16))) char lds[2 * STAGE_BYTES];
  __shared__ int64_t ridx[GATHER ? GATHER_MAX_CHUNK : 1];
  __shared__ double cred[G3T];

  const int b = blockIdx.x;
  const int q8 = total_wg / 8, r8 = total_wg % 8, x8 = b % 8;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int chunk = wg / ntiles;
  const int tile = wg - chunk * ntiles;
  int ti, tj;
  tile_coords(tile, nt, ti, tj);
  const bool diag = (ti == tj);
  const int I = ti * G3T, J = tj * G3T;

  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  const int nstage = (int)((r1 - r0 + G3K - 1) / G3K);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 2, wn = wave & 3;  // 2 (M, 128 rows each) × 4 (N, 64 cols each)
  if (GATHER) {
    for (int64_t g = r0 + tid; g < r1; g += G3THREADS) ridx[g - r0] = rows[g];
    __syncthreads();
  }
  // loader: one column, 8 consecutive rows (one k-octet) per thread and panel
  const int lc = tid & (G3T - 1), lh = tid >> 8;
  const int colA = I + lc, colB = J + lc;
  const bool inA = colA < p, inB = colB < p;
  const float* baseA = X + (inA ? colA : p - 1);
  const float* baseB = X + (inB ? colB : p - 1);
  const float shA = inA ? shift[colA] : 0.f, shB = inB ? shift[colB] : 0.f;
  float ra[8], rb[8];
  double csum = 0.0;

  auto gload = [&](int stage) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      int64_t g = r0 + (int64_t)stage * G3K + 8 * lh + j;
      g = g < r1 ? g : r1 - 1;
      const int64_t srow = GATHER ? ridx[g - r0] : g;
      ra[j] = baseA[srow * ldx];
      rb[j] = baseB[srow * ldx];
    }
  };
  auto split_store = [&](const float (&v)[8], float sh, bool incol, int64_t g0, int panel, char* buf, bool acc_cs) {
    bf16x8 l1, l2, l3;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float y = (incol && g0 + j < r1) ? v[j] - sh : 0.f;
      if (acc_cs) csum += (double)y;
      const __bf16 b1 = (__bf16)y;
      const float e1 = y - (float)b1;
      const __bf16 b2 = (__bf16)e1;
      const float e2 = e1 - (float)b2;
      l1[j] = b1;
      l2[j] = b2;
      l3[j] = (__bf16)e2;
    }
    *reinterpret_cast<bf16x8*>(buf + g3_off(panel, 0, lc, lh)) = l1;
    *reinterpret_cast<bf16x8*>(buf + g3_off(panel, 1, lc, lh)) = l2;
    *reinterpret_cast<bf16x8*>(buf + g3_off(panel, 2, lc, lh)) = l3;
  };
  auto sstore = [&](int stage, int bi) {
    char* buf = lds + bi * STAGE_BYTES;
    const int64_t g0 = r0 + (int64_t)stage * G3K + 8 * lh;
    split_store(ra, shA, inA, g0, 0, buf, diag);
    if (!diag) split_store(rb, shB, inB, g0, 1, buf, false);
  };

  f32x16 acc[4][2];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;

  if (nstage > 0) {
    gload(0);
    sstore(0, 0);
  }
  __syncthreads();
  const int bpanel = diag ? 0 : 1;
  const bool idle = diag && (wm * 128 >= (wn + 1) * 64);
  const int l31 = lane & 31, h = lane >> 5;
  int cur = 0;
  for (int stg = 0; stg < nstage; ++stg) {
    if (stg + 1 < nstage) gload(stg + 1);
    if (!idle) {
      const char* buf = lds + cur * STAGE_BYTES;
      bf16x8 bv[2][3];
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int l = 0; l < 3; ++l)
          bv[c][l] = *reinterpret_cast<const bf16x8*>(buf + g3_off(bpanel, l, wn * 64 + c * 32 + l31, h));
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        bf16x8 av[3];
#pragma unroll
        for (int l = 0; l < 3; ++l)
          av[l] = *reinterpret_cast<const bf16x8*>(buf + g3_off(0, l, wm * 128 + a * 32 + l31, h));
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          // fresh accumulator per K-step: the bf16 MFMA aligns its 16 products
          // and C to the largest operand and truncates below its window (no
          // sticky bit: 1 − 1 + 2⁻³⁰ → 0, scripts/mfma_rounding2.hip), so a
          // long chain into the running sum would collect a one-sided error
          // per MFMA; the K-step result joins the f32 sum with an RNE add.
          f32x16 t = {};
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[2], bv[c][0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[c][1], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[c][2], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[1], bv[c][0], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[c][1], t, 0, 0, 0);
          t = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[0], bv[c][0], t, 0, 0, 0);
          // packed f32 adds: the compiler inserts the MFMA→VALU wait states
          // (an inline-asm v_add_f32 reading t without them reads stale
          // accumulators — measured: Gram error 0.8)
          acc[a][c] += t;
        }
      }
    }
    if (stg + 1 < nstage) sstore(stg + 1, cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  float* out = part + ((size_t)chunk * ntiles + tile) * (G3T * G3T);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 128 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wn * 64 + c * 32 + l31;
        out[row * G3T + col] = acc[a][c][r];
      }
  if (diag) {
    if (lh == 1) cred[lc] = csum;
    __syncthreads();
    if (lh == 0) colpart[((size_t)chunk * nt + ti) * G3T + lc] = csum + cred[lc];
  }
}

// Sum chunk partials of one segment into G (full symmetric) and colsum.
// Each thread owns 4 consecutive tile elements (one float4 per chunk) and
// keeps 4 chunks' loads in flight (independent partial sums, fixed order).
template <int GT>
__global__ __launch_bounds__(256) void k_gram_reduce(const float* __restrict__ part,
                                                     const double* __restrict__ colpart, int nt, int ntiles, int p,
                                                     int c0, int c1, double* __restrict__ G,
                                                     double* __restrict__ colsum, int cmul = 1) {
  const int tile = blockIdx.y;
  const int e4 = blockIdx.x * blockDim.x + threadIdx.x;  // float4 index in tile
  int ti, tj;
  tile_coords(tile, nt, ti, tj);
  if (e4 < GT * GT / 4) {
    const size_t stride = (size_t)ntiles * (GT * GT) / 4;
    const f32x4* src = reinterpret_cast<const f32x4*>(part) + (size_t)tile * (GT * GT) / 4 + e4;
    double s[4][4] = {};
    int c = c0;
    for (; c + 4 <= c1; c += 4) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src[(size_t)(c + u) * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) s[u][q] += (double)v[u][q];
    }
    for (; c < c1; ++c) {
      const f32x4 v = src[(size_t)c * stride];
#pragma unroll
      for (int q = 0; q < 4; ++q) s[0][q] += (double)v[q];
    }
    const int e = 4 * e4;
    const int i = e / GT, j0 = e % GT;
    const int gi = ti * GT + i;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + q, gj = tj * GT + j;
      // diagonal tiles: only the upper triangle is valid (k_gram skips the
      // strictly-lower wave blocks); mirror it
      if (gi < p && gj < p && !(ti == tj && i > j)) {
        const double v = (s[0][q] + s[1][q]) + (s[2][q] + s[3][q]);
        G[(size_t)gi * p + gj] = v;
        if (gi != gj) G[(size_t)gj * p + gi] = v;  // (column-strided; skipping them measured no change, round 5)
      }
    }
  }
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (ti == tj && e < GT && cmul > 0) {
    const int gi = ti * GT + e;
    double v = 0.0;
    // colpart rows: cmul per chunk (the i8 quantiser writes one per scale block)
    for (int c = c0 * cmul; c < c1 * cmul; ++c) v += colpart[((size_t)c * nt + ti) * GT + e];
    if (gi < p) colsum[gi] = v;
  }
}

// Σ_ij O_ij G_ij straight from the chunk partials of one segment (the
// eigensolver's θ3 term tr(O·O²), O symmetric, G = the Gram of rows of O):
// the chunk sums as k_gram_reduce forms them, weighted by O and by the
// tile's multiplicity (off-diagonal tiles and the strict upper triangle of
// diagonal tiles stand for their mirror too); one partial per workgroup,
// tile-major (fixed order).  Replaces the fp64 G, its reduce, the column sums
// and a separate trace pass.
template <int GT>
__global__ __launch_bounds__(256) void k_gram_trace(const float* __restrict__ part, int nt, int ntiles, int p,
                                                    int c0, int c1, const float* __restrict__ O,
                                                    double* __restrict__ tr_part) {
  const int tile = blockIdx.y;
  const int e4 = blockIdx.x * blockDim.x + threadIdx.x;  // float4 index in tile
  int ti, tj;
  tile_coords(tile, nt, ti, tj);
  double acc = 0.0;
  if (e4 < GT * GT / 4) {
    const size_t stride = (size_t)ntiles * (GT * GT) / 4;
    const f32x4* src = reinterpret_cast<const f32x4*>(part) + (size_t)tile * (GT * GT) / 4 + e4;
    double s[4][4] = {};
    int c = c0;
    for (; c + 4 <= c1; c += 4) {
      f32x4 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = src[(size_t)(c + u) * stride];
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int q = 0; q < 4; ++q) s[u][q] += (double)v[u][q];
    }
    for (; c < c1; ++c) {
      const f32x4 v = src[(size_t)c * stride];
#pragma unroll
      for (int q = 0; q < 4; ++q) s[0][q] += (double)v[q];
    }
    const int e = 4 * e4;
    const int i = e / GT, j0 = e % GT;
    const int gi = ti * GT + i;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int j = j0 + q, gj = tj * GT + j;
      if (gi < p && gj < p && !(ti == tj && i > j)) {
        const double v = (s[0][q] + s[1][q]) + (s[2][q] + s[3][q]);
        const double w = (ti == tj && i == j) ? 1.0 : 2.0;
        acc += w * v * (double)O[(size_t)gi * p + gj];
      }
    }
  }
  __shared__ double red[4];
  acc = wave_sum_f64(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) tr_part[(size_t)tile * gridDim.x + blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

// Column mean over n rows: per (column, row-split) f64 partial sums.
__global__ void k_colsum_part(const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ rows, int64_t n,
                              int p, int64_t rows_per_split, double* __restrict__ part, PrepArgs pa = PrepArgs{}) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int sp = blockIdx.y;
  if (col >= p) return;
  const int64_t a = (int64_t)sp * rows_per_split;
  const int64_t e = min(n, a + rows_per_split);
  double v = 0.0;
  int64_t r = a;
  for (; r + 8 <= e; r += 8) {  // eight loads in flight, summed in row order
    float y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) y[u] = load_y(X, ldx, rows ? rows[r + u] : r + u, col, p, pa);
#pragma unroll
    for (int u = 0; u < 8; ++u) v += (double)y[u];
  }
  for (; r < e; ++r) v += (double)load_y(X, ldx, rows ? rows[r] : r, col, p, pa);
  part[(size_t)sp * p + col] = v;
}

__global__ void k_colsum_final(const double* __restrict__ part, int nsplit, int p, double inv_n,
                               double* __restrict__ mean) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= p) return;
  double v = 0.0;
  int s = 0;
  for (; s + 8 <= nsplit; s += 8) {  // eight loads in flight, summed in split order
    double y[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) y[u] = part[(size_t)(s + u) * p + col];
#pragma unroll
    for (int u = 0; u < 8; ++u) v += y[u];
  }
  for (; s < nsplit; ++s) v += part[(size_t)s * p + col];
  mean[col] = v * inv_n;
}

constexpr int MAXTERM = 8;
struct CovTerms {
  const double* G[MAXTERM];
  const double* cs[MAXTERM];
  double coef[MAXTERM];
  int nterm;
};

// C = (Σ_t c_t G_t − n d dᵀ)/(n − 1) with d = Σ_t c_t cs_t / n (the mean's
// offset from the shift), and mean = shift + d from row 0's threads.  Each
// thread forms its d_i, d_j from the column sums itself (the same sums as the
// separate mean kernel it replaces: one launch less on the non-sharded path)
__global__ void k_cov(CovTerms tm, const float* __restrict__ shift, int p, double n, double* __restrict__ C,
                      double* __restrict__ mean) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)p * p) return;
  const int i = (int)(e / p), j = (int)(e % p);
  double si = 0.0, sj = 0.0, g = 0.0;
  for (int t = 0; t < tm.nterm; ++t) {
    si += tm.coef[t] * tm.cs[t][i];
    sj += tm.coef[t] * tm.cs[t][j];
    g += tm.coef[t] * tm.G[t][e];
  }
  const double di = si / n, dj = sj / n;
  C[e] = (g - n * di * dj) / (n - 1.0);
  if (i == 0) mean[j] = (double)shift[j] + dj;
}

// ---------------------------------------------------------------------------
// Narrow matrices (p ≤ 64: VAE latents, tiny spectra): fp64 accumulation.
// Latent covariances can be badly conditioned (the leverage / Mahalanobis
// forms square it), so the FP32-MFMA path's ~1e-7 relative Gram error is not
// acceptable there; at p ≤ 64 the fp64 VALU work (n·p²/2 FMAs) is negligible.
// One workgroup per chunk of one segment: 64-row tiles of y = x − shift (fp64)
// in LDS, each thread owns a fixed set of upper-triangle pairs.
// ---------------------------------------------------------------------------
constexpr int SMALL_P = 64, SMALL_ROWS = 64, SMALL_CHUNK = 2048;

__global__ __launch_bounds__(256) void k_gram_small(const float* __restrict__ X, int64_t ldx,
                                                    const int64_t* __restrict__ rows, int p,
                                                    const float* __restrict__ shift,
                                                    const int64_t* __restrict__ span,
                                                    double* __restrict__ part, double* __restrict__ cpart) {
  __shared__ double ys[SMALL_ROWS][SMALL_P + 1];
  __shared__ short pi[SMALL_P * (SMALL_P + 1) / 2], pj[SMALL_P * (SMALL_P + 1) / 2];
  const int tid = threadIdx.x;
  const int npair = p * (p + 1) / 2;
  if (tid == 0) {
    int e = 0;
    for (int i = 0; i < p; ++i)
      for (int j = i; j < p; ++j) {
        pi[e] = (short)i;
        pj[e] = (short)j;
        ++e;
      }
  }
  const int64_t r0 = span[2 * blockIdx.x], r1 = span[2 * blockIdx.x + 1];  // rows [r0, r1)
  constexpr int MAXPT = (SMALL_P * (SMALL_P + 1) / 2 + 255) / 256;  // pairs per thread
  double acc[MAXPT];
#pragma unroll
  for (int u = 0; u < MAXPT; ++u) acc[u] = 0.0;
  double csum = 0.0;
  for (int64_t b = r0; b < r1; b += SMALL_ROWS) {
    const int nr = (int)min<int64_t>(SMALL_ROWS, r1 - b);
    __syncthreads();
    for (int e = tid; e < SMALL_ROWS * p; e += 256) {
      const int r = e / p, c = e % p;
      double v = 0.0;
      if (r < nr) {
        const int64_t sr = rows ? rows[b + r] : b + r;
        v = (double)X[sr * ldx + c] - (double)shift[c];
      }
      ys[r][c] = v;
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < MAXPT; ++u) {
      const int e = tid + 256 * u;
      if (e < npair) {
        const int i = pi[e], j = pj[e];
        double a = acc[u];
        for (int r = 0; r < nr; ++r) a += ys[r][i] * ys[r][j];
        acc[u] = a;
      }
    }
    if (tid < p)
      for (int r = 0; r < nr; ++r) csum += ys[r][tid];
  }
#pragma unroll
  for (int u = 0; u < MAXPT; ++u) {
    const int e = tid + 256 * u;
    if (e < npair) part[(size_t)blockIdx.x * npair + e] = acc[u];
  }
  if (tid < p) cpart[(size_t)blockIdx.x * p + tid] = csum;
}

// G (full symmetric) and colsum of one segment = ordered sum of its chunks
__global__ __launch_bounds__(256) void k_gram_small_reduce(const double* __restrict__ part,
                                                           const double* __restrict__ cpart, int p, int c0, int c1,
                                                           double* __restrict__ G, double* __restrict__ colsum) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int npair = p * (p + 1) / 2;
  if (e < npair) {
    // e -> (i, j), i <= j, row-major upper triangle
    int i = 0, rem = e;
    while (rem >= p - i) {
      rem -= p - i;
      ++i;
    }
    const int j = i + rem;
    double v = 0.0;
    for (int c = c0; c < c1; ++c) v += part[(size_t)c * npair + e];
    G[(size_t)i * p + j] = v;
    G[(size_t)j * p + i] = v;
  }
  if (e < p) {
    double v = 0.0;
    for (int c = c0; c < c1; ++c) v += cpart[(size_t)c * p + e];
    colsum[e] = v;
  }
}

// ---------------------------------------------------------------------------
// i8×3 Gram (default): the Gram on integer MFMA (v_mfma_i32_32x32x32_i8, 2×
// the bf16 rate, exact int32 accumulation).
//
// k_q8_quant (one HBM read of X) writes y = x − shift as three signed int8
// digit planes per 1536-row scale block b and column j:
//     y = s_bj · (a1 + a2/254 + a3/254²),   |a·| ≤ 127,   s_bj = 2^e ≥ max|y|/127
// (s a power of two, so y/s is exact; a1 = rint(y/s), a2 = rint(254·r1), a3 =
// rint(254·r2) with |r·| ≤ ½; the residual is ≤ ½·254⁻²·s ≈ 2⁻²⁴·max|y|).
// k_gram8d accumulates, per 128×128 tile, the six digit products of weight
// ≥ 254⁻² in three int32 sets (A1 = Σa1a1', A2 = Σa1a2'+a2a1', A3 = Σa1a3'+
// a3a1'+a2a2'; per block |A1| ≤ 1536·127² ≈ 2.5e7, |A3| ≤ 3·1536·127² ≈ 7.4e7
// < 2³¹, so the int32 sums are exact) and converts each block's sets to f32
// (a rounded int32 → f32 conversion: ≤ 2⁻²⁴ relative) folded into f32 running
// sums per 4096-row chunk: G += s_i s_j (A1 + A2/254 + A3/254²); chunks are
// summed in f64.  The dropped products are ≤ 2⁻²⁴·max|y_i|·max|y_j| per row,
// the size of an f32 rounding of the largest product.
//
// Outlier guard.  The representation error is relative to the block's
// column maximum, so one extreme row would cost the other 1535 rows of its
// block their precision.  k_q8_quant therefore screens every value against a
// per-column threshold τ·2^e_j (2^e_j ≥ median|y_j| over the first ≤ 4096
// rows, a robust scale; τ = 16; k_colexp_hist / k_q8_thresholds): a row with any value above it inside the workgroup's 32
// columns is left out of those columns' scale and digits (its digits there
// are 0) and marked in a per-row column-group bitmask.  k_gram_fixup adds the
// marked rows' missing products exactly (fp64: y_i y_j for every pair with
// at least one column in a marked group).  Clean data marks nothing and pays
// one scalar read-back; heavily marked data (> n/8 rows) falls back to the
// bf16×3 Gram (exact split, fp32-grade).
//
// Digit planes: [digit][32-row group][column P8][32 B] (the 32 B of a column
// are its 32 rows of one group — one MFMA K-step).  The digit planes are in
// processed-row order, so class subsets / CV folds (gather lists) are
// gathered once, by the quantiser.
// ---------------------------------------------------------------------------
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
constexpr int Q8T = 128, Q8K = 32, Q8BLK = 1536, Q8SPB = Q8BLK / Q8K;
constexpr float Q8BASE = 254.f;

struct Q8Plan {
  char* digits;   // 3 planes
  size_t plane;   // bytes per plane
  float* scale;   // [chunk][nblk][P8]
  int P8;         // padded columns (multiple of Q8T)
  int nblk;       // scale blocks per chunk
  const float* thr;  // [P8] outlier thresholds (τ × robust column scale)
  uint32_t* flags;   // [processed row][fw] column-group bitmask of screened-out values
  int fw;            // bitmask words per row
  uint32_t* nmark;   // number of (row, column group) marks
};

constexpr float Q8TAU = 16.f;     // outlier threshold in robust column scales (2^e ≥ median|y|)
constexpr int Q8GROUP = 32;       // columns per guard group (= quantiser workgroup width)

__device__ __forceinline__ uint32_t q8_byte(float a, int u) { return ((uint32_t)(int)a & 0xffu) << (8 * u); }

__device__ __forceinline__ uint32_t q8_pack4(float a0, float a1, float a2, float a3) {
  // low bytes of the four digits (two's complement int8) into one dword
  const uint32_t lo = __builtin_amdgcn_perm((uint32_t)(int)a1, (uint32_t)(int)a0, 0x0c0c0400u);
  const uint32_t hi = __builtin_amdgcn_perm((uint32_t)(int)a3, (uint32_t)(int)a2, 0x04000c0cu);
  return lo | hi;
}

// 16-B slot of piece P = 2·column + half in a group's staging image (32
// columns = 64 pieces): bits 0-2 are XORed with bits 3-5 (an involution).
// The writes (8 consecutive lanes: column quads 0..7 of one row slice, i.e.
// pieces 8cq + const) and the linear copy-out reads then hit 8 distinct 16-B
// bank groups per ds_write_b128 / ds_read_b128 lane group.
__device__ __forceinline__ int q8_qslot(int P) { return P ^ ((P >> 3) & 7); }

// grid (chunk · nblk + block, P8 / 32), 768 threads (12 waves): one 1536-row
// scale block × 32 columns.  Thread t owns column quad cq = t & 7 (columns
// 4cq .. 4cq+3: a wave instruction reads 8 rows × 128 B) and row slice
// rs = t >> 3 (rows 16rs .. 16rs+15 = half rs&1 of 32-row group rs>>1), so
// each (column, digit) of a thread is one 16-B piece of the digit image.  The
// pieces are staged through LDS (one digit plane, 24 KiB, at a time) so that
// the stores leave as contiguous 1-KiB runs (one 32-row group × 32 columns).
constexpr int Q8QC = 32;                   // columns per quantiser workgroup
constexpr int Q8QS = Q8BLK / 16;           // 16-row slices per block (96)
constexpr int Q8QT = Q8QS * (Q8QC / 4);    // threads (768)
// The quantiser after the load: v = this thread's 16 rows × 4 columns of
// y − shift.  Column sums, the outlier screen, the block scale, the digits
// and their LDS-staged stores (shared by k_q8_quant and k_q8_quant_prep).
// q8_tail's LDS (the caller declares it: k_q8_quant_prep overlays its own
// load-phase buffers on it)
// digit planes staged in LDS at once: 3 (one barrier, 147 KiB with the
// reduction buffers overlaid — the quantiser is one workgroup per CU by its
// registers anyway) or 1 (a barrier pair per plane); 3.02 vs 3.04 and 2.62 vs
// 2.69 ms on two boxes, identical digits (profiles/r05zc_quant_stage_ab.json)
#ifdef OCM_Q8_STAGE1
constexpr int Q8NST = 1;
#else
constexpr int Q8NST = 3;
#endif
template <int QC = Q8QC>
struct Q8TailLdsT {
  union {  // the reduction buffers are dead once the block scales are known
    struct {
      __attribute__((aligned(16))) float wmax[Q8QS][QC];
      __attribute__((aligned(16))) double wsum[Q8QS][QC];
      float pmax[8][QC];
      double psum[8][QC];
    } r;
    __attribute__((aligned(16))) char stage[Q8NST * Q8SPB * QC * 32];  // digit planes: 48 KiB each at QC = 32
  } u;
  __attribute__((aligned(16))) float fmax_[QC];
};
using Q8TailLds = Q8TailLdsT<>;
template <int QC = Q8QC>
// th: the thresholds of the thread's four columns, loaded by the caller in
// its load phase (a global load here would wait, through vmcnt, for every
// store the caller has issued — the write-through X′ rows)
__device__ __forceinline__ void q8_tail(f32x4 (&v)[16], int tid, int cq, int rs, int cg0, int c0, int64_t rb,
                                        const Q8Plan& q, int chunk, int b, const SegTable& st,
                                        double* __restrict__ colblk, Q8TailLdsT<QC>& L, const f32x4 th) {
  constexpr int NT = Q8QS * (QC / 4);  // threads
  char* stage = L.u.stage;
  auto& wmax = L.u.r.wmax;
  auto& wsum = L.u.r.wsum;
  auto& pmax = L.u.r.pmax;
  auto& psum = L.u.r.psum;
  float* fmax_ = L.fmax_;
#ifdef OCM_Q8_DIAG_COPY
  // timing diagnostic (make exp only; wrong results): no column sums, screen,
  // scales or digits — the loads, the LDS staging and the digit-plane stores,
  // i.e. the quantiser's traffic pattern alone
  (void)wsum; (void)wmax; (void)pmax; (void)psum; (void)fmax_; (void)th; (void)colblk; (void)c0;
  i32x4 w[3][4];
#pragma unroll
  for (int dg = 0; dg < 3; ++dg)
#pragma unroll
    for (int e = 0; e < 4; ++e)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        w[dg][e][k] = (int)(__builtin_bit_cast(uint32_t, v[4 * k][e]) ^ __builtin_bit_cast(uint32_t, v[4 * k + 1][e]) ^
                            __builtin_bit_cast(uint32_t, v[4 * k + 2][e]) ^ __builtin_bit_cast(uint32_t, v[4 * k + 3][e])) + dg;
#else
  // column sums over every row (the fix-up does not touch them)
  double cs[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int j = 0; j < 16; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) cs[e] += (double)v[j][e];
  // outlier screen: rows with a value above the threshold in this column group are
  // taken out of its scale and digits (k_gram_fixup adds them exactly)
  {
    uint32_t ext = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) ext |= (fabsf(v[j][e]) > th[e]) ? (1u << j) : 0u;
    // OR over the QC / 4 threads (consecutive lanes) that share this row slice
#pragma unroll
    for (int o = 1; o < QC / 4; o *= 2) ext |= __shfl_xor(ext, o, 64);
    if (ext) {
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((ext >> j) & 1u) v[j] = f32x4{0.f, 0.f, 0.f, 0.f};
      if (cq == 0) {
        const int grp = cg0 / Q8GROUP;
        for (int j = 0; j < 16; ++j)
          if ((ext >> j) & 1u) atomicOr(q.flags + (size_t)(rb + j) * q.fw + (grp >> 5), 1u << (grp & 31));
        atomicAdd(q.nmark, (uint32_t)__popc(ext));
      }
    }
  }
  f32x4 m = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 16; ++j)
#pragma unroll
    for (int e = 0; e < 4; ++e) m[e] = fmaxf(m[e], fabsf(v[j][e]));
  *reinterpret_cast<f32x4*>(&wmax[rs][4 * cq]) = m;
#pragma unroll
  for (int e = 0; e < 4; ++e) wsum[rs][4 * cq + e] = cs[e];
  __syncthreads();
  // two-level column reduction over the 48 slices (fixed order)
  if (tid < 8 * QC) {
    const int col = tid & (QC - 1), part = tid / QC;
    float mm = 0.f;
    double ss = 0.0;
    for (int w = part * (Q8QS / 8); w < (part + 1) * (Q8QS / 8); ++w) {
      mm = fmaxf(mm, wmax[w][col]);
      ss += wsum[w][col];
    }
    pmax[part][col] = mm;
    psum[part][col] = ss;
  }
  __syncthreads();
  if (tid < QC) {
    float mm = 0.f;
    double ss = 0.0;
#pragma unroll
    for (int w = 0; w < 8; ++w) {
      mm = fmaxf(mm, pmax[w][tid]);
      ss += psum[w][tid];
    }
    fmax_[tid] = mm;
    int ex = 0;
    (void)frexpf(mm * (1.f / 127.f), &ex);
    const size_t o = ((size_t)chunk * q.nblk + b) * q.P8 + cg0 + tid;
    q.scale[o] = mm > 0.f ? ldexpf(1.f, ex) : 1.f;
    colblk[o] = ss;
  }
  __syncthreads();
  const f32x4 mx = *reinterpret_cast<const f32x4*>(&fmax_[4 * cq]);
  i32x4 w[3][4];  // [digit][column e]
  f32x4 inv;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    int ex = 0;
    (void)frexpf(mx[e] * (1.f / 127.f), &ex);
    inv[e] = mx[e] > 0.f ? ldexpf(1.f, -ex) : 1.f;
  }
  // row quads outermost: v[4k .. 4k+3] are dead after quad k, so the digits
  // take the registers the values free (peak ≈ 64 + 12, not 64 + 48: no spills
  // at the 168-VGPR budget of three waves per SIMD).
  // Digits by the round-to-nearest-even of an add of 1.5·2²³ (round 5): for
  // |x| < 2²² the f32 sum x + 1.5·2²³ is 0x4B400000 + rint(x), so its low byte
  // IS the int8 digit (no v_rndne / v_cvt_i32) and subtracting 1.5·2²³ back
  // gives rint(x) exactly; in pairs of rows on packed f32 (v_pk_add / v_pk_mul):
  // the same digits as rintf, bit for bit (the Gram of the bench workload
  // hashes identically with either split: profiles/r05h_quant_ab.json; the
  // quantiser is HBM-bound, 3.03 vs 3.05 ms).  No implicit FMA contraction
  // (t2 is rounded before the add that rounds it to an integer, as rintf(t2)
  // saw it); the third digit's remainder is the one explicit FMA,
  // (t − a1)·254 − a2 with the exact product, as the contracted rintf form
  // computed it.
  {
#pragma clang fp contract(off)
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const f32x2 MG = {12582912.f, 12582912.f}, BASE = {Q8BASE, Q8BASE};
    auto bits = [](float f) { return __builtin_bit_cast(uint32_t, f); };
    auto pack = [&](f32x2 lo, f32x2 hi) -> int {  // low bytes of four sums → one dword (rows u = 0..3)
      const uint32_t l = __builtin_amdgcn_perm(bits(lo.y), bits(lo.x), 0x0c0c0400u);
      const uint32_t h = __builtin_amdgcn_perm(bits(hi.y), bits(hi.x), 0x04000c0cu);
      return (int)(l | h);
    };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const f32x2 ie = {inv[e], inv[e]};
        f32x2 A[2], B[2], Cd[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const f32x2 t = f32x2{v[4 * k + 2 * h][e], v[4 * k + 2 * h + 1][e]} * ie;  // exact, |t| ≤ 127
          A[h] = t + MG;
          const f32x2 d = t - (A[h] - MG);  // exact
          const f32x2 t2 = d * BASE;
          B[h] = t2 + MG;
          Cd[h] = __builtin_elementwise_fma(d, BASE, MG - B[h]) * BASE + MG;  // MG − B = −a2 exactly
        }
        w[0][e][k] = pack(A[0], A[1]);
        w[1][e][k] = pack(B[0], B[1]);
        w[2][e][k] = pack(Cd[0], Cd[1]);
      }
    }
  }
#endif  // OCM_Q8_DIAG_COPY
  // stage image: [group][column 0..31][32 B]; copy-out: 16 B per thread and
  // pass, 1 KiB contiguous per wave instruction (= one group)
  constexpr int GIMG = QC * 32;  // bytes per group image
  char* gdst = q.digits + ((size_t)chunk * (st.chunk_rows / Q8K) + (size_t)b * Q8SPB) * q.P8 * 32 + (size_t)cg0 * 32;
  const int grp = rs >> 1, half = rs & 1;
  if constexpr (Q8NST == 3) {
#pragma unroll
    for (int dg = 0; dg < 3; ++dg)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        *reinterpret_cast<i32x4*>(&stage[dg * Q8SPB * GIMG + grp * GIMG + q8_qslot(2 * (4 * cq + e) + half) * 16]) =
            w[dg][e];
    __syncthreads();
#pragma unroll
    for (int dg = 0; dg < 3; ++dg)
#pragma unroll
      for (int k = 0; k < Q8SPB * GIMG / (16 * NT); ++k) {
        const int o = 16 * (tid + NT * k);
        const int g = o / GIMG, within = o - g * GIMG;
        *reinterpret_cast<i32x4*>(gdst + (size_t)dg * q.plane + (size_t)g * q.P8 * 32 + within) =
            *reinterpret_cast<const i32x4*>(&stage[dg * Q8SPB * GIMG + g * GIMG + q8_qslot(within >> 4) * 16]);
      }
    return;
  }
#pragma unroll
  for (int dg = 0; dg < 3; ++dg) {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      *reinterpret_cast<i32x4*>(&stage[grp * GIMG + q8_qslot(2 * (4 * cq + e) + half) * 16]) = w[dg][e];
    __syncthreads();
    static_assert(Q8SPB * GIMG % (16 * NT) == 0, "copy-out passes");
#pragma unroll
    for (int k = 0; k < Q8SPB * GIMG / (16 * NT); ++k) {
      const int o = 16 * (tid + NT * k);  // byte offset in the stage image
      const int g = o / GIMG, within = o - g * GIMG;
      *reinterpret_cast<i32x4*>(gdst + (size_t)dg * q.plane + (size_t)g * q.P8 * 32 + within) =
          *reinterpret_cast<const i32x4*>(&stage[g * GIMG + q8_qslot(within >> 4) * 16]);
    }
    __syncthreads();
  }
}

// QC: columns per workgroup.  16-column workgroups (384 threads, two per CU)
// measured 4.25 against 3.02 ms for the default at 1M × 2048: rows read as
// 16 × 64 B per wave instruction lose more than the second workgroup per CU
// gains (profiles/r05j_quant_qc16_ab.json)
template <bool GATHER, int CG = 1, int QC = Q8QC>
__global__ __launch_bounds__(Q8QS * (QC / 4), 1) void k_q8_quant(const float* __restrict__ X, int64_t ldx,
                                                                 const int64_t* __restrict__ rows, int p,
                                                                 const float* __restrict__ shift, SegTable st,
                                                                 Q8Plan q, double* __restrict__ colblk, int cb0) {
  // CG > 1 (A/B): CG neighbouring 32-column groups of one row block on
  // consecutive workgroups (they run at the same time on other CUs), so each
  // row's CG·128 bytes are read close in time
  const int gbk = (int)(blockIdx.x / CG) + cb0;  // (chunk, block) of the call's chunk range
  const int chunk = gbk / q.nblk, b = gbk - chunk * q.nblk;
  const int tid = threadIdx.x;
  const int cq = tid % (QC / 4), rs = tid / (QC / 4);
  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  // blocks past the chunk's rows are written too (zero digits, scale 1): the
  // Gram kernels read whole blocks
  const int64_t rb = r0 + (int64_t)b * Q8BLK + 16 * rs;
  const int cg0 = (int)(blockIdx.y * CG + blockIdx.x % CG) * QC;  // first column of the workgroup
  const int c0 = cg0 + 4 * cq;                                    // first of this thread's 4 columns
  const bool vec = (ldx % 4 == 0) && (c0 + 3 < p) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  f32x4 sh;  // shift == nullptr: a zero shift (internal Grams)
#pragma unroll
  for (int e = 0; e < 4; ++e) sh[e] = (shift && c0 + e < p) ? shift[c0 + e] : 0.f;
  f32x4 v[16];
  const int64_t rblk = r0 + (int64_t)b * Q8BLK;  // first row of the block
  if (!GATHER && vec && (int64_t)Q8BLK * ldx * 4 < (1LL << 31)) {
    // contiguous rows: one buffer descriptor over the block's valid rows (one
    // address VGPR instead of 16 64-bit row pointers).  The whole byte offset,
    // row step included, goes in the VECTOR offset: only voffset is checked
    // against the descriptor's size (the scalar offset is not), so rows past
    // r1 — a block whose valid row count is not a multiple of 16 — read as 0
    // instead of touching memory past the end of X.
    const int64_t nvalid = max((int64_t)0, min(r1 - rblk, (int64_t)Q8BLK));
    const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(
        (void*)(X + rblk * ldx), 0, (uint32_t)(nvalid * ldx * 4), 0x00020000);
    const int voff = (int)((16 * rs * ldx + c0) * 4);
    const int rstep = (int)(ldx * 4);
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const f32x4 x = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_x, voff + j * rstep, 0, 0));
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = (rb + j < r1) ? x[e] - sh[e] : 0.f;
    }
  } else {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t g = rb + j;
      const int64_t gc = g < r1 ? g : r1 - 1;  // clamped: always a valid row
      const float* xr = X + (GATHER ? rows[gc] : gc) * ldx;
      f32x4 x;
      if (vec) {
        x = *reinterpret_cast<const f32x4*>(xr + c0);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e) x[e] = xr[min(c0 + e, p - 1)];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[j][e] = (g < r1 && c0 + e < p) ? x[e] - sh[e] : 0.f;
    }
  }
  __shared__ Q8TailLdsT<QC> lds;
  const float inf = __builtin_inff();  // q.thr == nullptr: no screen (internal Grams)
  q8_tail<QC>(v, tid, cq, rs, cg0, c0, rb, q, chunk, b, st, colblk, lds,
              q.thr ? *reinterpret_cast<const f32x4*>(q.thr + c0) : f32x4{inf, inf, inf, inf});
}

// k_q8_quant with the preprocessing of a lazy view applied in the load path
// (include/ocm.h ocm_prep; the fused forms of PrepArgs::fused_form, HH =
// window / 2 ∈ {0, 2, 7}).  Load phase, before any compute (k_q8_quant's
// memory-level parallelism): each lane's raw quad of its 16 rows, the rows'
// SNV (s_r, m_r) and — HH > 0 — the halo of two of its slice's rows (lane cq:
// rows cq and cq + 8, the HQ = ⌈HH/4⌉ quads left and right of the workgroup's
// 32 columns), which go to an LDS halo table as soon as they land: the row
// loop holds only the 16 output quads.  Per row, the eight lanes of a row
// slice put their quads in a wave-private LDS row image and read their
// (4 + 2·4HQ)-column window back from the image or the halo table; the row
// ends use the least-squares edge rows.  The load phase's LDS overlays
// q8_tail's.
#ifdef OCM_QP_DPP
// the quad of the lane CTRL's DPP row shift names (row_shr / row_shl inside 16 lanes)
// (old = 0, not the source: with old == src hipcc (ROCm 7.2) folded the four
// components' DPP moves into one and copied its result to all four)
template <int CTRL>
__device__ __forceinline__ float q8_dpp1(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int CTRL>
__device__ __forceinline__ f32x4 q8_dpp4(f32x4 x) {
  return f32x4{q8_dpp1<CTRL>(x.x), q8_dpp1<CTRL>(x.y), q8_dpp1<CTRL>(x.z), q8_dpp1<CTRL>(x.w)};
}
#endif
template <int HH>
struct Q8PrepLds {
  static constexpr int HQ = (HH + 3) / 4, WN = 2 * HH + 1;
  __attribute__((aligned(16))) float img[Q8QS][Q8QC];                 // one row image per row slice
  __attribute__((aligned(16))) f32x4 halo[HQ > 0 ? Q8QS * 16 * 2 * HQ : 1];  // [slice][row][side][quad]
  float etap[HH > 0 ? 2 * HH * WN : 1];                                // the edge rows
};
template <int HH>
union Q8PrepUnion {
  Q8TailLds tail;
  Q8PrepLds<HH> ld;
};
// WR (write-through, round 5): the preprocessed rows also go to xout (ldo),
// so the consumers after the Gram read X′ plainly and the stencil runs once
// (ocm_gram_f32_prep_write; contiguous rows only)
template <bool GATHER, int HH, bool WR = false>
__global__ __launch_bounds__(Q8QT, 1) void k_q8_quant_prep(const float* __restrict__ X, int64_t ldx,
                                                           const int64_t* __restrict__ rows, int p,
                                                           const float* __restrict__ shift, SegTable st, Q8Plan q,
                                                           double* __restrict__ colblk, int cb0, int ncg,
                                                           PrepArgs pa, float* __restrict__ xout, int64_t ldo) {
  static_assert(!(WR && GATHER), "write-through takes contiguous rows");
  constexpr int HQ = (HH + 3) / 4;
  constexpr int WN = 2 * HH + 1;
  __shared__ Q8PrepUnion<HH> lds;
  auto& L = lds.ld;
  // workgroup → (row block, column group), XCD-aware: a group's halo columns
  // belong to its neighbours, so the neighbours must read those lines close in
  // time on one XCD (its L2).  Workgroup i runs on XCD i mod 8: XCD x takes
  // the row blocks ≡ x (mod 8) and sweeps each one's column groups in order,
  // ≈ 32 neighbours in flight.  In the plain order (row blocks fastest) every
  // halo line came from HBM again: 25 GB fetched per launch for 8.2 GB of X
  // (profiles/r04x_pmc.json)
  const int nbk = (int)gridDim.x / ncg;
  int bki, cgi;
  {
    const int id = (int)blockIdx.x;
    const int nb8 = nbk & ~7, head = nb8 * ncg;  // row blocks in whole groups of eight
    if (id < head) {
      const int x = id & 7, kk = id >> 3;
      const int sweep = kk / ncg;  // this XCD's sweep-th row block
      bki = 8 * sweep + x;
      cgi = kk - sweep * ncg;
    } else {  // the last nbk mod 8 row blocks: row blocks fastest
      const int r = id - head, nt = nbk - nb8;
      bki = nb8 + r % nt;
      cgi = r / nt;
    }
  }
  const int gbk = bki + cb0;
  const int chunk = gbk / q.nblk, b = gbk - chunk * q.nblk;
  const int tid = threadIdx.x;
  const int cq = tid & 7, rs = tid >> 3;
  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  const int64_t rb = r0 + (int64_t)b * Q8BLK + 16 * rs;
  const int cg0 = cgi * Q8QC;
  const int c0 = cg0 + 4 * cq;
  f32x4 sh;
#pragma unroll
  for (int e = 0; e < 4; ++e) sh[e] = c0 + e < p ? shift[c0 + e] : 0.f;
#ifdef OCM_QP_NOSTENCIL
  const f32x4 th = {__builtin_inff(), __builtin_inff(), __builtin_inff(), __builtin_inff()};
#else
  const f32x4 th = *reinterpret_cast<const f32x4*>(q.thr + c0);
#endif
  const float* c = pa.taps + HH;  // interior taps, offset -HH..HH (scalar loads)
  float ct[HH + 1];
#pragma unroll
  for (int t = 0; t <= HH; ++t) ct[t] = HH > 0 ? c[t] : 0.f;
  const bool edge_wg = HH > 0 && (cg0 < HH || cg0 + Q8QC > p - HH);
  if (edge_wg)
    for (int i = tid; i < 2 * HH * WN; i += Q8QT) L.etap[i] = pa.taps[WN + i];
  // ---- load phase.  Addresses are clamped into the row (p % 4 = 0 here):
  // quads past p are never read back, halo quads outside the row are zeroed.
  constexpr bool sub = HH == 0;  // SNV alone subtracts the row mean
  f32x4 v[16];
  float srl[2], mrl[2];  // the SNV (s_r, m_r) of rows 2cq, 2cq + 1 (row j's come from lane j / 2 of the slice)
  const int cl0 = min(c0, p - 4);
  // contiguous rows: one buffer descriptor over the block's valid rows and
  // 32-bit row offsets (16 row pointers of 64 bits spilled registers);
  // rows past r1 read as 0 (their outputs are dropped below)
  const int64_t rblk = r0 + (int64_t)b * Q8BLK;
  constexpr bool bufd = !GATHER;  // prep_fused_gram: Q8BLK·ldx·4 < 2³¹
  const int64_t nvalid = max((int64_t)0, min(r1 - rblk, (int64_t)Q8BLK));
  const __amdgpu_buffer_rsrc_t rs_x = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(X + (bufd ? rblk * ldx : 0)), 0, bufd ? (uint32_t)(nvalid * ldx * 4) : 0u, 0x00020000);
  const __amdgpu_buffer_rsrc_t rs_o = __builtin_amdgcn_make_buffer_rsrc(
      (void*)(WR ? xout + rblk * ldo : nullptr), 0, WR ? (uint32_t)(nvalid * ldo * 4) : 0u, 0x00020000);
  auto load_q = [&](int jr, int col) -> f32x4 {  // the quad at column col of slice row jr
    if constexpr (bufd)
      return __builtin_bit_cast(
          f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs_x, (int)(((16 * rs + jr) * ldx + col) * 4), 0, 0));
    const int64_t g = rb + jr;
    const int64_t gc = g < r1 ? g : r1 - 1;  // clamped: always a valid row
    return *reinterpret_cast<const f32x4*>(X + (GATHER ? rows[gc] : gc) * ldx + col);
  };
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = load_q(j, cl0);
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int64_t g = rb + 2 * cq + u;
    const int64_t gc = g < r1 ? g : r1 - 1;
    const int64_t xi = GATHER ? rows[gc] : gc;
    srl[u] = pa.snv ? pa.rowstat[2 * xi + 1] : 1.f;
    mrl[u] = sub ? pa.rowstat[2 * xi] : 0.f;
  }
  if constexpr (HQ > 0) {
    f32x4 hq[2][2][HQ];  // [row cq, cq + 8][left / right][quad]
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int side = 0; side < 2; ++side)
#pragma unroll
        for (int i = 0; i < HQ; ++i) {
          const int col = side == 0 ? cg0 - 4 * HQ + 4 * i : cg0 + Q8QC + 4 * i;
          const f32x4 t4 = load_q(cq + 8 * u, min(max(col, 0), p - 4));
          hq[u][side][i] = col >= 0 && col < p ? t4 : f32x4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int side = 0; side < 2; ++side)
#pragma unroll
        for (int i = 0; i < HQ; ++i) L.halo[((rs * 16 + cq + 8 * u) * 2 + side) * HQ + i] = hq[u][side][i];
  }
  if (edge_wg) __syncthreads();  // etap (the halo table and the row images are wave-private)
  float* row_img = L.img[rs];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const int64_t g = rb + j;
    f32x4 xs = v[j];
    if constexpr (sub) {
      const float mrj = __shfl(mrl[j & 1], j >> 1, 8);
#pragma unroll
      for (int e = 0; e < 4; ++e) xs[e] = __fsub_rn(xs[e], mrj);
    }
    const float srj = __shfl(srl[j & 1], j >> 1, 8);
    const f32x4* hrow = L.halo + (rs * 16 + j) * 2 * HQ;  // this row's halo: [side][quad]
    float win[4 + 2 * 4 * HQ];  // columns c0 − 4HQ .. c0 + 3 + 4HQ
#ifdef OCM_QP_DPP
    // (make exp A/B; measured: the same digits and X′ bit for
    // bit, and no faster — cheese write-through quantiser 5.95–5.98 against
    // 5.86–5.95 ms, profiles/r06k_qp_dpp_ab.txt: the LDS row image is not what
    // holds the fused quantiser back; its VALU work (3310 instructions, the
    // taps already on packed f32) and the extra X′ write stream are)
    // the neighbouring quads of the slice by DPP lane shifts
    // (row_shr / row_shl by s lanes inside the 16-lane DPP row: lanes whose
    // source falls outside their own eight-lane slice take the halo instead),
    // the out-of-slice quads from the halo table, which the load phase filled:
    // nothing waits on this row's own LDS store; the row image only where the
    // grid's edge workgroups read it (the least-squares edge rows)
    if (edge_wg) *reinterpret_cast<f32x4*>(row_img + 4 * cq) = xs;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int e = 0; e < 4; ++e) win[4 * HQ + e] = xs[e];
#pragma unroll
    for (int sft = 1; sft <= HQ; ++sft) {
      static_assert(HQ <= 2, "DPP shifts of one or two lanes");
      f32x4 l4 = sft == 1 ? q8_dpp4<0x111>(xs) : q8_dpp4<0x112>(xs);  // row_shr: quad cq − sft
      f32x4 r4 = sft == 1 ? q8_dpp4<0x101>(xs) : q8_dpp4<0x102>(xs);  // row_shl: quad cq + sft
      const int ql = cq - sft, qr = cq + sft;
      if (ql < 0) l4 = hrow[HQ + ql];
      if (qr >= Q8QC / 4) r4 = hrow[HQ + (qr - Q8QC / 4)];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        win[4 * (HQ - sft) + e] = l4[e];
        win[4 * (HQ + sft) + e] = r4[e];
      }
    }
#else
    // the lanes of one row slice exchange their quads through the row image
    // (wave-private: LDS instructions of a wave execute in order)
    *reinterpret_cast<f32x4*>(row_img + 4 * cq) = xs;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < 1 + 2 * HQ; ++k) {
      const int qp = cq - HQ + k;  // quad of the row image (−HQ .. 8 + HQ − 1)
      const f32x4* src = qp < 0 ? hrow + (HQ + qp)
                       : qp >= Q8QC / 4 ? hrow + HQ + (qp - Q8QC / 4)
                                        : reinterpret_cast<const f32x4*>(row_img) + qp;
      const f32x4 t4 = *src;
#pragma unroll
      for (int e = 0; e < 4; ++e) win[4 * k + e] = t4[e];
    }
#endif
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int o = 4 * HQ + e;  // window index of column c0 + e
      float a;
      if constexpr (HH == 0) {
        a = win[o];
      } else {  // odd derivative
#ifdef OCM_QP_NOSTENCIL  // make exp timing diagnostic: no stencil arithmetic (wrong values)
        a = win[o + 1] - win[o - 1];
#else
        a = 0.f;
#pragma unroll
        for (int t = 1; t <= HH; ++t) a = fmaf(ct[t], __fsub_rn(win[o + t], win[o - t]), a);
#endif
      }
      y[e] = ocm::mul_nc(a, srj);  // s_r = 1 without SNV (exact)
    }
    if constexpr (HH > 0) {
      // the row's first / last HH columns: the edge rows over the row's first /
      // last WN samples (prep_fused_gram keeps them inside this workgroup's
      // image and halo); deriv ≥ 1 subtracts the output column's own sample
      if (edge_wg) {
        auto at = [&](int col) -> float {
          const int d = col - cg0;
          const float* hf = reinterpret_cast<const float*>(hrow);
          return *(d < 0 ? hf + 4 * HQ + d : d >= Q8QC ? hf + 4 * HQ + (d - Q8QC) : row_img + d);
        };
        // (rolled loops: two workgroup columns of the grid run this, and
        // unrolled it would keep 4·WN addresses live across the row loop)
#pragma unroll 1
        for (int e = 0; e < 4; ++e) {
          const int jc = c0 + e;
          const bool left = jc < HH;
          float a = 0.f;
          if (left || (jc >= p - HH && jc < p)) {
            const int i = left ? jc : HH + jc - (p - HH);
            const int s0 = left ? 0 : p - WN;
            const float ref = at(jc);
#pragma unroll 1
            for (int t = 0; t < WN; ++t) a = fmaf(L.etap[i * WN + t], __fsub_rn(at(s0 + t), ref), a);
            a = ocm::mul_nc(a, srj);
          }
#pragma unroll
          for (int u = 0; u < 4; ++u)
            if (u == e && (left || (jc >= p - HH && jc < p))) y[u] = a;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();  // the image is rewritten by the next row
    if constexpr (WR) {  // eight lanes: one row's 128 B (p % 4 == 0: a quad is all in or all out);
                         // rows past r1 fall outside the descriptor and are dropped
      if (c0 < p)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) unsigned int, y), rs_o, (int)(((16 * rs + j) * ldo + c0) * 4),
                                               0, 0);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) v[j][e] = (g < r1 && c0 + e < p) ? __fsub_rn(y[e], sh[e]) : 0.f;
  }
  __syncthreads();  // q8_tail's LDS overlays the load phase's
  q8_tail(v, tid, cq, rs, cg0, c0, rb, q, chunk, b, st, colblk, lds.tail, th);
}

// Column sums of the quantiser's per-block partials: rows [c0, c1) of colblk
// (P8 wide) → colsum (p).  16 fixed row slices per column, combined in order.
__global__ __launch_bounds__(256) void k_colblk_sum(const double* __restrict__ colblk, int64_t c0, int64_t c1,
                                                    int P8, int p, double* __restrict__ colsum) {
  __shared__ double red[16][16];
  const int cl = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int col = blockIdx.x * 16 + cl;
  double v0 = 0.0, v1 = 0.0;
  int64_t r = c0 + sl;
  for (; r + 16 < c1; r += 32) {
    v0 += colblk[(size_t)r * P8 + col];
    v1 += colblk[(size_t)(r + 16) * P8 + col];
  }
  if (r < c1) v0 += colblk[(size_t)r * P8 + col];
  red[sl][cl] = v0 + v1;
  __syncthreads();
  if (sl == 0 && col < p) {
    double t = 0.0;
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    colsum[col] = t;
  }
}

// ---------------------------------------------------------------------------
// Outlier guard kernels (see the i8×3 header above).
// ---------------------------------------------------------------------------
// Robust column scale of the sample: a histogram of the binary exponent of
// |y| (y = x − shift) per column over the first ≤ 4096 processed rows; the
// median bin gives 2^e ≥ median|y| (≈ 0.67σ for Gaussian data, and a few
// extreme rows in the sample do not move it).  grid (⌈p/64⌉, row splits),
// 256 threads: lane = column, the 4 waves stride over the split's rows.
constexpr int QX_BINS = 128, QX_EMIN = -62;  // bin = clamp(e, −62, 65) + 62; zeros → bin 0
__global__ __launch_bounds__(256) void k_colexp_hist(const float* __restrict__ X, int64_t ldx,
                                                     const int64_t* __restrict__ rows, int64_t n, int p,
                                                     const float* __restrict__ shift, int64_t rows_per_split,
                                                     uint32_t* __restrict__ hist, PrepArgs pa) {
  __shared__ uint32_t h[64][QX_BINS];
  for (int e = threadIdx.x; e < 64 * QX_BINS; e += 256) (&h[0][0])[e] = 0u;
  __syncthreads();
  const int c = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + c;
  const int64_t a = (int64_t)blockIdx.y * rows_per_split;
  const int64_t e = min(n, a + rows_per_split);
  if (col < p) {
    const float sh = shift[col];
    for (int64_t r = a + w; r < e; r += 4) {
      const float y = fabsf(load_y(X, ldx, rows ? rows[r] : r, col, p, pa) - sh);
      int ex = 0;
      (void)frexpf(y, &ex);
      const int bin = y > 0.f ? min(max(ex, QX_EMIN), QX_EMIN + QX_BINS - 1) - QX_EMIN : 0;
      atomicAdd(&h[c][bin], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < 64 * QX_BINS; i += 256) {
    const int cc = i / QX_BINS, bin = i % QX_BINS;
    const uint32_t v = h[cc][bin];
    if (v && blockIdx.x * 64 + cc < p) atomicAdd(hist + (size_t)(blockIdx.x * 64 + cc) * QX_BINS + bin, v);
  }
}

// thr_j = τ·max(2^e_j, 2⁻⁸·max_k 2^e_k), e_j the median exponent bin of
// column j (padded columns: +inf).  The floor keeps near-constant sample
// columns from marking every later row.  First the median bins, one wave per
// column (lane L holds bins 2L, 2L + 1; a wave prefix sum finds the first bin
// whose cumulative count reaches half the sample — a thread walking its
// column's bins one dependent load at a time took 63 µs), then the floor and
// the padding in one workgroup.
__global__ __launch_bounds__(256) void k_q8_colmed(const uint32_t* __restrict__ hist, int64_t nsamp, int p,
                                                   float* __restrict__ thr) {
  static_assert(QX_BINS == 128, "two bins per lane");
  const int lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (c >= p) return;  // whole waves
  const uint32_t half = (uint32_t)((nsamp + 1) / 2);
  const uint32_t h0 = hist[(size_t)c * QX_BINS + 2 * lane], h1 = hist[(size_t)c * QX_BINS + 2 * lane + 1];
  uint32_t inc = h0 + h1;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(inc, o, 64);
    if (lane >= o) inc += v;
  }
  const uint32_t pre = inc - h0 - h1;
  const uint64_t hit = __ballot(inc >= half);
  const int L = hit ? __builtin_ctzll(hit) : 63;
  const uint32_t preL = __shfl(pre, L, 64), h0L = __shfl(h0, L, 64);
  const int bin = hit ? (preL + h0L >= half ? 2 * L : 2 * L + 1) : QX_BINS - 1;
  if (lane == 0) thr[c] = bin == 0 ? 0.f : ldexpf(1.f, bin + QX_EMIN);  // provisional
}

__global__ __launch_bounds__(1024) void k_q8_thresholds(int p, int P8, float* __restrict__ thr) {
  __shared__ float red[16];
  float mx = 0.f;
  for (int c = threadIdx.x; c < p; c += 1024) mx = fmaxf(mx, thr[c]);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, 64));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  float gmax = 0.f;
#pragma unroll
  for (int w = 0; w < 16; ++w) gmax = fmaxf(gmax, red[w]);
  const float floor_ = gmax * (1.f / 256.f);
  for (int c = threadIdx.x; c < P8; c += 1024)
    thr[c] = c < p ? Q8TAU * fmaxf(thr[c], floor_) : __builtin_inff();
}

// zero nf flag words and 4 counters, fill n3 words of b3 with v3 (one launch)
__global__ __launch_bounds__(256) void k_guard_init(uint32_t* __restrict__ flags, size_t nf,
                                                    uint32_t* __restrict__ counters, uint32_t* __restrict__ b3,
                                                    size_t n3, uint32_t v3) {
  const size_t tot = nf + 4 + n3;
  for (size_t e = (size_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (size_t)gridDim.x * 256) {
    if (e < nf) flags[e] = 0u;
    else if (e < nf + 4) counters[e - nf] = 0u;
    else b3[e - nf - 4] = v3;
  }
}

// Marked-row compaction, in processed-row order: per 4096-row block the
// number of marked rows, then each block writes its rows at the prefix of the
// counts before it (ordered lists → a deterministic fix-up sum).
constexpr int FLAG_BLK = 4096;
__device__ __forceinline__ bool row_marked(const uint32_t* __restrict__ flags, int fw, int64_t r) {
  uint32_t o = 0;
  for (int w = 0; w < fw; ++w) o |= flags[(size_t)r * fw + w];
  return o != 0;
}

__global__ __launch_bounds__(256) void k_flag_count(const uint32_t* __restrict__ flags, int fw, int64_t n,
                                                    uint32_t* __restrict__ cnt) {
  __shared__ uint32_t red[4];
  const int64_t base = (int64_t)blockIdx.x * FLAG_BLK + 16 * threadIdx.x;
  uint32_t c = 0;
  for (int j = 0; j < 16; ++j)
    if (base + j < n && row_marked(flags, fw, base + j)) ++c;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

__global__ __launch_bounds__(256) void k_flag_emit(const uint32_t* __restrict__ flags, int fw, int64_t n,
                                                   const uint32_t* __restrict__ cnt, int nblk,
                                                   int64_t* __restrict__ list, uint32_t* __restrict__ nlist) {
  __shared__ uint32_t pre[256];
  uint32_t off = 0;
  for (int b = 0; b < (int)blockIdx.x; ++b) off += cnt[b];
  const int64_t base = (int64_t)blockIdx.x * FLAG_BLK + 16 * threadIdx.x;
  uint32_t mine = 0;
  for (int j = 0; j < 16; ++j)
    if (base + j < n && row_marked(flags, fw, base + j)) mine |= 1u << j;
  pre[threadIdx.x] = (uint32_t)__popc(mine);
  __syncthreads();
  if (threadIdx.x == 0) {  // 256-entry exclusive scan
    uint32_t acc = 0;
    for (int t = 0; t < 256; ++t) {
      const uint32_t v = pre[t];
      pre[t] = acc;
      acc += v;
    }
  }
  __syncthreads();
  uint32_t w = off + pre[threadIdx.x];
  for (int j = 0; j < 16; ++j)
    if ((mine >> j) & 1u) list[w++] = base + j;
  if (blockIdx.x == (unsigned)(nblk - 1) && threadIdx.x == 255) *nlist = w;
}

// G_s += Σ_{marked rows f of segment s} [group(i) or group(j) marked for f] · y_fi y_fj
// (fp64).  grid (upper-triangle 64×64 tiles, segments), 256 threads, each
// thread a 4×4 block of the tile; 16 marked rows per LDS stage.
struct FixSeg {
  int64_t begin[MAXSEG + 1];
  int32_t nseg;
};
constexpr int FX_T = 64, FX_R = 16;
__global__ __launch_bounds__(256) void k_gram_fixup(const float* __restrict__ X, int64_t ldx,
                                                    const int64_t* __restrict__ rows, int p,
                                                    const float* __restrict__ shift, FixSeg fs,
                                                    const int64_t* __restrict__ list,
                                                    const uint32_t* __restrict__ nlist,
                                                    const uint32_t* __restrict__ flags, int fw, int nt,
                                                    double* __restrict__ G, PrepArgs pa) {
  __shared__ double yi[FX_R][FX_T], yj[FX_R][FX_T];
  __shared__ uint32_t mk[FX_R];  // bit 0/1: groups of the I columns, bit 2/3: of the J columns
  const int seg = blockIdx.y;
  int ti, tj;
  tile_coords(blockIdx.x, nt, ti, tj);
  const int I = ti * FX_T, J = tj * FX_T;
  const int64_t lo = fs.begin[seg], hi = fs.begin[seg + 1];
  const int64_t total = (int64_t)*nlist;
  auto lower = [&](int64_t key) {
    int64_t a = 0, b = total;
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (list[m] < key) a = m + 1; else b = m;
    }
    return a;
  };
  const int64_t fa = lower(lo), fb = lower(hi);
  if (fa >= fb) return;
  const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
  const int gI = I / Q8GROUP, gJ = J / Q8GROUP;
  double acc[4][4] = {};
  for (int64_t f0 = fa; f0 < fb; f0 += FX_R) {
    const int nr = (int)min<int64_t>(FX_R, fb - f0);
    __syncthreads();
    for (int e = tid; e < FX_R * FX_T; e += 256) {
      const int r = e / FX_T, c = e % FX_T;
      double a = 0.0, b = 0.0;
      if (r < nr) {
        const int64_t pos = list[f0 + r];
        const int64_t xrow = rows ? rows[pos] : pos;
        if (I + c < p) a = (double)load_y(X, ldx, xrow, I + c, p, pa) - (double)shift[I + c];
        if (J + c < p) b = (double)load_y(X, ldx, xrow, J + c, p, pa) - (double)shift[J + c];
      }
      yi[r][c] = a;
      yj[r][c] = b;
    }
    if (tid < FX_R) {
      uint32_t m = 0;
      if (tid < nr) {
        const int64_t pos = list[f0 + tid];
        auto bit = [&](int g) { return (flags[(size_t)pos * fw + (g >> 5)] >> (g & 31)) & 1u; };
        m = bit(gI) | (bit(gI + 1) << 1) | (bit(gJ) << 2) | (bit(gJ + 1) << 3);
      }
      mk[tid] = m;
    }
    __syncthreads();
    for (int r = 0; r < nr; ++r) {
      const uint32_t m = mk[r];
      const bool mi = (m >> (ty >> 3)) & 1u;        // rows 4ty..4ty+3 lie in group gI + (ty >= 8)
      const bool mj = (m >> (2 + (tx >> 3))) & 1u;
      if (!(mi || mj)) continue;
#pragma unroll
      for (int a = 0; a < 4; ++a) {
        const double u = yi[r][4 * ty + a];
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = fma(u, yj[r][4 * tx + b], acc[a][b]);
      }
    }
  }
  double* Gs = G + (size_t)seg * p * p;
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int gi = I + 4 * ty + a, gj = J + 4 * tx + b;
      if (gi >= p || gj >= p) continue;
      Gs[(size_t)gi * p + gj] += acc[a][b];
      if (ti != tj) Gs[(size_t)gj * p + gi] += acc[a][b];
    }
}

// ---------------------------------------------------------------------------
// k_gram8d — the i8×3 Gram without an LDS stage or workgroup barrier.  The
// digit-plane layout makes one MFMA operand fragment (32 columns × 32 rows:
// lane (r, h) ← column r, bytes 16h..16h+15 of the group) one contiguous
// 1-KiB run, so every wave loads its own A and B fragments straight into
// registers with buffer loads, two stages ahead (2 × 48 VGPRs).  The two
// waves sharing a panel read the same bytes (the CU's L1 serves the second).
// One wave per SIMD, 64×64 per wave; the scale-block flush goes through
// wave-private LDS.
// ---------------------------------------------------------------------------
// band shape of the Gram's tile order (tile rows × tile columns); make exp
// builds override it for A/B
#ifndef OCM_G8_BAND_R
#define OCM_G8_BAND_R 4
#endif
#ifndef OCM_G8_BAND_C
#define OCM_G8_BAND_C 8
#endif
constexpr int G8_BAND_R = OCM_G8_BAND_R, G8_BAND_C = OCM_G8_BAND_C;
__global__ __launch_bounds__(256, 1) void k_gram8d(Q8Plan q, SegTable st, int nt, int ntiles, int total_wg,
                                                   int nwg, int nblocks, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) float scl[4][2 * 64];        // wave-private: row, column scales
  __shared__ __attribute__((aligned(16))) float runl[4][4][4][64][4];  // wave-private f32 running sums

  const int b = blockIdx.x;
  const int q8 = total_wg / 8, r8 = total_wg % 8, x8 = b % 8;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int chunk = wg / nwg;
  // 64×64 blocks packed four per workgroup: the upper triangle of 128×128
  // tiles has 4·ntiles − nt valid blocks (a diagonal tile's strictly-lower
  // block is its mirror), so no wave idles on a diagonal tile.  Blocks are
  // enumerated tile by tile: diagonal tile (0,0) (0,1) (1,1), off-diagonal
  // tiles (0,0) (0,1) (1,0) (1,1).
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int bi = (wg - chunk * nwg) * 4 + wave;
  if (bi >= nblocks) return;  // no barrier in this kernel
  // Tiles are visited in bands of 4 tile rows × 8 tile columns (upper
  // triangle), so the ≈ 32 tiles an XCD runs at once share 12 panels rather
  // than one row panel and 32 column panels: 15 % fewer bytes fetched beyond
  // L2 and 1.5–2 % faster than the row-major triangle order (r02_band).  The
  // walk is wave-uniform scalar work, ≤ ntiles steps at kernel start.
  int ti = -1, tj = 0, wm = 0, wn = 0;
  {
    int rem = bi;
    for (int u = 0; u < nt && ti < 0; u += G8_BAND_R)
      for (int v = u; v < nt && ti < 0; v += G8_BAND_C)
        for (int a = u; a < min(nt, u + G8_BAND_R) && ti < 0; ++a)
          for (int c = max(v, a); c < min(nt, v + G8_BAND_C); ++c) {
            const int nbk = (a == c) ? 3 : 4;
            if (rem < nbk) {
              ti = a;
              tj = c;
              wm = (a == c) ? (rem == 2) : (rem >> 1);
              wn = (a == c) ? (rem >= 1) : (rem & 1);
              break;
            }
            rem -= nbk;
          }
  }
  const int tile = ti * nt - ti * (ti - 1) / 2 + (tj - ti);  // triangle index (the reduce's layout)
  const int I = ti * Q8T, J = tj * Q8T;
  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  const int nb = (int)((r1 - r0 + Q8BLK - 1) / Q8BLK);
  // whole scale blocks (the loop body is one block of 24 stages); the
  // quantiser zero-fills every block of a chunk
  const int nstage3 = nb * Q8SPB;
  const size_t gbase = (size_t)chunk * (st.chunk_rows / Q8K);

  const int lane = threadIdx.x & 63;
  const int l31 = lane & 31, h = lane >> 5;
  const size_t gstride = (size_t)q.P8 * 32;
  const uint32_t span = (uint32_t)((size_t)nstage3 * gstride);
  const char* cbase = q.digits + gbase * gstride;
  __amdgpu_buffer_rsrc_t ra[3], rb[3];
#pragma unroll
  for (int dg = 0; dg < 3; ++dg) {
    ra[dg] = __builtin_amdgcn_make_buffer_rsrc((void*)(cbase + dg * q.plane + (size_t)(I + wm * 64) * 32), 0, span,
                                               0x00020000);
    rb[dg] = __builtin_amdgcn_make_buffer_rsrc((void*)(cbase + dg * q.plane + (size_t)(J + wn * 64) * 32), 0, span,
                                               0x00020000);
  }
  const int voff = l31 * 32 + h * 16;
  const float* srow = q.scale + (size_t)chunk * q.nblk * q.P8 + I + wm * 64 + lane;
  const float* scol = q.scale + (size_t)chunk * q.nblk * q.P8 + J + wn * 64 + lane;

#define Q8D_LOAD_B(FB, x_, dg_, so_) \
  FB[x_][dg_] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(rb[dg_], voff + x_ * 1024, so_, 0)
#define Q8D_LOAD(FA, FB, STG)                                                                         \
  do {                                                                                              \
    const int so_ = (STG) * (int)gstride;                                                           \
    _Pragma("unroll") for (int x_ = 0; x_ < 2; ++x_)                                                \
    _Pragma("unroll") for (int dg_ = 0; dg_ < 3; ++dg_) {                                           \
      FA[x_][dg_] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(ra[dg_], voff + x_ * 1024, so_, 0); \
      Q8D_LOAD_B(FB, x_, dg_, so_);                                                                 \
    }                                                                                               \
  } while (0)
// Z: first stage of a scale block — each accumulator's first product starts
// from an inline zero (no separate reset after the flush)
#define Q8D_MFMA(FA, FB, Z)                                                                           \
  do {                                                                                              \
    _Pragma("unroll") for (int a_ = 0; a_ < 2; ++a_)                                                \
    _Pragma("unroll") for (int c_ = 0; c_ < 2; ++c_) {                                              \
      acc1[a_][c_] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[a_][0], FB[c_][0], (Z) ? i32x16{} : acc1[a_][c_], 0, 0, 0); \
      acc2[a_][c_] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[a_][0], FB[c_][1], (Z) ? i32x16{} : acc2[a_][c_], 0, 0, 0); \
      acc2[a_][c_] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[a_][1], FB[c_][0], acc2[a_][c_], 0, 0, 0); \
      acc3[a_][c_] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[a_][0], FB[c_][2], (Z) ? i32x16{} : acc3[a_][c_], 0, 0, 0); \
      acc3[a_][c_] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[a_][2], FB[c_][0], acc3[a_][c_], 0, 0, 0); \
      acc3[a_][c_] = __builtin_amdgcn_mfma_i32_32x32x32_i8(FA[a_][1], FB[c_][1], acc3[a_][c_], 0, 0, 0); \
    }                                                                                               \
  } while (0)

  i32x16 acc1[2][2], acc2[2][2], acc3[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      acc1[a][c] = i32x16{};
      acc2[a][c] = i32x16{};
      acc3[a][c] = i32x16{};
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<f32x4*>(&runl[wave][a * 2 + c][g][lane][0]) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  float SR = 0.f, SC = 0.f;  // this lane's row / column scale of the current block
  auto flush = [&]() __attribute__((always_inline)) {
    constexpr float w2 = 1.f / 254.f, w3 = 1.f / (254.f * 254.f);
    scl[wave][lane] = SR;  // wave-private: LDS is in order within the wave
    scl[wave][64 + lane] = SC;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float sj = scl[wave][64 + c * 32 + l31];
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          // row scales of registers 4g..4g+3: rows 8g + 4h + 0..3
          const f32x4 si = *reinterpret_cast<const f32x4*>(&scl[wave][a * 32 + 8 * g + 4 * h]);
          f32x4* rp = reinterpret_cast<f32x4*>(&runl[wave][a * 2 + c][g][lane][0]);
          f32x4 rv = *rp;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int r = 4 * g + e;
            const float v = fmaf((float)acc3[a][c][r], w3, fmaf((float)acc2[a][c][r], w2, (float)acc1[a][c][r]));
            rv[e] = fmaf(v, si[e] * sj, rv[e]);
          }
          *rp = rv;
        }
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  };
// stage STG computes on set CUR; the loads of stage STG+2 fill set NXT first
#define Q8D_S0 F0A, F0B, F2A, F2B
#define Q8D_S1 F1A, F1B, F0A, F0B
#define Q8D_S2 F2A, F2B, F1A, F1B
// diagnostic builds only (make exp; timing, not results): NOLOAD never
// refreshes the operands after the prologue, HALFB refreshes only A (the
// load path's share of the kernel time)
#ifdef OCM_G8_DIAG_NOLOAD  // diagnostic build only (make exp): operands never refreshed after the prologue
#define Q8D_REFILL(NA, NB, STG) (void)0
#elif defined(OCM_G8_DIAG_HALFB)  // diagnostic: B operands never refreshed (half the loads)
#define Q8D_REFILL(NA, NB, STG)                                                                       \
  do {                                                                                              \
    const int so_ = (STG) * (int)gstride;                                                           \
    _Pragma("unroll") for (int x_ = 0; x_ < 2; ++x_)                                                \
    _Pragma("unroll") for (int dg_ = 0; dg_ < 3; ++dg_)                                             \
      NA[x_][dg_] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(ra[dg_], voff + x_ * 1024, so_, 0); \
  } while (0)
#else
#define Q8D_REFILL(NA, NB, STG) Q8D_LOAD(NA, NB, STG)
#endif
#if !defined(OCM_G8_BURST) && !defined(OCM_G8_DIAG_NOLOAD) && !defined(OCM_G8_DIAG_HALFB)
  // the 12 refill loads of stage STG+2 interleaved one per two MFMAs of stage
  // STG, in the order the next stages consume them: 399 vs 387 TF for the
  // loads issued as one burst before the MFMAs (OCM_G8_BURST, exp builds)
  auto step_il = [&](i32x4 (&CA)[2][3], i32x4 (&CB)[2][3], i32x4 (&NA)[2][3], i32x4 (&NB)[2][3], int stg,
                     bool z) __attribute__((always_inline)) {
    const int so_ = min(stg + 2, nstage3 - 1) * (int)gstride;
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int x = i / 6, r = i % 6, dg = r / 2;
      if (r & 1)
        NB[x][dg] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(rb[dg], voff + x * 1024, so_, 0);
      else
        NA[x][dg] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(ra[dg], voff + x * 1024, so_, 0);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * i + jj, blk = j / 6, kind = j % 6, a = blk >> 1, c = blk & 1;
        if (kind == 0) acc1[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][0], CB[c][0], z ? i32x16{} : acc1[a][c], 0, 0, 0);
        if (kind == 1) acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][0], CB[c][1], z ? i32x16{} : acc2[a][c], 0, 0, 0);
        if (kind == 2) acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][1], CB[c][0], acc2[a][c], 0, 0, 0);
        if (kind == 3) acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][0], CB[c][2], z ? i32x16{} : acc3[a][c], 0, 0, 0);
        if (kind == 4) acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][2], CB[c][0], acc3[a][c], 0, 0, 0);
        if (kind == 5) acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][1], CB[c][1], acc3[a][c], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
#define Q8D_STEP_(STG, Z, CA, CB, NA, NB) step_il(CA, CB, NA, NB, (STG), (Z))
#else
#define Q8D_STEP_(STG, Z, CA, CB, NA, NB)                                                             \
  do {                                                                                              \
    Q8D_REFILL(NA, NB, min((STG) + 2, nstage3 - 1));                                                \
    __builtin_amdgcn_sched_barrier(0);                                                              \
    Q8D_MFMA(CA, CB, Z);                                                         \
    __builtin_amdgcn_sched_barrier(0);                                                              \
  } while (0)
#endif
#define Q8D_STEP(STG, Z, ...) Q8D_STEP_(STG, Z, __VA_ARGS__)

  i32x4 F0A[2][3], F0B[2][3], F1A[2][3], F1B[2][3], F2A[2][3], F2B[2][3];
  Q8D_LOAD(F0A, F0B, 0);
  Q8D_LOAD(F1A, F1B, min(1, nstage3 - 1));
#if defined(OCM_G8_DIAG_NOLOAD) || defined(OCM_G8_DIAG_HALFB)
  Q8D_LOAD(F2A, F2B, min(2, nstage3 - 1));
#endif
  for (int blk = 0; blk < nb; ++blk) {
    // stage s0+u uses set u % 3 (s0 is a multiple of 48); the loads of stage
    // s0+u+2 go to set (u+2) % 3.  The block's scales are fetched early (they
    // are used by the flush after the last stage).
    const int s0 = blk * Q8SPB;
#pragma unroll
    for (int u = 0; u < Q8SPB; u += 3) {
      Q8D_STEP(s0 + u, u == 0, Q8D_S0);
      Q8D_STEP(s0 + u + 1, false, Q8D_S1);
      if (u == 0) {
        SR = srow[(size_t)blk * q.P8];
        SC = scol[(size_t)blk * q.P8];
      }
      Q8D_STEP(s0 + u + 2, false, Q8D_S2);
    }
    flush();
  }
#undef Q8D_STEP
#undef Q8D_STEP_
#undef Q8D_REFILL
#undef Q8D_S0
#undef Q8D_S1
#undef Q8D_S2
#undef Q8D_MFMA
#undef Q8D_LOAD
#undef Q8D_LOAD_B

  float* out = part + ((size_t)chunk * ntiles + tile) * (Q8T * Q8T);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wn * 64 + c * 32 + l31;
        out[row * Q8T + col] = runl[wave][a * 2 + c][r >> 2][lane][r & 3];
      }
}

// ---------------------------------------------------------------------------
// k_gram8e — k_gram8d's work on the 16×16×64 integer MFMA
// (v_mfma_i32_16x16x64_i8, 16 cycles) instead of 32×32×32 (32 cycles): 419
// vs 386 TF in one process (r03q; the chip holds a higher clock on the
// 16×16 shape).  Same digit planes, 64×64 wave blocks, band order, three
// int32 sets and f32 running sums, so the partials are bit for bit those of
// k_gram8d (the int32 sums are exact; each element's f32 flushes run in the
// same order).  Default launch: a workgroup is one tile's four blocks
// (off-diagonal tiles first, then the diagonal ones packed) and its waves
// meet at a barrier every two stages — a fragment is then loaded by two
// waves of one CU at about the same time and the L1 serves one of them
// (the L2 → CU path is the limit: at full MFMA rate a CU would take 64 B/clk
// of fragments from it).  A stage is 64 rows (two 32-row digit
// groups): lane (c, g) of a fragment holds column c (0..15) of a 16-column
// sub-panel, bytes 16(g & 1) .. +15 of group g >> 1 — the voffset picks the
// group, so the quantiser's layout is unchanged.  Per stage a wave loads 24
// fragments (4 sub-panels × 3 digits for A and for B) for 96 MFMAs, one load
// per four MFMAs, one stage ahead into the other of two register sets.
// ---------------------------------------------------------------------------
// SKIP (the θ3 trace Gram's instantiation only): a chunk stops at its last
// row's stage pair instead of running its last block's zero-padded stages —
// the trace Gram takes all its rows as ONE chunk (a 2048-row Gram of 136 tiles
// as two chunks was 272 workgroups: 34 per XCD of 32 CUs, two rounds of 24
// stages) and so runs 24 + 8 stages in one round.  Not in the headline
// instantiation: the branch in the unrolled stage loop cost it 3 %
// (profiles/r05s9_gram_stage_skip_ab.txt).
template <bool ALIGNED, int SYNC, bool FRONT = false, bool SKIP = false>
__global__ __launch_bounds__(256, 1) void k_gram8e(Q8Plan q, SegTable st, int nt, int ntiles, int total_wg,
                                                   int nwg, int nblocks, float* __restrict__ part, int chunk0) {
  __shared__ __attribute__((aligned(16))) float scl[4][2 * 64];      // wave-private: row, column scales
  __shared__ __attribute__((aligned(16))) float runl[4][16][64][4];  // wave-private f32 running sums

  const int b = blockIdx.x;
  const int q8 = total_wg / 8, r8 = total_wg % 8, x8 = b % 8;
  // XCD-aware remap (each XCD a contiguous range of chunks); chunk0 < 0 (A/B
  // only): dispatch order, the eight XCDs on neighbouring tiles of one chunk
  const int wg = chunk0 < 0 ? b : (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int cl = wg / nwg, chunk = (chunk0 < 0 ? 0 : chunk0) + cl;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int bi = (wg - cl * nwg) * 4 + wave;
  // SYNC > 0: a workgroup barrier every SYNC stages keeps the four waves in
  // step, so the second wave's load of a shared panel fragment finds it in
  // the CU's L1; a wave past the last block then computes a copy of the last
  // block (never stored) instead of leaving
  const bool dead = bi >= nblocks;
  if (dead && SYNC == 0) return;
  if (dead) bi = nblocks - 1;
  int ti = -1, tj = 0, wm = 0, wn = 0;
  if (ALIGNED) {
    // off-diagonal tiles first, in band order, four blocks each: a
    // workgroup's four waves are one tile's four blocks, so each A and B
    // panel fragment is fetched by two waves of the same CU (the L1 serves the
    // second); then the nt diagonal tiles, three blocks each, packed
    const int noff = 4 * (ntiles - nt);
    if (bi < noff) {
      int rem = bi >> 2;
      wm = (bi >> 1) & 1;
      wn = bi & 1;
      for (int u = 0; u < nt && ti < 0; u += G8_BAND_R)
        for (int v = u; v < nt && ti < 0; v += G8_BAND_C)
          for (int a = u; a < min(nt, u + G8_BAND_R) && ti < 0; ++a)
            for (int c = max(v, a + 1); c < min(nt, v + G8_BAND_C); ++c) {
              if (rem == 0) {
                ti = a;
                tj = c;
                break;
              }
              --rem;
            }
    } else {
      const int d = (bi - noff) / 3, r = (bi - noff) - 3 * d;
      ti = tj = d;
      wm = (r == 2);
      wn = (r >= 1);
    }
  } else {
    int rem = bi;
    for (int u = 0; u < nt && ti < 0; u += G8_BAND_R)
      for (int v = u; v < nt && ti < 0; v += G8_BAND_C)
        for (int a = u; a < min(nt, u + G8_BAND_R) && ti < 0; ++a)
          for (int c = max(v, a); c < min(nt, v + G8_BAND_C); ++c) {
            const int nbk = (a == c) ? 3 : 4;
            if (rem < nbk) {
              ti = a;
              tj = c;
              wm = (a == c) ? (rem == 2) : (rem >> 1);
              wn = (a == c) ? (rem >= 1) : (rem & 1);
              break;
            }
            rem -= nbk;
          }
  }
  const int tile = ti * nt - ti * (ti - 1) / 2 + (tj - ti);
  const int I = ti * Q8T, J = tj * Q8T;
  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  const int nb = (int)((r1 - r0 + Q8BLK - 1) / Q8BLK);
  constexpr int SPB = Q8BLK / 64;  // 64-row stages per scale block (24)
  const int nstage = nb * SPB;
  const size_t gbase = (size_t)chunk * (st.chunk_rows / Q8K);

  const int lane = threadIdx.x & 63;
  const int l15 = lane & 15, g4 = lane >> 4;
  const size_t gstride = (size_t)q.P8 * 32;
  const uint32_t span = (uint32_t)((size_t)nb * Q8SPB * gstride);
  const char* cbase = q.digits + gbase * gstride;
  __amdgpu_buffer_rsrc_t ra[3], rb[3];
#pragma unroll
  for (int dg = 0; dg < 3; ++dg) {
    ra[dg] = __builtin_amdgcn_make_buffer_rsrc((void*)(cbase + dg * q.plane + (size_t)(I + wm * 64) * 32), 0, span,
                                               0x00020000);
    rb[dg] = __builtin_amdgcn_make_buffer_rsrc((void*)(cbase + dg * q.plane + (size_t)(J + wn * 64) * 32), 0, span,
                                               0x00020000);
  }
  // sub-panel x of the wave's 64 columns: column 16x + l15, group g4 >> 1, half g4 & 1
  const int voff = (g4 >> 1) * (int)gstride + l15 * 32 + (g4 & 1) * 16;
  const int sstride = 2 * (int)gstride;
  const float* srow = q.scale + (size_t)chunk * q.nblk * q.P8 + I + wm * 64 + lane;
  const float* scol = q.scale + (size_t)chunk * q.nblk * q.P8 + J + wn * 64 + lane;

  i32x4 acc1[4][4], acc2[4][4], acc3[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      acc1[a][c] = i32x4{};
      acc2[a][c] = i32x4{};
      acc3[a][c] = i32x4{};
      *reinterpret_cast<f32x4*>(&runl[wave][a * 4 + c][lane][0]) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  float SR = 0.f, SC = 0.f;
  auto flush = [&]() __attribute__((always_inline)) {
    constexpr float w2 = 1.f / 254.f, w3 = 1.f / (254.f * 254.f);
    scl[wave][lane] = SR;  // wave-private: LDS is in order within the wave
    scl[wave][64 + lane] = SC;
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      // row scales of registers 0..3: rows 16a + 4g4 + 0..3
      const f32x4 si = *reinterpret_cast<const f32x4*>(&scl[wave][a * 16 + 4 * g4]);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float sj = scl[wave][64 + c * 16 + l15];
        f32x4* rp = reinterpret_cast<f32x4*>(&runl[wave][a * 4 + c][lane][0]);
        f32x4 rv = *rp;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = fmaf((float)acc3[a][c][e], w3, fmaf((float)acc2[a][c][e], w2, (float)acc1[a][c][e]));
          rv[e] = fmaf(v, si[e] * sj, rv[e]);
        }
        *rp = rv;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // fragment load i (0..23) of a stage, in the order the stage's MFMAs first
  // use them: A0, B0, B1, B2, B3, A1, A2, A3 (three digits each)
  auto load_frag = [&](i32x4 (&FA)[4][3], i32x4 (&FB)[4][3], int i, int so) __attribute__((always_inline)) {
    const int grp = i / 3, dg = i % 3;
    if (grp >= 1 && grp <= 4)
      FB[grp - 1][dg] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(rb[dg], voff + (grp - 1) * 512, so, 0);
    else {
      const int x = grp == 0 ? 0 : grp - 4;
      FA[x][dg] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(ra[dg], voff + x * 512, so, 0);
    }
  };
  // one stage: 96 MFMAs on (CA, CB), sub-blocks row-major, six products each;
  // the 24 loads of the next stage into (NA, NB), one per four MFMAs
  auto step = [&](i32x4 (&CA)[4][3], i32x4 (&CB)[4][3], i32x4 (&NA)[4][3], i32x4 (&NB)[4][3], int stg,
                  bool z) __attribute__((always_inline)) {
    const int so = min(stg + 1, nstage - 1) * sstride;
    // FRONT (A/B only): the 24 loads one per two MFMAs over the first half of
    // the stage instead of one per four over the whole stage — 392 vs 439 TF
    constexpr int GRP = FRONT ? 48 : 24, PER = 96 / GRP;
#pragma unroll
    for (int i = 0; i < GRP; ++i) {
#ifndef OCM_G8E_DIAG_NOLOAD  // diagnostic build only (make exp): operands never refreshed (timing, not results)
      if (i < 24) load_frag(NA, NB, i, so);
#else
      (void)so;
#endif
#pragma unroll
      for (int jj = 0; jj < PER; ++jj) {
        const int j = PER * i + jj, blk = j / 6, kind = j % 6, a = blk >> 2, c = blk & 3;
        if (kind == 0) acc1[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(CA[a][0], CB[c][0], z ? i32x4{} : acc1[a][c], 0, 0, 0);
        if (kind == 1) acc2[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(CA[a][0], CB[c][1], z ? i32x4{} : acc2[a][c], 0, 0, 0);
        if (kind == 2) acc2[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(CA[a][1], CB[c][0], acc2[a][c], 0, 0, 0);
        if (kind == 3) acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(CA[a][0], CB[c][2], z ? i32x4{} : acc3[a][c], 0, 0, 0);
        if (kind == 4) acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(CA[a][2], CB[c][0], acc3[a][c], 0, 0, 0);
        if (kind == 5) acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(CA[a][1], CB[c][1], acc3[a][c], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    if (SYNC > 0 && stg % SYNC == SYNC - 1) __builtin_amdgcn_s_barrier();
  };

  const int nvs = SKIP ? (int)((r1 - r0 + 63) / 64) : nstage;  // stages holding rows (the rest are zero digits)
  i32x4 F0A[4][3], F0B[4][3], F1A[4][3], F1B[4][3];
#pragma unroll
  for (int i = 0; i < 24; ++i) load_frag(F0A, F0B, i, 0);
  for (int blk = 0; blk < nb; ++blk) {
    const int s0 = blk * SPB;
#pragma unroll
    for (int u = 0; u < SPB; u += 2) {
      if (SKIP && u > 0 && s0 + u >= nvs) break;
      step(F0A, F0B, F1A, F1B, s0 + u, u == 0);
      if (u == 0) {
        SR = srow[(size_t)blk * q.P8];
        SC = scol[(size_t)blk * q.P8];
      }
      step(F1A, F1B, F0A, F0B, s0 + u + 1, false);
    }
    flush();
  }

  if (dead) return;
  float* out = part + ((size_t)chunk * ntiles + tile) * (Q8T * Q8T);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * 64 + a * 16 + 4 * g4 + e;
        const int col = wn * 64 + c * 16 + l15;
        out[row * Q8T + col] = runl[wave][a * 4 + c][lane][e];
      }
}

#ifdef OCM_G8_LDS
// ---------------------------------------------------------------------------
// k_gram8x (experiment, make exp only: OCM_GRAM8_ORDER=lds) — k_gram8e with
// the panels shared through LDS.  Measured (r03u, r03v): bit-identical, 362–367
// TF against the default launch's 439–445 in the same processes, with the
// partner reads as one burst or split — not kept.  One workgroup per
// 128×128 tile (off-diagonal tiles in band order, then the diagonal ones; a
// diagonal tile's mirror wave loads and stages its share but computes
// nothing).  Waves (wm, wn) and (wm, 1−wn) need the same A panel, (wm, wn)
// and (1−wm, wn) the same B panel: each wave loads only half of its 24
// fragments per 64-row stage from global memory (A sub-panels 2wn, 2wn+1 and
// B sub-panels 2wm, 2wm+1: its "own" 12), writes them to a two-slot LDS ring
// and reads the other 12 from its partners' slots, so the L2 → CU traffic is
// halved.  Stage t: read the partners' fragments of t (written before the
// barrier that ended stage t−1); the 24 MFMAs of own × own sub-blocks cover
// that read; the own loads of stage t+2 go out one per MFMA group, and the
// own fragments of t+1 (loaded during t−1) are written to the other slot
// during the last 72 MFMAs; lgkmcnt(0) + barrier.  Sub-block indices are kept
// relative (own first): actual sub-panel = relative ^ (2·wn) for A and
// ^ (2·wm) for B, applied to the load offsets and the output positions only.
// Same exact int32 sets and f32 flush order as k_gram8d/8e: bit-identical.
// ---------------------------------------------------------------------------
constexpr int G8X_FRAG = 1024, G8X_WSLOT = 12 * G8X_FRAG, G8X_SLOT = 4 * G8X_WSLOT;
__global__ __launch_bounds__(256, 1) void k_gram8x(Q8Plan q, SegTable st, int nt, int ntiles, int total_wg,
                                                   float* __restrict__ part) {
  __shared__ __attribute__((aligned(1024))) char ring[2 * G8X_SLOT];     // 96 KiB
  __shared__ __attribute__((aligned(16))) float runl[4][16][64][4];      // 64 KiB: wave-private f32 running sums

  const int b = blockIdx.x;
  const int q8 = total_wg / 8, r8 = total_wg % 8, x8 = b % 8;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int chunk = wg / ntiles;
  const int tix = wg - chunk * ntiles;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  int ti = -1, tj = 0;
  if (tix < ntiles - nt) {
    int rem = tix;
    for (int u = 0; u < nt && ti < 0; u += G8_BAND_R)
      for (int v = u; v < nt && ti < 0; v += G8_BAND_C)
        for (int a = u; a < min(nt, u + G8_BAND_R) && ti < 0; ++a)
          for (int c = max(v, a + 1); c < min(nt, v + G8_BAND_C); ++c) {
            if (rem == 0) {
              ti = a;
              tj = c;
              break;
            }
            --rem;
          }
  } else {
    ti = tj = tix - (ntiles - nt);
  }
  const bool mirror = (ti == tj) && wm == 1 && wn == 0;  // a diagonal tile's strictly-lower block
  const int tile = ti * nt - ti * (ti - 1) / 2 + (tj - ti);
  const int I = ti * Q8T, J = tj * Q8T;
  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  const int nb = (int)((r1 - r0 + Q8BLK - 1) / Q8BLK);
  constexpr int SPB = Q8BLK / 64;  // 64-row stages per scale block (24, a multiple of 3)
  const int nstage = nb * SPB;
  const size_t gbase = (size_t)chunk * (st.chunk_rows / Q8K);

  const int lane = threadIdx.x & 63;
  const int l15 = lane & 15, g4 = lane >> 4;
  const size_t gstride = (size_t)q.P8 * 32;
  const uint32_t span = (uint32_t)((size_t)nb * Q8SPB * gstride);
  const char* cbase = q.digits + gbase * gstride;
  __amdgpu_buffer_rsrc_t ra[3], rb[3];
#pragma unroll
  for (int dg = 0; dg < 3; ++dg) {
    ra[dg] = __builtin_amdgcn_make_buffer_rsrc((void*)(cbase + dg * q.plane + (size_t)(I + wm * 64) * 32), 0, span,
                                               0x00020000);
    rb[dg] = __builtin_amdgcn_make_buffer_rsrc((void*)(cbase + dg * q.plane + (size_t)(J + wn * 64) * 32), 0, span,
                                               0x00020000);
  }
  // own sub-panels: A 2wn + j, B 2wm + j (j = 0, 1)
  const int voff = (g4 >> 1) * (int)gstride + l15 * 32 + (g4 & 1) * 16;
  const int voffA = voff + 2 * wn * 512, voffB = voff + 2 * wm * 512;
  const int sstride = 2 * (int)gstride;
  const float* srow = q.scale + (size_t)chunk * q.nblk * q.P8 + I + wm * 64 + lane;
  const float* scol = q.scale + (size_t)chunk * q.nblk * q.P8 + J + wn * 64 + lane;
  // LDS: own fragment i of slot u at ring + u·SLOT + wave·WSLOT + i·FRAG;
  // partner A fragments from wave ^ 1 (its own A, indices 0..5), partner B
  // from wave ^ 2 (its own B, indices 6..11)
  char* const wr_base = ring + wave * G8X_WSLOT + lane * 16;
  const char* const rdA_base = ring + (wave ^ 1) * G8X_WSLOT + lane * 16;
  const char* const rdB_base = ring + (wave ^ 2) * G8X_WSLOT + 6 * G8X_FRAG + lane * 16;

  i32x4 acc1[4][4], acc2[4][4], acc3[4][4];  // [relative a][relative c]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      acc1[a][c] = i32x4{};
      acc2[a][c] = i32x4{};
      acc3[a][c] = i32x4{};
      *reinterpret_cast<f32x4*>(&runl[wave][a * 4 + c][lane][0]) = f32x4{0.f, 0.f, 0.f, 0.f};
    }
  float SR = 0.f, SC = 0.f;
  auto flush = [&]() __attribute__((always_inline)) {
    constexpr float w2 = 1.f / 254.f, w3 = 1.f / (254.f * 254.f);
#pragma unroll
    for (int a = 0; a < 4; ++a) {
      const int aa = a ^ (2 * wn);  // actual sub-panel: rows 16aa + 4g4 + e
      f32x4 si;
#pragma unroll
      for (int e = 0; e < 4; ++e) si[e] = __shfl(SR, aa * 16 + 4 * g4 + e);
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float sj = __shfl(SC, (c ^ (2 * wm)) * 16 + l15);
        f32x4* rp = reinterpret_cast<f32x4*>(&runl[wave][a * 4 + c][lane][0]);
        f32x4 rv = *rp;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float v = fmaf((float)acc3[a][c][e], w3, fmaf((float)acc2[a][c][e], w2, (float)acc1[a][c][e]));
          rv[e] = fmaf(v, si[e] * sj, rv[e]);
        }
        *rp = rv;
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // own fragment i (0..5: A j = i / 3, 6..11: B j = (i − 6) / 3; digit i % 3)
  auto gload = [&](i32x4 (&OA)[2][3], i32x4 (&OB)[2][3], int i, int so) __attribute__((always_inline)) {
    const int j = (i % 6) / 3, dg = i % 3;
    if (i < 6)
      OA[j][dg] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(ra[dg], voffA + j * 512, so, 0);
    else
      OB[j][dg] = (i32x4)__builtin_amdgcn_raw_buffer_load_b128(rb[dg], voffB + j * 512, so, 0);
  };
  auto mfma6 = [&](const i32x4 (&A)[3], const i32x4 (&B)[3], int a, int c, bool z) __attribute__((always_inline)) {
    acc1[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[0], z ? i32x4{} : acc1[a][c], 0, 0, 0);
    acc2[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[1], z ? i32x4{} : acc2[a][c], 0, 0, 0);
    acc2[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B[0], acc2[a][c], 0, 0, 0);
    acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[2], z ? i32x4{} : acc3[a][c], 0, 0, 0);
    acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2], B[0], acc3[a][c], 0, 0, 0);
    acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B[1], acc3[a][c], 0, 0, 0);
  };
  i32x4 PA[2][3], PB[2][3];  // partner fragments of the current stage
  // stage t: CUR = own(t), NXT = own(t+1) (landed, staged to LDS during t),
  // FUT = own(t+2) (loaded during t)
  auto step = [&](i32x4 (&CA)[2][3], i32x4 (&CB)[2][3], i32x4 (&NA)[2][3], i32x4 (&NB)[2][3], i32x4 (&FA)[2][3],
                  i32x4 (&FB)[2][3], int stg, bool z) __attribute__((always_inline)) {
    const int rs = (stg & 1) * G8X_SLOT, ws = ((stg + 1) & 1) * G8X_SLOT;
    const int so = min(stg + 2, nstage - 1) * sstride;
    // partner B (used from the second quarter) first, partner A (third
    // quarter) two sub-blocks later: the LDS read burst is spread
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int dg = 0; dg < 3; ++dg)
        PB[j][dg] = *reinterpret_cast<const i32x4*>(rdB_base + rs + (j * 3 + dg) * G8X_FRAG);
    // 16 sub-blocks in four quarters: own × own, own × partner, partner × own, partner × partner
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const int qd = g >> 2, a = g & 1 ? 1 : 0, c = (g >> 1) & 1;
      if (g == 2) {
#pragma unroll
        for (int j = 0; j < 2; ++j)
#pragma unroll
          for (int dg = 0; dg < 3; ++dg)
            PA[j][dg] = *reinterpret_cast<const i32x4*>(rdA_base + rs + (j * 3 + dg) * G8X_FRAG);
      }
      if (g < 12) gload(FA, FB, g, so);
      if (g >= 4) {
        const int i = g - 4;  // 12 staging writes over the last 12 sub-blocks
        const int jj = (i % 6) / 3, dg = i % 3;
        *reinterpret_cast<i32x4*>(wr_base + ws + i * G8X_FRAG) = i < 6 ? NA[jj][dg] : NB[jj][dg];
      }
      if (!mirror) {
        if (qd == 0) mfma6(CA[a], CB[c], a, c, z);
        if (qd == 1) mfma6(CA[a], PB[c], a, 2 + c, z);
        if (qd == 2) mfma6(PA[a], CB[c], 2 + a, c, z);
        if (qd == 3) mfma6(PA[a], PB[c], 2 + a, 2 + c, z);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  };

  i32x4 O0A[2][3], O0B[2][3], O1A[2][3], O1B[2][3], O2A[2][3], O2B[2][3];
#pragma unroll
  for (int i = 0; i < 12; ++i) gload(O0A, O0B, i, 0);
#pragma unroll
  for (int i = 0; i < 12; ++i) gload(O1A, O1B, i, min(1, nstage - 1) * sstride);
#pragma unroll
  for (int i = 0; i < 12; ++i) {
    const int jj = (i % 6) / 3, dg = i % 3;
    *reinterpret_cast<i32x4*>(wr_base + i * G8X_FRAG) = i < 6 ? O0A[jj][dg] : O0B[jj][dg];
  }
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
  for (int blk = 0; blk < nb; ++blk) {
    const int s0 = blk * SPB;
#pragma unroll
    for (int u = 0; u < SPB; u += 3) {
      step(O0A, O0B, O1A, O1B, O2A, O2B, s0 + u, u == 0);
      if (u == 0) {
        SR = srow[(size_t)blk * q.P8];
        SC = scol[(size_t)blk * q.P8];
      }
      step(O1A, O1B, O2A, O2B, O0A, O0B, s0 + u + 1, false);
      step(O2A, O2B, O0A, O0B, O1A, O1B, s0 + u + 2, false);
    }
    if (!mirror) flush();
  }
  if (mirror) return;
  float* out = part + ((size_t)chunk * ntiles + tile) * (Q8T * Q8T);
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = wm * 64 + (a ^ (2 * wn)) * 16 + 4 * g4 + e;
        const int col = wn * 64 + (c ^ (2 * wm)) * 16 + l15;
        out[row * Q8T + col] = runl[wave][a * 4 + c][lane][e];
      }
}
#endif  // OCM_G8_LDS

#ifdef OCM_G8_LDS
// ---------------------------------------------------------------------------
// k_gram8s (experiment, make exp only) — the i8×3 Gram with the workgroup's
// two 128-column panels shared through LDS.  One workgroup per 128×128 tile,
// four waves of 64×64; each 64-row phase (two 32-row stages) of both panels
// (48 KiB) is copied once into a 3-slot LDS ring by LDS-DMA
// (global_load_lds_dwordx4: one 1-KiB fragment per wave-instruction, 12 per
// wave per phase + the block's row/column scales into a 4-slot scale ring),
// three phases ahead.  Each wave reads its fragments with ds_read_b128 one
// stage ahead of the MFMAs that use them, one read per two MFMAs; one counted
// vmcnt wait + one raw barrier per phase, between the two stages.  The fragment
// image is lane-linear with the halves of column r swapped when bit 3 of r is
// set (applied on the DMA source and on the read): conflict-free reads.
// Measured (r02_lds, 1M × 2048): parity equal to k_gram8d (3.6e-8 vs fp64),
// 305 TF against k_gram8d's 393 in the same process pair — halving the
// vector-memory bytes per MFMA does not pay for the per-phase barrier; kept
// for the next round's LDS / tile-order work, never in libocm.
// ---------------------------------------------------------------------------
constexpr int G8S_FRAG = 1024;
constexpr int G8S_OPS = 2 * 2 * 3 * 4 * G8S_FRAG;  // [stage][A|B][digit][32-col block] = 48 KiB
constexpr int G8S_NSLOT = 3;
constexpr int G8S_SCL = 4 * 512;                   // [wave][64 row scales | 64 column scales]
constexpr int G8S_NSCL = 4;

// LDS-DMA with a scalar 64-bit base and a 32-bit per-lane offset (saddr form):
// no per-lane 64-bit addresses to keep live across the loop
__device__ __forceinline__ void g8s_dma16(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}
__device__ __forceinline__ void g8s_dma4(const void* sbase, uint32_t voff, uint32_t lds) {
  uint32_t keep;
  asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\tglobal_load_lds_dword %1, %2\n\ts_mov_b32 m0, %0"
               : "=&s"(keep)
               : "v"(voff), "s"(sbase), "s"(lds)
               : "memory");
}

__global__ __launch_bounds__(256, 1) void k_gram8s(Q8Plan q, SegTable st, int nt, int ntiles, int total_wg,
                                                   float* __restrict__ part) {
  __shared__ __attribute__((aligned(1024))) char lds[G8S_NSLOT * G8S_OPS + G8S_NSCL * G8S_SCL];

  const int b = blockIdx.x;
  const int q8 = total_wg / 8, r8 = total_wg % 8, x8 = b % 8;
  const int wg = (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + b / 8;
  const int chunk = wg / ntiles;
  const int tile = wg - chunk * ntiles;
  int ti, tj;
  tile_coords(tile, nt, ti, tj);
  const int I = ti * Q8T, J = tj * Q8T;
  int s = 0;
  while (s + 1 < st.nseg && chunk >= st.cprefix[s + 1]) ++s;
  const int64_t r0 = st.begin[s] + (int64_t)(chunk - st.cprefix[s]) * st.chunk_rows;
  const int64_t r1 = min(r0 + (int64_t)st.chunk_rows, st.begin[s + 1]);
  const int nb = (int)((r1 - r0 + Q8BLK - 1) / Q8BLK);
  constexpr int PPB = Q8SPB / 2;  // phases per scale block
  const int nph = nb * PPB;
  const size_t gbase = (size_t)chunk * (st.chunk_rows / Q8K);

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int l31 = lane & 31, h = lane >> 5;
  const bool skip = (ti == tj && wm > wn);  // the mirror block of a diagonal tile: computed, not stored
  const size_t gstride = (size_t)q.P8 * 32;

  // DMA role: stage (wave >> 1) of a phase, operand (wave & 1): 3 digits × 4 column blocks
  const int sg_dma = wave >> 1, op_dma = wave & 1;
  const uint32_t srcoff = (uint32_t)(lane >> 1) * 32 + 16 * ((lane & 1) ^ ((lane >> 4) & 1));
  const char* dma_base = q.digits + (gbase + sg_dma) * gstride + (size_t)(op_dma ? J : I) * 32;
  const uint32_t lds0 = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds);
  const float* scl_src = q.scale + (size_t)chunk * q.nblk * q.P8;
  const uint32_t scloff = (uint32_t)lane * 4;
  const int srow0 = I + wm * 64, scol0 = J + wn * 64;

  auto issue = [&](int ph) __attribute__((always_inline)) {
    const int phc = min(ph, nph - 1);
    const uint32_t sb = lds0 + (uint32_t)((ph % G8S_NSLOT) * G8S_OPS);
    const size_t poff = (size_t)phc * 2 * gstride;
#pragma unroll
    for (int dg = 0; dg < 3; ++dg)
#pragma unroll
      for (int x = 0; x < 4; ++x)
        g8s_dma16(dma_base + dg * q.plane + poff + x * G8S_FRAG, srcoff,
                  sb + (((sg_dma * 2 + op_dma) * 3 + dg) * 4 + x) * G8S_FRAG);
    const size_t so = (size_t)(phc / PPB) * q.P8;
    const uint32_t scb = lds0 + (uint32_t)(G8S_NSLOT * G8S_OPS + (ph % G8S_NSCL) * G8S_SCL + wave * 512);
    g8s_dma4(scl_src + so + srow0, scloff, scb);
    g8s_dma4(scl_src + so + scol0, scloff, scb + 256);
  };
  const int rdoff = 16 * (2 * l31 + (h ^ ((l31 >> 3) & 1)));
  auto frag = [&](int slot, int sg, int op, int dg, int xb) __attribute__((always_inline)) -> i32x4 {
    return *reinterpret_cast<const i32x4*>(lds + slot * G8S_OPS + (((sg * 2 + op) * 3 + dg) * 4 + xb) * G8S_FRAG +
                                           rdoff);
  };

  i32x16 acc1[2][2], acc2[2][2], acc3[2][2];
  float run[2][2][16];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      acc1[a][c] = i32x16{};
      acc2[a][c] = i32x16{};
      acc3[a][c] = i32x16{};
#pragma unroll
      for (int r = 0; r < 16; ++r) run[a][c][r] = 0.f;
    }
  // one stage: 24 MFMAs on (CA, CB); the 12 fragments of the next stage read
  // from LDS into (NA, NB), one per two MFMAs
  auto half = [&](i32x4 (&CA)[2][3], i32x4 (&CB)[2][3], i32x4 (&NA)[2][3], i32x4 (&NB)[2][3], int rslot,
                  int rsg) __attribute__((always_inline)) {
#pragma unroll
    for (int i = 0; i < 12; ++i) {
      const int x = i / 6, r = i % 6, dg = r / 2;
      if (r & 1)
        NB[x][dg] = frag(rslot, rsg, 1, dg, 2 * wn + x);
      else
        NA[x][dg] = frag(rslot, rsg, 0, dg, 2 * wm + x);
#pragma unroll
      for (int jj = 0; jj < 2; ++jj) {
        const int j = 2 * i + jj, blk = j / 6, kind = j % 6, a = blk >> 1, c = blk & 1;
        if (kind == 0) acc1[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][0], CB[c][0], acc1[a][c], 0, 0, 0);
        if (kind == 1) acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][0], CB[c][1], acc2[a][c], 0, 0, 0);
        if (kind == 2) acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][1], CB[c][0], acc2[a][c], 0, 0, 0);
        if (kind == 3) acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][0], CB[c][2], acc3[a][c], 0, 0, 0);
        if (kind == 4) acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][2], CB[c][0], acc3[a][c], 0, 0, 0);
        if (kind == 5) acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(CA[a][1], CB[c][1], acc3[a][c], 0, 0, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  i32x4 R0A[2][3], R0B[2][3], R1A[2][3], R1B[2][3];
  issue(0);
  issue(1);
  issue(2);
  asm volatile("s_waitcnt vmcnt(28)\n\ts_barrier" ::: "memory");  // phase 0 landed for every wave
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int dg = 0; dg < 3; ++dg) {
      R0A[x][dg] = frag(0, 0, 0, dg, 2 * wm + x);
      R0B[x][dg] = frag(0, 0, 1, dg, 2 * wn + x);
    }
  for (int ph = 0; ph < nph; ++ph) {
    half(R0A, R0B, R1A, R1B, ph % G8S_NSLOT, 1);
    // this wave's DMAs of phase ph+1 are done (those of ph+2 may fly); every
    // wave's reads of slot ph%3 are done: it takes phase ph+3
    asm volatile("s_waitcnt vmcnt(14) lgkmcnt(0)\n\ts_barrier" ::: "memory");
    issue(ph + 3);
    half(R1A, R1B, R0A, R0B, (ph + 1) % G8S_NSLOT, 0);
    if (ph % PPB == PPB - 1) {
      constexpr float w2 = 1.f / 254.f, w3 = 1.f / (254.f * 254.f);
      const float* scl = reinterpret_cast<const float*>(lds + G8S_NSLOT * G8S_OPS + (ph % G8S_NSCL) * G8S_SCL +
                                                        wave * 512);
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float sj = scl[64 + c * 32 + l31];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x4 si = *reinterpret_cast<const f32x4*>(&scl[a * 32 + 8 * g + 4 * h]);
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int r = 4 * g + e;
              const float v = fmaf((float)acc3[a][c][r], w3, fmaf((float)acc2[a][c][r], w2, (float)acc1[a][c][r]));
              run[a][c][r] = fmaf(v, si[e] * sj, run[a][c][r]);
            }
          }
          acc1[a][c] = i32x16{};
          acc2[a][c] = i32x16{};
          acc3[a][c] = i32x16{};
        }
      }
    }
  }
  // no LDS-DMA may still be landing when the workgroup's LDS is released
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (skip) return;
  float* out = part + ((size_t)chunk * ntiles + tile) * (Q8T * Q8T);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wn * 64 + c * 32 + l31;
        out[row * Q8T + col] = run[a][c][r];
      }
}
#endif  // OCM_G8_LDS

int gram_small(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int32_t p, const float* shift,
               const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out, hipStream_t st) {
  // chunks never straddle a segment: span = (lo, hi) row range per chunk
  std::vector<int64_t> span;
  std::vector<int> cpre(nseg + 1, 0);
  for (int s = 0; s < nseg; ++s) {
    cpre[s] = (int)(span.size() / 2);
    for (int64_t a = seg_offsets[s]; a < seg_offsets[s + 1]; a += SMALL_CHUNK) {
      span.push_back(a);
      span.push_back(std::min<int64_t>(a + SMALL_CHUNK, seg_offsets[s + 1]));
    }
  }
  const int nchunk = (int)(span.size() / 2);
  cpre[nseg] = nchunk;
  const int npair = p * (p + 1) / 2;
  const size_t need = (size_t)nchunk * (npair + p) * sizeof(double) + span.size() * sizeof(int64_t) + 1024;
  void* w = ocm::workspace(ctx, need, st);
  if (!w) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(w)};
  double* part = cv.take<double>((size_t)nchunk * npair);
  double* cpart = cv.take<double>((size_t)nchunk * p);
  int64_t* dspan = cv.take<int64_t>(span.size());
  if (nchunk > 0) {
    // pageable source: staged before the call returns
    OCM_HIP(hipMemcpyAsync(dspan, span.data(), span.size() * sizeof(int64_t), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_gram_small, dim3(nchunk), dim3(256), 0, st, X, ldx, rows, p, shift, dspan, part, cpart);
    OCM_CHECK_LAUNCH("k_gram_small");
  }
  for (int s = 0; s < nseg; ++s) {
    double* Gs = G_out + (size_t)s * p * p;
    double* cs = colsum_out + (size_t)s * p;
    if (cpre[s + 1] == cpre[s]) {
      OCM_HIP(hipMemsetAsync(Gs, 0, (size_t)p * p * sizeof(double), st));
      OCM_HIP(hipMemsetAsync(cs, 0, (size_t)p * sizeof(double), st));
      continue;
    }
    hipLaunchKernelGGL(k_gram_small_reduce, dim3((npair + 255) / 256), dim3(256), 0, st, part, cpart, p, cpre[s],
                       cpre[s + 1], Gs, cs);
    OCM_CHECK_LAUNCH("k_gram_small_reduce");
  }
  return OCM_OK;
}

template <int GT, int BK>
int gram_impl(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
              const float* shift, const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out,
              hipStream_t st, int64_t chunk_rows, bool split3 = false) {
  if (GT != 256) split3 = false;
  using Cfg = GramCfg<GT, BK>;
  const int nt = (p + GT - 1) / GT;
  const int ntiles = nt * (nt + 1) / 2;
  const bool vec = (ldx % 4 == 0) && (p % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  if (rows) chunk_rows = std::min<int64_t>(chunk_rows, GATHER_MAX_CHUNK);
  chunk_rows = (int64_t)ocm::align_up((size_t)chunk_rows, Cfg::BK);

  // total chunks over all segments (an empty segment owns 0 chunks)
  std::vector<int32_t> cprefix(nseg + 1, 0);
  for (int s = 0; s < nseg; ++s) {
    const int64_t len = seg_offsets[s + 1] - seg_offsets[s];
    cprefix[s + 1] = cprefix[s] + (int32_t)((len + chunk_rows - 1) / chunk_rows);
  }
  const int64_t nchunks = cprefix[nseg];
  const size_t part_elems = (size_t)nchunks * ntiles * GT * GT;
  const size_t col_elems = (size_t)nchunks * nt * GT;
  void* wsp = ocm::workspace(ctx, part_elems * sizeof(float) + col_elems * sizeof(double) + 4096, st);
  if (!wsp) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(wsp)};
  float* part = cv.take<float>(part_elems);
  double* colpart = cv.take<double>(col_elems);

  // launch in groups of ≤ MAXSEG segments; chunk ids are global
  for (int s0 = 0; s0 < nseg; s0 += MAXSEG) {
    const int s1 = std::min(nseg, s0 + MAXSEG);
    SegTable tab{};
    tab.nseg = s1 - s0;
    tab.chunk_rows = (int32_t)chunk_rows;
    for (int s = s0; s <= s1; ++s) {
      tab.begin[s - s0] = seg_offsets[s];
      tab.cprefix[s - s0] = cprefix[s] - cprefix[s0];
    }
    const int64_t gchunks = cprefix[s1] - cprefix[s0];
    if (gchunks == 0) continue;
    const int64_t total = gchunks * ntiles;
    OCM_REQUIRE(total < (1LL << 31), "ocm_gram_f32: too many workgroups");
    float* pg = part + (size_t)cprefix[s0] * ntiles * GT * GT;
    double* col_g = colpart + (size_t)cprefix[s0] * nt * GT;
    ocm::TimedRegion tr(ctx, OCM_KERNEL_GRAM, st);
    dim3 grid((unsigned)total), blk(Cfg::THREADS);
#define OCM_GRAM_LAUNCH(V_, G_)                                                                                    \
  hipLaunchKernelGGL((k_gram<GT, BK, V_, G_>), grid, blk, 0, st, X, ldx, rows, p, shift, tab, nt, ntiles, (int)total, \
                     pg, col_g)
    if (split3) {
      if (rows)
        hipLaunchKernelGGL(k_gram3<true>, grid, dim3(G3THREADS), 0, st, X, ldx, rows, p, shift, tab, nt, ntiles,
                           (int)total, pg, col_g);
      else
        hipLaunchKernelGGL(k_gram3<false>, grid, dim3(G3THREADS), 0, st, X, ldx, rows, p, shift, tab, nt, ntiles,
                           (int)total, pg, col_g);
    } else if (rows) {
      if (vec) OCM_GRAM_LAUNCH(true, true); else OCM_GRAM_LAUNCH(false, true);
    } else {
      if (vec) OCM_GRAM_LAUNCH(true, false); else OCM_GRAM_LAUNCH(false, false);
    }
#undef OCM_GRAM_LAUNCH
    OCM_CHECK_LAUNCH("k_gram");
  }
  for (int s = 0; s < nseg; ++s) {
    double* Gs = G_out + (size_t)s * p * p;
    double* cs = colsum_out + (size_t)s * p;
    if (cprefix[s + 1] == cprefix[s]) {
      OCM_HIP(hipMemsetAsync(Gs, 0, (size_t)p * p * sizeof(double), st));
      OCM_HIP(hipMemsetAsync(cs, 0, (size_t)p * sizeof(double), st));
      continue;
    }
    dim3 g((GT * GT / 4 + 255) / 256, ntiles);
    hipLaunchKernelGGL(k_gram_reduce<GT>, g, dim3(256), 0, st, part, colpart, nt, ntiles, p, cprefix[s],
                       cprefix[s + 1], Gs, cs);
    OCM_CHECK_LAUNCH("k_gram_reduce");
  }
  return OCM_OK;
}

// i8×3 path: thresholds → quantise (one read of X, outlier screen) →
// integer-MFMA Gram → f64 reduce → (marked rows only) exact fix-up.
// Returns OCM_OK, or 1 when more than n/8 rows had values screened out: the
// caller then recomputes the Gram on the bf16×3 path.
int gram_impl8(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
               const float* shift, const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out,
               hipStream_t st, int64_t chunk_rows, bool k32, const PrepArgs& pa = PrepArgs{},
               bool unguarded = false, float* xout = nullptr, int64_t ldo = 0, const float* tr_O = nullptr,
               double* tr_part = nullptr) {
  // unguarded: an internal Gram (the eigensolver's θ3 of the off-diagonal
  // deflated covariance) — no outlier screen (no thresholds, nothing marked,
  // no read-back, no guard buffers to initialise), shift may be nullptr (zero),
  // not timed, ctx->last_gram_marks left alone.  tr_O (unguarded, one
  // segment): no G at all — tr_part[ntiles · 16] = the partials of
  // Σ_ij tr_O_ij G_ij (k_gram_trace)
  const bool prep = pa.w > 0 || pa.snv;
  const int P8 = (int)ocm::align_up((size_t)p, Q8T);
  const int nt = P8 / Q8T;
  const int ntiles = nt * (nt + 1) / 2;
  if (chunk_rows <= 0) {
    // enough workgroups to fill the chip (≥ 4 per CU), ≤ 4096 rows per chunk
    const int64_t want = std::max<int64_t>(1, (4LL * ctx->num_cus + ntiles - 1) / ntiles);
    chunk_rows = std::min<int64_t>(4096, (n + want - 1) / want);
  }
  // whole scale blocks (the Gram kernels' loop body)
  chunk_rows = std::max<int64_t>(Q8BLK, (int64_t)ocm::align_up((size_t)chunk_rows, Q8BLK));
  std::vector<int32_t> cprefix(nseg + 1, 0);
  for (int s = 0; s < nseg; ++s) {
    const int64_t len = seg_offsets[s + 1] - seg_offsets[s];
    cprefix[s + 1] = cprefix[s] + (int32_t)((len + chunk_rows - 1) / chunk_rows);
  }
  const int64_t nchunks = cprefix[nseg];
  const int nblk = (int)(chunk_rows / Q8BLK);
  const size_t plane = (size_t)nchunks * chunk_rows * P8;  // 1 B per digit
  const size_t scale_elems = (size_t)nchunks * nblk * P8;
  const size_t col_elems = (size_t)nchunks * nblk * P8;  // per scale block
  const size_t part_elems = (size_t)nchunks * ntiles * Q8T * Q8T;
  // guard buffers
  const int ngrp = P8 / Q8GROUP, fw = (ngrp + 31) / 32;
  const int64_t nsamp = std::min<int64_t>(n, 4096);
  const int nsplit = (int)std::min<int64_t>((nsamp + 255) / 256, 16);
  const int64_t rps = (nsamp + nsplit - 1) / nsplit;
  const int nfblk = (int)((n + FLAG_BLK - 1) / FLAG_BLK);
  const size_t guard_bytes = (size_t)P8 * 4 + (size_t)n * fw * 4 + (size_t)p * QX_BINS * 4 + (size_t)nfblk * 4 +
                             (size_t)n * 8 + 16 * 256;
  void* wsp = ocm::workspace(ctx, 3 * plane + scale_elems * 4 + col_elems * 8 + part_elems * 4 + guard_bytes +
                                      4 * 4096, st);
  if (!wsp) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(wsp)};
  char* digits = cv.take<char>(3 * plane);
  float* scale = cv.take<float>(scale_elems);
  double* colpart = cv.take<double>(col_elems);
  float* part = cv.take<float>(part_elems);
  float* thr = cv.take<float>(P8);
  uint32_t* flags = cv.take<uint32_t>((size_t)n * fw);
  uint32_t* xhist = cv.take<uint32_t>((size_t)p * QX_BINS);
  uint32_t* fcnt = cv.take<uint32_t>(nfblk);
  int64_t* flist = cv.take<int64_t>(n);
  uint32_t* counters = cv.take<uint32_t>(4);  // [0] marks, [1] listed rows
  auto* host = static_cast<uint32_t*>(ocm::host_staging(ctx, 64));
  if (!host) return OCM_ERR_NOMEM;

  // the guard's buffers in one launch (three memsets cost ≈ 5 µs each plus
  // their gaps): row flags and counters zero, then the thresholds +inf
  // (unguarded) or the exponent histogram zero
  if (!unguarded) {
    const size_t nf = (size_t)n * fw, third = (size_t)p * QX_BINS;
    const size_t tot = nf + 4 + third;
    hipLaunchKernelGGL(k_guard_init, dim3((unsigned)std::min<size_t>((tot + 255) / 256, 4096)), dim3(256), 0, st,
                       flags, nf, counters, xhist, third, 0u);
    OCM_CHECK_LAUNCH("k_guard_init");
  }
  if (!unguarded) {
    hipLaunchKernelGGL(k_colexp_hist, dim3((p + 63) / 64, nsplit), dim3(256), 0, st, X, ldx, rows, nsamp, p, shift,
                       rps, xhist, pa);
    hipLaunchKernelGGL(k_q8_colmed, dim3((p + 3) / 4), dim3(256), 0, st, xhist, nsamp, p, thr);
    hipLaunchKernelGGL(k_q8_thresholds, dim3(1), dim3(1024), 0, st, p, P8, thr);
    OCM_CHECK_LAUNCH("k_q8_thresholds");
  }

  // all quantiser launches first, then the mark count is read back while the
  // Gram runs
  std::vector<SegTable> tabs;
  std::vector<int> tab_s0;
  for (int s0 = 0; s0 < nseg; s0 += MAXSEG) {
    const int s1 = std::min(nseg, s0 + MAXSEG);
    SegTable tab{};
    tab.nseg = s1 - s0;
    tab.chunk_rows = (int32_t)chunk_rows;
    for (int s = s0; s <= s1; ++s) {
      tab.begin[s - s0] = seg_offsets[s];
      tab.cprefix[s - s0] = cprefix[s] - cprefix[s0];
    }
    const int64_t gchunks = cprefix[s1] - cprefix[s0];
    if (gchunks == 0) continue;
    OCM_REQUIRE(gchunks * ntiles < (1LL << 31) && gchunks < 65536 * 1024LL, "ocm_gram_f32: too many workgroups");
    tabs.push_back(tab);
    tab_s0.push_back(s0);
  }
  auto plan_for = [&](int s0) {
    Q8Plan q{};
    q.digits = digits + (size_t)cprefix[s0] * chunk_rows * P8;
    q.plane = plane;
    q.scale = scale + (size_t)cprefix[s0] * nblk * P8;
    q.P8 = P8;
    q.nblk = nblk;
    q.thr = unguarded ? nullptr : thr;
    q.flags = flags;
    q.fw = fw;
    q.nmark = counters;
    return q;
  };
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  OCM_HIP(hipStreamIsCapturing(st, &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  // k_gram8e's block order and wave sync: tile-aligned workgroups with a
  // barrier every two stages (437 TF against 417 for the packed walk without
  // barriers, r03s).  The product library launches only that variant; the
  // A/B selectors (OCM_GRAM8_ORDER = packed | aligned | sync1 | front | sync4
  // | sync3, OCM_GRAM8_XCD, OCM_GRAM8_PIECES, OCM_Q8_CG) exist only in
  // `make exp` builds (OCM_EXP_SELECTORS), which the product never loads.
  int order = 3;
  bool no_remap = false;
  int pieces = 1;
  int qcg = 1;  // column groups per quantiser workgroup
#ifdef OCM_EXP_SELECTORS
  const char* ord = getenv("OCM_GRAM8_ORDER");
  if (ord && !strcmp(ord, "packed")) order = 0;
  if (ord && !strcmp(ord, "aligned")) order = 1;
  if (ord && !strcmp(ord, "sync1")) order = 2;
  if (ord && !strcmp(ord, "front")) order = 6;
  if (ord && !strcmp(ord, "sync4")) order = 7;
  if (ord && !strcmp(ord, "sync3")) order = 8;
  const char* xr = getenv("OCM_GRAM8_XCD");  // "0": no XCD remap (A/B)
  no_remap = xr && !strcmp(xr, "0");
#ifdef OCM_G8_LDS
  if (ord && !strcmp(ord, "lds")) order = 4;
  if (ord && !strcmp(ord, "lds32")) order = 5;
#endif
  // Quantiser / Gram overlap (measured: no gain): the chunks are
  // cut into `pieces` ranges; the quantiser of range i+1 runs on a side stream
  // while the Gram of range i runs on the launch stream.
  if (const char* pv = getenv("OCM_GRAM8_PIECES")) pieces = std::max(1, atoi(pv));
  if (const char* qv = getenv("OCM_Q8_CG")) qcg = atoi(qv);
#endif
  if (capturing || k32 || unguarded || tabs.size() != 1) pieces = 1;
  if (pieces > 1) {
    const int64_t gch = cprefix[tab_s0[0] + tabs[0].nseg] - cprefix[tab_s0[0]];
    pieces = (int)std::min<int64_t>(pieces, gch / 2);
    if (pieces < 2) pieces = 1;
  }
  hipStream_t qs = st;  // the quantiser's stream
  if (rows || (qcg != 2 && qcg != 4)) qcg = 1;
  std::vector<hipEvent_t> qev;
  if (pieces > 1) {
    if (!ctx->side) OCM_HIP(hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking));
    qs = ctx->side;
    while ((int)ctx->fork_ev.size() < pieces + 1) {
      hipEvent_t e;
      OCM_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
      ctx->fork_ev.push_back(e);
    }
    qev.assign(ctx->fork_ev.begin(), ctx->fork_ev.begin() + pieces + 1);
    OCM_HIP(hipEventRecord(qev[pieces], st));  // everything queued before this call
    OCM_HIP(hipStreamWaitEvent(qs, qev[pieces], 0));
  }
  const int nblocks = 4 * ntiles - nt, nwg = (nblocks + 3) / 4;
  auto quantise = [&](size_t t, int64_t c0, int64_t c1) {
    const int s0 = tab_s0[t];
    const Q8Plan q = plan_for(s0);
    double* col_g = colpart + (size_t)cprefix[s0] * nblk * P8;
    const int cgw = qcg;  // column groups per quantiser workgroup (P8 / 32 is a multiple of 4)
    dim3 gq((unsigned)((c1 - c0) * nblk * cgw), (unsigned)(P8 / Q8QC / cgw));
    ocm::TimedRegion tq(ctx, OCM_KERNEL_QUANT, qs, !unguarded);
    if (prep) {
      const int ncg = P8 / Q8QC;
      const dim3 gp((unsigned)((c1 - c0) * nblk * ncg));
#define Q8P_LAUNCH(G_, H_, W_)                                                                                \
  hipLaunchKernelGGL((k_q8_quant_prep<G_, H_, W_>), gp, dim3(Q8QT), 0, qs, X, ldx, rows, p, shift, tabs[t], q, \
                     col_g, (int)(c0 * nblk), ncg, pa, xout, ldo)
      if (pa.h == 0) {
        if (rows) Q8P_LAUNCH(true, 0, false); else if (xout) Q8P_LAUNCH(false, 0, true); else Q8P_LAUNCH(false, 0, false);
      } else if (pa.h == 2) {
        if (rows) Q8P_LAUNCH(true, 2, false); else if (xout) Q8P_LAUNCH(false, 2, true); else Q8P_LAUNCH(false, 2, false);
      } else {
        if (rows) Q8P_LAUNCH(true, 7, false); else if (xout) Q8P_LAUNCH(false, 7, true); else Q8P_LAUNCH(false, 7, false);
      }
#undef Q8P_LAUNCH
    } else if (rows)
      hipLaunchKernelGGL(k_q8_quant<true>, gq, dim3(Q8QT), 0, qs, X, ldx, rows, p, shift, tabs[t], q, col_g,
                         (int)(c0 * nblk));
#ifdef OCM_EXP_SELECTORS
    else if (cgw == 4)
      hipLaunchKernelGGL((k_q8_quant<false, 4>), gq, dim3(Q8QT), 0, qs, X, ldx, rows, p, shift, tabs[t], q, col_g,
                         (int)(c0 * nblk));
    else if (cgw == 2)
      hipLaunchKernelGGL((k_q8_quant<false, 2>), gq, dim3(Q8QT), 0, qs, X, ldx, rows, p, shift, tabs[t], q, col_g,
                         (int)(c0 * nblk));
#endif
    else
      hipLaunchKernelGGL(k_q8_quant<false>, gq, dim3(Q8QT), 0, qs, X, ldx, rows, p, shift, tabs[t], q, col_g,
                         (int)(c0 * nblk));
  };
  auto gram = [&](size_t t, int64_t c0, int64_t c1) {
    const int s0 = tab_s0[t];
    const int64_t total = (c1 - c0) * nwg;
    const Q8Plan q = plan_for(s0);
    float* pg = part + (size_t)cprefix[s0] * ntiles * Q8T * Q8T;
    ocm::TimedRegion tr(ctx, OCM_KERNEL_GRAM, st, !unguarded);
#define G8E_LAUNCH(A_, S_)                                                                                   \
  hipLaunchKernelGGL((k_gram8e<A_, S_>), dim3((unsigned)total), dim3(256), 0, st, q, tabs[t], nt, ntiles, (int)total, \
                     nwg, nblocks, pg, (no_remap && c0 == 0) ? -1 : (int)c0)
#define G8E_LAUNCH3(A_, S_, F_)                                                                                      \
  hipLaunchKernelGGL((k_gram8e<A_, S_, F_>), dim3((unsigned)total), dim3(256), 0, st, q, tabs[t], nt, ntiles,         \
                     (int)total, nwg, nblocks, pg, (int)c0)
    if (tr_O && !k32 && order == 3)
      hipLaunchKernelGGL((k_gram8e<true, 2, false, true>), dim3((unsigned)total), dim3(256), 0, st, q, tabs[t], nt,
                         ntiles, (int)total, nwg, nblocks, pg, (int)c0);
    else if (!k32 && order == 3) G8E_LAUNCH(true, 2);
#ifdef OCM_EXP_SELECTORS
    else if (!k32 && order == 0) G8E_LAUNCH(false, 0);
    else if (!k32 && order == 1) G8E_LAUNCH(true, 0);
    else if (!k32 && order == 2) G8E_LAUNCH(true, 1);
    else if (!k32 && order == 6) G8E_LAUNCH3(true, 2, true);
    else if (!k32 && order == 7) G8E_LAUNCH(true, 4);
    else if (!k32 && order == 8) G8E_LAUNCH(true, 3);
#endif
#undef G8E_LAUNCH
#undef G8E_LAUNCH3
#ifdef OCM_G8_LDS
    else if (!k32 && order >= 4 && order <= 5) {
      const int64_t total_x = (c1 - c0) * ntiles;
      if (order == 4)
        hipLaunchKernelGGL(k_gram8x, dim3((unsigned)total_x), dim3(256), 0, st, q, tabs[t], nt, ntiles, (int)total_x,
                           pg);
      else
        hipLaunchKernelGGL(k_gram8s, dim3((unsigned)total_x), dim3(256), 0, st, q, tabs[t], nt, ntiles, (int)total_x,
                           pg);
    }
#endif
    else
      hipLaunchKernelGGL(k_gram8d, dim3((unsigned)total), dim3(256), 0, st, q, tabs[t], nt, ntiles, (int)total, nwg,
                         nblocks, pg);
  };
  // all quantiser launches first (or, with pieces, range by range on the side
  // stream), then the mark count is read back while the Gram runs
  hipEvent_t ev = nullptr;
  const bool readback = !capturing && !unguarded;
  if (readback) OCM_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  if (pieces == 1) {
    for (size_t t = 0; t < tabs.size(); ++t) quantise(t, 0, cprefix[tab_s0[t] + tabs[t].nseg] - cprefix[tab_s0[t]]);
    OCM_CHECK_LAUNCH("k_q8_quant");
    if (readback) {
      OCM_HIP(hipMemcpyAsync(host, counters, 4, hipMemcpyDeviceToHost, st));
      OCM_HIP(hipEventRecord(ev, st));
    }
    for (size_t t = 0; t < tabs.size(); ++t) gram(t, 0, cprefix[tab_s0[t] + tabs[t].nseg] - cprefix[tab_s0[t]]);
    OCM_CHECK_LAUNCH("k_gram8d/8e");
  } else {
    const int64_t gch = cprefix[tab_s0[0] + tabs[0].nseg] - cprefix[tab_s0[0]];
    std::vector<int64_t> cut(pieces + 1);
    for (int i = 0; i <= pieces; ++i) cut[i] = gch * i / pieces;
    for (int i = 0; i < pieces; ++i) {
      quantise(0, cut[i], cut[i + 1]);
      OCM_HIP(hipEventRecord(qev[i], qs));
    }
    OCM_CHECK_LAUNCH("k_q8_quant");
    OCM_HIP(hipMemcpyAsync(host, counters, 4, hipMemcpyDeviceToHost, qs));
    OCM_HIP(hipEventRecord(ev, qs));
    for (int i = 0; i < pieces; ++i) {
      OCM_HIP(hipStreamWaitEvent(st, qev[i], 0));
      gram(0, cut[i], cut[i + 1]);
    }
    OCM_CHECK_LAUNCH("k_gram8e");
    OCM_HIP(hipStreamWaitEvent(st, ev, 0));  // the read-back is done before the workspace is reused
  }
  if (tr_O) {
    hipLaunchKernelGGL(k_gram_trace<Q8T>, dim3(Q8T * Q8T / 4 / 256, ntiles), dim3(256), 0, st, part, nt, ntiles, p, 0,
                       cprefix[1], tr_O, tr_part);
    OCM_CHECK_LAUNCH("k_gram_trace");
    return OCM_OK;
  }
  for (int s = 0; s < nseg; ++s) {
    double* Gs = G_out + (size_t)s * p * p;
    double* cs = colsum_out + (size_t)s * p;
    if (cprefix[s + 1] == cprefix[s]) {
      OCM_HIP(hipMemsetAsync(Gs, 0, (size_t)p * p * sizeof(double), st));
      OCM_HIP(hipMemsetAsync(cs, 0, (size_t)p * sizeof(double), st));
      continue;
    }
    dim3 g((Q8T * Q8T / 4 + 255) / 256, ntiles);
    // colsum comes from k_colblk_sum (cmul = 0: the reduce skips it)
    hipLaunchKernelGGL(k_gram_reduce<Q8T>, g, dim3(256), 0, st, part, colpart, nt, ntiles, p, cprefix[s],
                       cprefix[s + 1], Gs, cs, 0);
    hipLaunchKernelGGL(k_colblk_sum, dim3(P8 / 16), dim3(256), 0, st, colpart, (int64_t)cprefix[s] * nblk,
                       (int64_t)cprefix[s + 1] * nblk, P8, p, cs);
    OCM_CHECK_LAUNCH("k_colblk_sum");
    OCM_CHECK_LAUNCH("k_gram_reduce");
  }
  if (unguarded) return OCM_OK;  // thresholds +inf: nothing was marked
  if (!capturing) {  // capturing: the fix-up runs on device-side counts
    const hipError_t e = hipEventSynchronize(ev);
    (void)hipEventDestroy(ev);
    if (e != hipSuccess) return ocm::fail(OCM_ERR_HIP, std::string("gram mark read-back: ") + hipGetErrorString(e));
    ctx->last_gram_marks = host[0];
    if (host[0] == 0) return OCM_OK;
  }
  hipLaunchKernelGGL(k_flag_count, dim3(nfblk), dim3(256), 0, st, flags, fw, n, fcnt);
  hipLaunchKernelGGL(k_flag_emit, dim3(nfblk), dim3(256), 0, st, flags, fw, n, fcnt, nfblk, flist, counters + 1);
  OCM_CHECK_LAUNCH("k_flag_emit");
  if (!capturing) {
    // the fix-up costs p²/2 fp64 FMAs per marked row: past n/8 rows the
    // bf16×3 Gram of everything is cheaper
    OCM_HIP(hipMemcpyAsync(host + 1, counters + 1, 4, hipMemcpyDeviceToHost, st));
    OCM_HIP(hipStreamSynchronize(st));
    if ((int64_t)host[1] > n / 8) return 1;
  }
  const int nt64 = (p + FX_T - 1) / FX_T;
  for (int s0 = 0; s0 < nseg; s0 += MAXSEG) {
    const int s1 = std::min(nseg, s0 + MAXSEG);
    FixSeg fs{};
    fs.nseg = s1 - s0;
    for (int s = s0; s <= s1; ++s) fs.begin[s - s0] = seg_offsets[s];
    hipLaunchKernelGGL(k_gram_fixup, dim3(nt64 * (nt64 + 1) / 2, s1 - s0), dim3(256), 0, st, X, ldx, rows, p, shift,
                       fs, flist, counters + 1, flags, fw, nt64, G_out + (size_t)s0 * p * p, pa);
  }
  OCM_CHECK_LAUNCH("k_gram_fixup");
  return OCM_OK;
}

// The Gram of a lazy view (ocm_prep) on the paths without a fused load:
// the preprocessed rows go to a temporary device buffer (processed-row
// order, so the gather list is consumed here) and the plain dispatch runs on it.
int gram_dispatch(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                  const float* shift, const int64_t* seg_offsets, int32_t nseg, int32_t mode, int64_t chunk_rows,
                  double* G_out, double* colsum_out, hipStream_t st);

int gram_materialised(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                      const float* shift, const int64_t* seg_offsets, int32_t nseg, int32_t mode, int64_t chunk_rows,
                      const PrepArgs& pa, double* G_out, double* colsum_out, hipStream_t st) {
  float* Y = nullptr;
  OCM_HIP(hipMallocAsync(reinterpret_cast<void**>(&Y), (size_t)n * p * sizeof(float), st));
  ++ctx->prep_materialised;
  int rc = ocm::prep_apply(ctx, X, ldx, rows, n, p, pa, Y, p, st);
  if (rc == OCM_OK)
    rc = gram_dispatch(ctx, Y, p, nullptr, n, p, shift, seg_offsets, nseg, mode, chunk_rows, G_out, colsum_out, st);
  const hipError_t e = hipFreeAsync(Y, st);
  if (rc == OCM_OK && e != hipSuccess) return ocm::fail(OCM_ERR_HIP, std::string("hipFreeAsync: ") + hipGetErrorString(e));
  return rc;
}

bool prep_fused_gram(const float* X, int64_t ldx, int32_t p, int32_t mode, const PrepArgs& pa) {
  return (mode == OCM_GRAM_I8X3) && p > SMALL_P && p % 4 == 0 && ldx % 4 == 0 &&
         (reinterpret_cast<uintptr_t>(X) & 15) == 0 && pa.fused_form() && p >= pa.w + 8 &&
         (int64_t)Q8BLK * ldx * 4 < (1LL << 31) &&
         // the right edge rows' samples inside the last column group's row image
         (pa.h < 7 || p % Q8QC != 4);
}

int gram_dispatch(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                  const float* shift, const int64_t* seg_offsets, int32_t nseg, int32_t mode, int64_t chunk_rows,
                  double* G_out, double* colsum_out, hipStream_t st) {
  if (p <= SMALL_P) return gram_small(ctx, X, ldx, rows, p, shift, seg_offsets, nseg, G_out, colsum_out, st);
  if (mode == OCM_GRAM_I8X3 || mode == OCM_GRAM_I8X3_K32) {
    const int rc = gram_impl8(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, G_out, colsum_out, st, chunk_rows,
                              mode == OCM_GRAM_I8X3_K32);
    if (rc != 1) return rc;
    mode = OCM_GRAM_BF16X3;  // too many screened rows: recompute on the exact bf16×3 split
  }
  // f32 accumulation length per partial: short chunks keep the tiles of one
  // chunk co-resident on an XCD (L2 reuse) and the tail short; the partial
  // buffer is capped at 512 chunks (≈4.7 GB for p = 2048).
  const int64_t cr = chunk_rows > 0 ? std::max<int64_t>(64, chunk_rows) : std::max<int64_t>(2048, (n + 511) / 512);
  if (mode == OCM_GRAM_BF16X3)
    return gram_impl<256, 32>(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, G_out, colsum_out, st, cr, true);
  if (p > 128)
    return gram_impl<256, 32>(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, G_out, colsum_out, st, cr);
  return gram_impl<128, 32>(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, G_out, colsum_out, st, cr);
}

}  // namespace

namespace ocm {
int trace_gram_rows_i8(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t n, int p, const float* O, double* tr_part,
                       int* ntr, hipStream_t st) {
  const int nt = (int)(ocm::align_up((size_t)p, Q8T) / Q8T);
  *ntr = nt * (nt + 1) / 2 * (Q8T * Q8T / 4 / 256);
  if (p <= SMALL_P) return OCM_ERR_ARG;  // the caller takes the G path
  const int64_t seg[2] = {0, n};
  // as few chunks as keep one round of workgroups (chunks × tiles ≤ CUs; one
  // at p = 2048): the SKIP instantiation stops each chunk at its last row
  const int64_t nch = std::max<int64_t>(1, std::min<int64_t>(ctx->num_cus / std::max(1, nt * (nt + 1) / 2),
                                                             (n + Q8BLK - 1) / Q8BLK));
  const int64_t chunk = (int64_t)ocm::align_up((size_t)((n + nch - 1) / nch), Q8BLK);
  return gram_impl8(ctx, X, ldx, nullptr, n, p, nullptr, seg, 1, nullptr, nullptr, st, chunk, false, PrepArgs{},
                    true, nullptr, 0, O, tr_part);
}
}  // namespace ocm

extern "C" {

int ocm_colmean_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                    double* mean_out, void* stream) {
  OCM_REQUIRE(ctx && X && mean_out, "ocm_colmean_f32: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p, "ocm_colmean_f32: bad shape");
  hipStream_t st = (hipStream_t)stream;
  // short row splits: the shift sample (4096 rows) spreads over ≥ 1024 workgroups
  const int64_t per = 32;
  const int nsplit = (int)std::min<int64_t>((n + per - 1) / per, 4096);
  const int64_t rps = (n + nsplit - 1) / nsplit;
  auto* part = static_cast<double*>(ocm::workspace(ctx, (size_t)nsplit * p * sizeof(double), st));
  if (!part) return OCM_ERR_NOMEM;
  dim3 g1((p + 255) / 256, nsplit);
  hipLaunchKernelGGL(k_colsum_part, g1, dim3(256), 0, st, X, ldx, rows, n, p, rps, part, PrepArgs{});
  OCM_CHECK_LAUNCH("k_colsum_part");
  hipLaunchKernelGGL(k_colsum_final, dim3((p + 255) / 256), dim3(256), 0, st, part, nsplit, p, 1.0 / (double)n,
                     mean_out);
  OCM_CHECK_LAUNCH("k_colsum_final");
  return OCM_OK;
}

int ocm_gram_f32_ex(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                    const float* shift, const int64_t* seg_offsets, int32_t nseg, int32_t mode, int64_t chunk_rows,
                    double* G_out, double* colsum_out, void* stream) {
  OCM_REQUIRE(ctx && X && shift && seg_offsets && G_out && colsum_out, "ocm_gram_f32: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p && nseg > 0, "ocm_gram_f32: bad shape");
  OCM_REQUIRE(seg_offsets[0] == 0 && seg_offsets[nseg] == n, "ocm_gram_f32: seg_offsets must span [0, n]");
  OCM_REQUIRE(mode == OCM_GRAM_I8X3 || mode == OCM_GRAM_F32 || mode == OCM_GRAM_BF16X3 || mode == OCM_GRAM_I8X3_K32,
              "ocm_gram_f32: bad mode");
  for (int s = 0; s < nseg; ++s)
    OCM_REQUIRE(seg_offsets[s + 1] >= seg_offsets[s], "ocm_gram_f32: seg_offsets not ascending");
  return gram_dispatch(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, mode, chunk_rows, G_out, colsum_out,
                       (hipStream_t)stream);
}

int ocm_gram_f32_prep(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                      const float* shift, const int64_t* seg_offsets, int32_t nseg, int32_t mode,
                      int64_t chunk_rows, const ocm_prep* prep, double* G_out, double* colsum_out, void* stream) {
  OCM_REQUIRE(ctx && X && shift && seg_offsets && G_out && colsum_out, "ocm_gram_f32_prep: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p && nseg > 0, "ocm_gram_f32_prep: bad shape");
  OCM_REQUIRE(seg_offsets[0] == 0 && seg_offsets[nseg] == n, "ocm_gram_f32_prep: seg_offsets must span [0, n]");
  OCM_REQUIRE(mode == OCM_GRAM_I8X3 || mode == OCM_GRAM_F32 || mode == OCM_GRAM_BF16X3 || mode == OCM_GRAM_I8X3_K32,
              "ocm_gram_f32_prep: bad mode");
  for (int s = 0; s < nseg; ++s)
    OCM_REQUIRE(seg_offsets[s + 1] >= seg_offsets[s], "ocm_gram_f32_prep: seg_offsets not ascending");
  if (int rc = ocm::check_prep(prep, p, "ocm_gram_f32_prep")) return rc;
  const PrepArgs pa = ocm::prep_args(prep);
  hipStream_t st = (hipStream_t)stream;
  if (prep_fused_gram(X, ldx, p, mode, pa)) {
    const int rc = gram_impl8(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, G_out, colsum_out, st, chunk_rows,
                              false, pa);
    if (rc != 1) return rc;
    mode = OCM_GRAM_BF16X3;  // too many screened rows: the exact split on the materialised rows
  }
  return gram_materialised(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, mode, chunk_rows, pa, G_out,
                           colsum_out, st);
}

int ocm_gram_f32_prep_write(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t n, int32_t p, const float* shift,
                            const int64_t* seg_offsets, int32_t nseg, int64_t chunk_rows, const ocm_prep* prep,
                            double* G_out, double* colsum_out, float* xout, int64_t ldo, void* stream) {
  OCM_REQUIRE(ctx && X && shift && seg_offsets && G_out && colsum_out && xout,
              "ocm_gram_f32_prep_write: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p && ldo >= p && nseg > 0, "ocm_gram_f32_prep_write: bad shape");
  OCM_REQUIRE(seg_offsets[0] == 0 && seg_offsets[nseg] == n, "ocm_gram_f32_prep_write: seg_offsets must span [0, n]");
  for (int s = 0; s < nseg; ++s)
    OCM_REQUIRE(seg_offsets[s + 1] >= seg_offsets[s], "ocm_gram_f32_prep_write: seg_offsets not ascending");
  if (int rc = ocm::check_prep(prep, p, "ocm_gram_f32_prep_write")) return rc;
  const PrepArgs pa = ocm::prep_args(prep);
  hipStream_t st = (hipStream_t)stream;
  const bool wr_ok = ldo % 4 == 0 && (reinterpret_cast<uintptr_t>(xout) & 15) == 0 &&
                     (int64_t)Q8BLK * ldo * 4 < (1LL << 31);  // the store descriptor's 32-bit offsets
  if (wr_ok && prep_fused_gram(X, ldx, p, OCM_GRAM_I8X3, pa)) {
    const int rc = gram_impl8(ctx, X, ldx, nullptr, n, p, shift, seg_offsets, nseg, G_out, colsum_out, st, chunk_rows,
                              false, pa, false, xout, ldo);
    if (rc != 1) return rc;
    // too many screened rows: the quantiser has written every row, so the
    // exact split runs on X′
    return gram_dispatch(ctx, xout, ldo, nullptr, n, p, shift, seg_offsets, nseg, OCM_GRAM_BF16X3, chunk_rows, G_out,
                         colsum_out, st);
  }
  // no fused quantiser for this shape or transform: the eager pass into xout
  if (int rc = ocm::prep_apply(ctx, X, ldx, nullptr, n, p, pa, xout, ldo, st)) return rc;
  return gram_dispatch(ctx, xout, ldo, nullptr, n, p, shift, seg_offsets, nseg, OCM_GRAM_I8X3, chunk_rows, G_out,
                       colsum_out, st);
}

int ocm_colmean_f32_prep(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                         const ocm_prep* prep, double* mean_out, void* stream) {
  OCM_REQUIRE(ctx && X && mean_out, "ocm_colmean_f32_prep: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p, "ocm_colmean_f32_prep: bad shape");
  if (int rc = ocm::check_prep(prep, p, "ocm_colmean_f32_prep")) return rc;
  hipStream_t st = (hipStream_t)stream;
  const int64_t per = 32;
  const int nsplit = (int)std::min<int64_t>((n + per - 1) / per, 4096);
  const int64_t rps = (n + nsplit - 1) / nsplit;
  auto* part = static_cast<double*>(ocm::workspace(ctx, (size_t)nsplit * p * sizeof(double), st));
  if (!part) return OCM_ERR_NOMEM;
  hipLaunchKernelGGL(k_colsum_part, dim3((p + 255) / 256, nsplit), dim3(256), 0, st, X, ldx, rows, n, p, rps, part,
                     ocm::prep_args(prep));
  OCM_CHECK_LAUNCH("k_colsum_part");
  hipLaunchKernelGGL(k_colsum_final, dim3((p + 255) / 256), dim3(256), 0, st, part, nsplit, p, 1.0 / (double)n,
                     mean_out);
  OCM_CHECK_LAUNCH("k_colsum_final");
  return OCM_OK;
}

int ocm_gram_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                 const float* shift, const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out,
                 void* stream) {
  return ocm_gram_f32_ex(ctx, X, ldx, rows, n, p, shift, seg_offsets, nseg, OCM_GRAM_I8X3, 0, G_out, colsum_out,
                         stream);
}

int ocm_gram_last_marks(ocm_ctx* ctx, int64_t* marks_out) {
  OCM_REQUIRE(ctx && marks_out, "ocm_gram_last_marks: NULL argument");
  *marks_out = (int64_t)ctx->last_gram_marks;
  return OCM_OK;
}

int ocm_cov_from_gram(ocm_ctx* ctx, const double* const* G_list, const double* const* colsum_list,
                      const double* coef, int32_t nterm, const float* shift, int64_t n, int32_t p, double* C_out,
                      double* mean_out, void* stream) {
  OCM_REQUIRE(ctx && G_list && colsum_list && coef && shift && C_out && mean_out, "ocm_cov_from_gram: NULL argument");
  OCM_REQUIRE(nterm >= 1 && nterm <= MAXTERM, "ocm_cov_from_gram: 1..8 terms");
  OCM_REQUIRE(n >= 2 && p > 0, "ocm_cov_from_gram: need n >= 2");
  hipStream_t st = (hipStream_t)stream;
  CovTerms tm{};
  tm.nterm = nterm;
  for (int t = 0; t < nterm; ++t) {
    tm.G[t] = G_list[t];
    tm.cs[t] = colsum_list[t];
    tm.coef[t] = coef[t];
  }
  (void)ctx;
  const size_t pp = (size_t)p * p;
  hipLaunchKernelGGL(k_cov, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, tm, shift, p, (double)n, C_out,
                     mean_out);
  OCM_CHECK_LAUNCH("k_cov");
  return OCM_OK;
}

}  // extern "C"
