// K1 — shifted Gram / column sums on FP32 MFMA, and the covariance built
// from it.  Replaces the full SVD of the centred class matrix in
// utils/SIMCA.py:64-66 (sklearn/decomposition/_pca.py:544-584): the SIMCA
// fit needs the eigen-decomposition of C = Σ(x-μ)(x-μ)ᵀ/(n-1), and C is one
// dense contraction over the spectra rows.
//
// Layout: X row-major n×p float32 (spectra × wavelengths).  A workgroup owns
// one 128×128 tile (ti ≤ tj) of G = Σ yᵀy (y = x - shift) over one chunk of
// rows; it streams 32-row × 128-column panels of the two column blocks
// through double-buffered LDS (coalesced 512-B row segments, shift
// subtracted on the way in) and accumulates with v_mfma_f32_32x32x2_f32
// (exact f32 FMA chain).  Every 1024 rows the f32 accumulators are flushed
// into f64 registers, so long chunks keep ≈1e-7 relative error; chunk
// partials are summed in f64 by a second kernel.  Diagonal tiles also
// accumulate the column sums.  Workgroup ids are remapped so that all tiles
// of one row chunk run on one XCD and share its L2.
#include <cstdlib>
#include <string>
#include <vector>

#include "ocm_internal.h"

namespace {

constexpr int GT = 128;       // output tile edge
constexpr int GBK = 32;       // rows per LDS stage
constexpr int GTHREADS = 256; // 4 waves, 2×2 of 64×64
constexpr int GFLUSH = 32;    // stages per f32 -> f64 flush (1024 rows)
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

template <bool VEC>
__device__ __forceinline__ f32x4 load_row4(const float* __restrict__ X, int64_t ldx, int64_t srow, int col, int p) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  const float* src = X + srow * ldx + col;
  if (VEC && col + 3 < p) {
    v = *reinterpret_cast<const f32x4*>(src);
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e)
      if (col + e < p) v[e] = src[e];
  }
  return v;
}

// ACC64: flush the f32 MFMA accumulators into f64 registers every GFLUSH
// stages (long chunks, 1 wave/SIMD); otherwise f32 over the whole (short)
// chunk and f32 partials (≤ 256 registers → 2 workgroups per CU).
template <bool VEC, bool ACC64, typename PT>
__global__ __launch_bounds__(GTHREADS, ACC64 ? 1 : 2) void k_gram(const float* __restrict__ X, int64_t ldx,
                                                       const int64_t* __restrict__ rows, int p,
                                                       const float* __restrict__ shift, SegTable st, int nt,
                                                       int ntiles, int total_wg, PT* __restrict__ part,
                                                       double* __restrict__ colpart) {
  __shared__ __attribute__((aligned(16))) float lds[2][2][GBK][GT];  // [buf][A/B][row][col] 64 KiB

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
  const int nstage = (int)((r1 - r0 + GBK - 1) / GBK);

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int l31 = lane & 31, h = lane >> 5;

  // loader mapping: 32 float4 per 128-col row segment, 8 rows per pass
  const int c4 = tid & 31, rr = tid >> 5;
  f32x4 shA, shB;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const int ca = I + 4 * c4 + e, cb = J + 4 * c4 + e;
    shA[e] = ca < p ? shift[ca] : 0.f;
    shB[e] = cb < p ? shift[cb] : 0.f;
  }

  f32x4 ra[4], rb[4];
  double csum64[4] = {0.0, 0.0, 0.0, 0.0};

  auto gload = [&](int stage) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int64_t g = r0 + (int64_t)stage * GBK + rr + 8 * j;
      f32x4 va = {0.f, 0.f, 0.f, 0.f}, vb = {0.f, 0.f, 0.f, 0.f};
      if (g < r1) {
        const int64_t srow = rows ? rows[g] : g;
        va = load_row4<VEC>(X, ldx, srow, I + 4 * c4, p) - shA;
        if (!diag) vb = load_row4<VEC>(X, ldx, srow, J + 4 * c4, p) - shB;
        // padded columns must stay exactly zero
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if (I + 4 * c4 + e >= p) va[e] = 0.f;
          if (J + 4 * c4 + e >= p) vb[e] = 0.f;
        }
      }
      ra[j] = va;
      rb[j] = vb;
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      *reinterpret_cast<f32x4*>(&lds[buf][0][rr + 8 * j][4 * c4]) = ra[j];
      if (!diag) *reinterpret_cast<f32x4*>(&lds[buf][1][rr + 8 * j][4 * c4]) = rb[j];
      if (diag) {
#pragma unroll
        for (int e = 0; e < 4; ++e) csum64[e] += (double)ra[j][e];
      }
    }
  };

  f32x16 acc[2][2];
  double acc64[2][2][ACC64 ? 16 : 1];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c) {
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][c][r] = 0.f;
#pragma unroll
      for (int r = 0; r < (ACC64 ? 16 : 1); ++r) acc64[a][c][r] = 0.0;
    }

  if (nstage > 0) {
    gload(0);
    sstore(0);
  }
  __syncthreads();
  const int bsel = diag ? 0 : 1;
  int cur = 0;
  for (int stg = 0; stg < nstage; ++stg) {
    if (stg + 1 < nstage) gload(stg + 1);
    const float* As = &lds[cur][0][0][0];
    const float* Bs = &lds[cur][bsel][0][0];
#pragma unroll
    for (int kk = 0; kk < GBK / 2; ++kk) {
      const int krow = (2 * kk + h) * GT;
      const float a0 = As[krow + wm * 64 + l31];
      const float a1 = As[krow + wm * 64 + 32 + l31];
      const float b0 = Bs[krow + wn * 64 + l31];
      const float b1 = Bs[krow + wn * 64 + 32 + l31];
      acc[0][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b0, acc[0][0], 0, 0, 0);
      acc[0][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0, b1, acc[0][1], 0, 0, 0);
      acc[1][0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b0, acc[1][0], 0, 0, 0);
      acc[1][1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1, b1, acc[1][1], 0, 0, 0);
    }
    if (stg + 1 < nstage) sstore(cur ^ 1);
    __syncthreads();
    cur ^= 1;
    if (ACC64 && ((stg + 1) % GFLUSH == 0 || stg + 1 == nstage)) {
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            acc64[a][c][ACC64 ? r : 0] += (double)acc[a][c][r];
            acc[a][c][r] = 0.f;
          }
    }
  }

  // partial tile out: [chunk][tile][GT][GT]
  PT* out = part + ((size_t)chunk * ntiles + tile) * (GT * GT);
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = wm * 64 + a * 32 + (r & 3) + 8 * (r >> 2) + 4 * h;
        const int col = wn * 64 + c * 32 + l31;
        out[row * GT + col] = ACC64 ? (PT)acc64[a][c][ACC64 ? r : 0] : (PT)acc[a][c][r];
      }

  if (diag) {
    // reduce the 8 row groups of each column through LDS (reuse stage buffer)
    __syncthreads();
    double* red = reinterpret_cast<double*>(&lds[0][0][0][0]);  // [8][128]
#pragma unroll
    for (int e = 0; e < 4; ++e) red[rr * GT + 4 * c4 + e] = csum64[e];
    __syncthreads();
    if (tid < GT) {
      double v = 0.0;
#pragma unroll
      for (int g = 0; g < 8; ++g) v += red[g * GT + tid];
      colpart[((size_t)chunk * nt + ti) * GT + tid] = v;
    }
  }
}

// Sum chunk partials of one segment into G (full symmetric) and colsum.
template <typename PT>
__global__ void k_gram_reduce(const PT* __restrict__ part, const double* __restrict__ colpart, int nt,
                              int ntiles, int p, int c0, int c1, double* __restrict__ G, double* __restrict__ colsum) {
  const int tile = blockIdx.y;
  const int e = blockIdx.x * blockDim.x + threadIdx.x;  // element in tile
  int ti, tj;
  tile_coords(tile, nt, ti, tj);
  if (e < GT * GT) {
    const int i = e / GT, j = e % GT;
    const int gi = ti * GT + i, gj = tj * GT + j;
    double v = 0.0;
    for (int c = c0; c < c1; ++c) v += (double)part[((size_t)c * ntiles + tile) * (GT * GT) + e];
    if (gi < p && gj < p) {
      G[(size_t)gi * p + gj] = v;
      if (ti != tj) G[(size_t)gj * p + gi] = v;
    }
  }
  if (ti == tj && e < GT) {
    const int gi = ti * GT + e;
    double v = 0.0;
    for (int c = c0; c < c1; ++c) v += colpart[((size_t)c * nt + ti) * GT + e];
    if (gi < p) colsum[gi] = v;
  }
}

// Column mean over n rows: per (column, row-split) f64 partial sums.
__global__ void k_colsum_part(const float* __restrict__ X, int64_t ldx, const int64_t* __restrict__ rows, int64_t n,
                              int p, int64_t rows_per_split, double* __restrict__ part) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  const int sp = blockIdx.y;
  if (col >= p) return;
  const int64_t a = (int64_t)sp * rows_per_split;
  const int64_t e = min(n, a + rows_per_split);
  double v = 0.0;
  for (int64_t r = a; r < e; ++r) {
    const int64_t sr = rows ? rows[r] : r;
    v += (double)X[sr * ldx + col];
  }
  part[(size_t)sp * p + col] = v;
}

__global__ void k_colsum_final(const double* __restrict__ part, int nsplit, int p, double inv_n,
                               double* __restrict__ mean) {
  const int col = blockIdx.x * blockDim.x + threadIdx.x;
  if (col >= p) return;
  double v = 0.0;
  for (int s = 0; s < nsplit; ++s) v += part[(size_t)s * p + col];
  mean[col] = v * inv_n;
}

constexpr int MAXTERM = 8;
struct CovTerms {
  const double* G[MAXTERM];
  const double* cs[MAXTERM];
  double coef[MAXTERM];
  int nterm;
};

__global__ void k_cov_mean(CovTerms tm, const float* __restrict__ shift, int p, double n,
                           double* __restrict__ dvec, double* __restrict__ mean) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p) return;
  double s = 0.0;
  for (int t = 0; t < tm.nterm; ++t) s += tm.coef[t] * tm.cs[t][i];
  const double d = s / n;
  dvec[i] = d;
  mean[i] = (double)shift[i] + d;
}

__global__ void k_cov(CovTerms tm, const double* __restrict__ dvec, int p, double n, double* __restrict__ C) {
  const size_t e = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (size_t)p * p) return;
  const int i = (int)(e / p), j = (int)(e % p);
  double g = 0.0;
  for (int t = 0; t < tm.nterm; ++t) g += tm.coef[t] * tm.G[t][e];
  C[e] = (g - n * dvec[i] * dvec[j]) / (n - 1.0);
}

}  // namespace

extern "C" {

int ocm_colmean_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                    double* mean_out, void* stream) {
  OCM_REQUIRE(ctx && X && mean_out, "ocm_colmean_f32: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p, "ocm_colmean_f32: bad shape");
  hipStream_t st = (hipStream_t)stream;
  const int64_t per = 256;
  const int nsplit = (int)std::min<int64_t>((n + per - 1) / per, 4096);
  const int64_t rps = (n + nsplit - 1) / nsplit;
  auto* part = static_cast<double*>(ocm::workspace(ctx, (size_t)nsplit * p * sizeof(double), st));
  if (!part) return OCM_ERR_NOMEM;
  dim3 g1((p + 255) / 256, nsplit);
  hipLaunchKernelGGL(k_colsum_part, g1, dim3(256), 0, st, X, ldx, rows, n, p, rps, part);
  OCM_CHECK_LAUNCH("k_colsum_part");
  hipLaunchKernelGGL(k_colsum_final, dim3((p + 255) / 256), dim3(256), 0, st, part, nsplit, p, 1.0 / (double)n,
                     mean_out);
  OCM_CHECK_LAUNCH("k_colsum_final");
  return OCM_OK;
}

int ocm_gram_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t n, int32_t p,
                 const float* shift, const int64_t* seg_offsets, int32_t nseg, double* G_out, double* colsum_out,
                 void* stream) {
  OCM_REQUIRE(ctx && X && shift && seg_offsets && G_out && colsum_out, "ocm_gram_f32: NULL argument");
  OCM_REQUIRE(n > 0 && p > 0 && ldx >= p && nseg > 0, "ocm_gram_f32: bad shape");
  OCM_REQUIRE(seg_offsets[0] == 0 && seg_offsets[nseg] == n, "ocm_gram_f32: seg_offsets must span [0, n]");
  for (int s = 0; s < nseg; ++s)
    OCM_REQUIRE(seg_offsets[s + 1] >= seg_offsets[s], "ocm_gram_f32: seg_offsets not ascending");
  hipStream_t st = (hipStream_t)stream;
  const int nt = (p + GT - 1) / GT;
  const int ntiles = nt * (nt + 1) / 2;
  const bool vec = (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);

  // Variant: "acc64" (f64 flush, long chunks) or "f32" (short chunks, f32
  // partials, 2 WG/CU).  OCM_GRAM_VARIANT / OCM_GRAM_CHUNK override (A/B).
  bool acc64 = false;
  int64_t chunk_rows = 0;
  if (const char* e = std::getenv("OCM_GRAM_VARIANT")) acc64 = std::string(e) == "acc64";
  if (const char* e = std::getenv("OCM_GRAM_CHUNK")) chunk_rows = std::atoll(e);
  if (chunk_rows <= 0) {
    if (acc64) {
      // enough workgroups to fill 256 CUs several times, ≥ 2048 rows
      const int64_t target_wg = (int64_t)ctx->num_cus * 8;
      const int64_t want_chunks = std::max<int64_t>(1, target_wg / ntiles);
      chunk_rows = std::max<int64_t>(2048, (n + want_chunks - 1) / want_chunks);
    } else {
      chunk_rows = 8192;  // f32 accumulation length (≈ 6e-8·√8192 relative per partial)
    }
  }
  chunk_rows = (int64_t)ocm::align_up((size_t)chunk_rows, GBK);
  if (chunk_rows > (1 << 30)) chunk_rows = 1 << 30;

  // total chunks over all segments (an empty segment owns 0 chunks)
  std::vector<int32_t> cprefix(nseg + 1, 0);
  for (int s = 0; s < nseg; ++s) {
    const int64_t len = seg_offsets[s + 1] - seg_offsets[s];
    cprefix[s + 1] = cprefix[s] + (int32_t)((len + chunk_rows - 1) / chunk_rows);
  }
  const int64_t nchunks = cprefix[nseg];
  const size_t part_elems = (size_t)nchunks * ntiles * GT * GT;
  const size_t col_elems = (size_t)nchunks * nt * GT;
  const size_t pbytes = acc64 ? sizeof(double) : sizeof(float);
  void* wsp = ocm::workspace(ctx, part_elems * pbytes + col_elems * sizeof(double) + 4096, st);
  if (!wsp) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(wsp)};
  void* part = acc64 ? (void*)cv.take<double>(part_elems) : (void*)cv.take<float>(part_elems);
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
    const size_t poff = (size_t)cprefix[s0] * ntiles * GT * GT;
    double* col_g = colpart + (size_t)cprefix[s0] * nt * GT;
    ocm::TimedRegion tr(ctx, OCM_KERNEL_GRAM, st);
    dim3 grid((unsigned)total), blk(GTHREADS);
    if (acc64) {
      double* pg = static_cast<double*>(part) + poff;
      if (vec)
        hipLaunchKernelGGL((k_gram<true, true, double>), grid, blk, 0, st, X, ldx, rows, p, shift, tab, nt, ntiles,
                           (int)total, pg, col_g);
      else
        hipLaunchKernelGGL((k_gram<false, true, double>), grid, blk, 0, st, X, ldx, rows, p, shift, tab, nt, ntiles,
                           (int)total, pg, col_g);
    } else {
      float* pg = static_cast<float*>(part) + poff;
      if (vec)
        hipLaunchKernelGGL((k_gram<true, false, float>), grid, blk, 0, st, X, ldx, rows, p, shift, tab, nt, ntiles,
                           (int)total, pg, col_g);
      else
        hipLaunchKernelGGL((k_gram<false, false, float>), grid, blk, 0, st, X, ldx, rows, p, shift, tab, nt, ntiles,
                           (int)total, pg, col_g);
    }
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
    dim3 g((GT * GT + 255) / 256, ntiles);
    if (acc64)
      hipLaunchKernelGGL(k_gram_reduce<double>, g, dim3(256), 0, st, static_cast<const double*>(part), colpart, nt,
                         ntiles, p, cprefix[s], cprefix[s + 1], Gs, cs);
    else
      hipLaunchKernelGGL(k_gram_reduce<float>, g, dim3(256), 0, st, static_cast<const float*>(part), colpart, nt,
                         ntiles, p, cprefix[s], cprefix[s + 1], Gs, cs);
    OCM_CHECK_LAUNCH("k_gram_reduce");
  }
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
  auto* dvec = static_cast<double*>(ocm::workspace(ctx, (size_t)p * sizeof(double), st));
  if (!dvec) return OCM_ERR_NOMEM;
  hipLaunchKernelGGL(k_cov_mean, dim3((p + 255) / 256), dim3(256), 0, st, tm, shift, p, (double)n, dvec, mean_out);
  OCM_CHECK_LAUNCH("k_cov_mean");
  const size_t pp = (size_t)p * p;
  hipLaunchKernelGGL(k_cov, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, tm, dvec, p, (double)n, C_out);
  OCM_CHECK_LAUNCH("k_cov");
  return OCM_OK;
}

}  // extern "C"
