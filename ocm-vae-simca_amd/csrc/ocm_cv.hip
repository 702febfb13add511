// Fold engine kernels for class-wise SIMCA cross-validation
// (utils/CVSIMCA.py:103-269, SURVEY.md §8e "CVSIMCA").
//
// The reference refits a full SIMCA per (param combo, LV, fold) and predicts
// the held-out rows (utils/CVSIMCA.py:179-199).  Here the fold models come
// from ONE Gram pass (per-fold segments, train Gram = total − fold, fp64) and
// ONE eigensolve per fold at LV_max; every LV ≤ LV_max reuses that basis:
//   T²_LV = Σ_{j<LV} t_j² / λ_j,        Q_LV = Q_{LVmax} + Σ_{LV≤j<LVmax} t_j²
// (the leading-LV PCA of the same class matrix is the leading LV of the same
// decomposition, utils/SIMCA.py:64-70).  These kernels turn the LV_max scores
// of a row set into per-LV T²/Q (training rows: limit statistics) and into
// confusion counts for every (LV, limit set) decision at once (test rows).
#include <algorithm>
#include <vector>

#include "ocm_internal.h"

namespace {

constexpr int MAXTERM_C = 8;
constexpr int CV_MAXK = 64;

struct CombineTerms {
  const double* G[MAXTERM_C];
  const double* cs[MAXTERM_C];
  double coef[MAXTERM_C];
  int nterm;
  int accumulate;  // 1: out += Σ coef·G (out is also read), 0: out = Σ coef·G
};

__global__ __launch_bounds__(256) void k_combine(CombineTerms tm, int64_t count, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= count) return;
  double v = tm.accumulate ? out[e] : 0.0;
  for (int t = 0; t < tm.nterm; ++t) v += tm.coef[t] * tm.G[t][e];
  out[e] = v;
}

__global__ __launch_bounds__(256) void k_combine_cs(CombineTerms tm, int p, double* __restrict__ out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= p) return;
  double v = tm.accumulate ? out[e] : 0.0;
  for (int t = 0; t < tm.nterm; ++t) v += tm.coef[t] * tm.cs[t][e];
  out[e] = v;
}

// Row r: t (k floats, row-major m×k), q.  Per LV: T² (f64) and Q (f32), plus
// per-block moment partials {ΣT², ΣT²², ΣQ, ΣQ²} (deterministic reduction).
template <int KB>
__global__ __launch_bounds__(256) void k_cv_prefix(const float* __restrict__ T, int64_t m, int k,
                                                   const float* __restrict__ Q, const double* __restrict__ inv,
                                                   const int* __restrict__ lvs, int nlv, double* __restrict__ T2_out,
                                                   float* __restrict__ Q_out, double* __restrict__ part) {
  __shared__ double sinv[CV_MAXK];
  __shared__ int slv[CV_MAXK];
  __shared__ double sred[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  if (tid < CV_MAXK) sinv[tid] = tid < k ? inv[tid] : 0.0;
  if (tid < nlv) slv[tid] = lvs[tid];
  __syncthreads();
  const int64_t r = (int64_t)blockIdx.x * 256 + tid;
  const bool own = r < m;
  double t2sq[KB];  // t_j² (registers: every index below is compile-time)
  double qres = 0.0;
  const float* tr = T + (own ? r : 0) * k;
#pragma unroll
  for (int j = 0; j < KB; ++j) {
    const double t = (own && j < k) ? (double)tr[j] : 0.0;
    t2sq[j] = t * t;
  }
  if (own) qres = (double)Q[r];
  for (int l = 0; l < nlv; ++l) {
    const int lv = slv[l];
    double t2 = 0.0, q = qres;
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      if (j < lv) t2 += t2sq[j] * sinv[j];
      else q += t2sq[j];  // zero beyond k
    }
    const float qf = (float)q;
    if (own) {
      if (T2_out) T2_out[(int64_t)l * m + r] = t2;
      if (Q_out) Q_out[(int64_t)l * m + r] = qf;
    }
    if (part) {
      const double qd = own ? (double)qf : 0.0;
      double s0 = own ? t2 : 0.0, s1 = own ? t2 * t2 : 0.0, s2 = qd, s3 = qd * qd;
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
      if (tid < 4)
        part[((int64_t)blockIdx.x * nlv + l) * 4 + tid] =
            (sred[0][tid] + sred[1][tid]) + (sred[2][tid] + sred[3][tid]);
      __syncthreads();
    }
  }
}

// stats[l][c] = Σ_blocks part[b][l][c] in a fixed order
__global__ __launch_bounds__(256) void k_cv_prefix_reduce(const double* __restrict__ part, int64_t nblk, int nlv,
                                                          double* __restrict__ stats) {
  const int l = blockIdx.x, c = threadIdx.x >> 6, lane = threadIdx.x & 63;
  double v = 0.0;
  for (int64_t b = lane; b < nblk; b += 64) v += part[(b * nlv + l) * 4 + c];
  v = wave_sum_f64(v);
  if (lane == 0) stats[l * 4 + c] = v;
}

// Confusion counts of every configuration over m rows; rows < m_split are
// part 0 (held-out target fold), the rest part 1 (other-class rows).
// counts[cfg][part][{TP, TN, FP, FN}] as in utils/SIMCA.py:240-245.
template <int KB>
__global__ __launch_bounds__(256) void k_cv_counts(const float* __restrict__ T, int64_t m, int k,
                                                   const float* __restrict__ Q, const double* __restrict__ inv,
                                                   const uint8_t* __restrict__ positive, int64_t m_split,
                                                   const ocm_cv_config* __restrict__ cfg, int ncfg,
                                                   unsigned long long* __restrict__ counts,
                                                   double* __restrict__ accept_out) {
  extern __shared__ unsigned int scount[];  // ncfg × 8
  __shared__ double sinv[CV_MAXK];
  const int tid = threadIdx.x;
  for (int i = tid; i < ncfg * 8; i += 256) scount[i] = 0u;
  if (tid < CV_MAXK) sinv[tid] = tid < k ? inv[tid] : 0.0;
  __syncthreads();
  for (int64_t r = (int64_t)blockIdx.x * 256 + tid; r < m; r += (int64_t)gridDim.x * 256) {
    double t2sq[KB];
    const float* tr = T + r * k;
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      const double t = j < k ? (double)tr[j] : 0.0;
      t2sq[j] = t * t;
    }
    const double qres = (double)Q[r];
    const int part = r < m_split ? 0 : 4;
    const bool pos = positive[r] != 0;
    for (int c = 0; c < ncfg; ++c) {
      const ocm_cv_config cf = cfg[c];
      double t2 = 0.0, q = qres;
#pragma unroll
      for (int j = 0; j < KB; ++j) {
        if (j < cf.lv) t2 += t2sq[j] * sinv[j];
        else q += t2sq[j];
      }
      const double qf = (double)(float)q;
      const bool acc = ocm::dred_of(cf.type, t2 * cf.t2_scale, qf * cf.q_scale) < cf.dlim;
      // TP: accepted positive, TN: rejected negative, FP: accepted negative, FN: rejected positive
      const int slot = acc ? (pos ? 0 : 2) : (pos ? 3 : 1);
      atomicAdd(&scount[c * 8 + part + slot], 1u);
      if (accept_out) accept_out[(int64_t)c * m + r] = acc ? 1.0 : 0.0;
    }
  }
  __syncthreads();
  for (int i = tid; i < ncfg * 8; i += 256)
    if (scount[i]) atomicAdd(&counts[i], (unsigned long long)scount[i]);
}

// {TP, TN, FP, FN} of one class column of the prediction matrix
// (utils/SIMCA.py:238-245): accept[r·stride] ∈ {0, 1}, positive[r] = (y_true == class)
__global__ __launch_bounds__(256) void k_confusion(const double* __restrict__ accept, int64_t m, int64_t stride,
                                                   const uint8_t* __restrict__ positive,
                                                   unsigned long long* __restrict__ counts) {
  __shared__ unsigned int sc[4];
  if (threadIdx.x < 4) sc[threadIdx.x] = 0u;
  __syncthreads();
  unsigned int c[4] = {0u, 0u, 0u, 0u};
  for (int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x; r < m; r += (int64_t)gridDim.x * 256) {
    const double a = accept[r * stride];
    const bool pos = positive[r] != 0;
    if (a == 1.0) ++c[pos ? 0 : 2];       // TP / FP
    else if (a == 0.0) ++c[pos ? 3 : 1];  // FN / TN
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    unsigned int v = c[i];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(&sc[i], v);
  }
  __syncthreads();
  if (threadIdx.x < 4 && sc[threadIdx.x]) atomicAdd(&counts[threadIdx.x], (unsigned long long)sc[threadIdx.x]);
}

int combine_impl(const double* const* G_list, const double* const* colsum_list, const double* coef, int32_t nterm,
                 int32_t p, double* G_out, double* colsum_out, hipStream_t st) {
  const int64_t pp = (int64_t)p * p;
  for (int t0 = 0; t0 < nterm; t0 += MAXTERM_C) {
    CombineTerms tm{};
    tm.nterm = std::min(MAXTERM_C, nterm - t0);
    tm.accumulate = t0 > 0;
    for (int t = 0; t < tm.nterm; ++t) {
      tm.G[t] = G_list[t0 + t];
      tm.cs[t] = colsum_list ? colsum_list[t0 + t] : nullptr;
      tm.coef[t] = coef[t0 + t];
    }
    if (G_out) {
      hipLaunchKernelGGL(k_combine, dim3((unsigned)((pp + 255) / 256)), dim3(256), 0, st, tm, pp, G_out);
      OCM_CHECK_LAUNCH("k_combine");
    }
    if (colsum_out && colsum_list) {
      hipLaunchKernelGGL(k_combine_cs, dim3((p + 255) / 256), dim3(256), 0, st, tm, p, colsum_out);
      OCM_CHECK_LAUNCH("k_combine_cs");
    }
  }
  return OCM_OK;
}

}  // namespace

extern "C" {

int ocm_gram_combine(ocm_ctx* ctx, const double* const* G_list, const double* const* colsum_list,
                     const double* coef, int32_t nterm, int32_t p, double* G_out, double* colsum_out, void* stream) {
  OCM_REQUIRE(ctx && G_list && coef && nterm >= 1 && p >= 1, "ocm_gram_combine: bad argument");
  OCM_REQUIRE(G_out || colsum_out, "ocm_gram_combine: no output");
  for (int t = 0; t < nterm; ++t) {
    OCM_REQUIRE(G_list[t], "ocm_gram_combine: NULL Gram");
    OCM_REQUIRE(G_list[t] != G_out || t == 0, "ocm_gram_combine: G_out may alias only the first term");
  }
  return combine_impl(G_list, colsum_list, coef, nterm, p, G_out, colsum_out, (hipStream_t)stream);
}

int ocm_cv_prefix(ocm_ctx* ctx, const float* T, int64_t m, int32_t k, const float* Q, const double* inv_evals,
                  const int32_t* lvs, int32_t nlv, double* T2_out, float* Q_out, double* stats_out, void* stream) {
  OCM_REQUIRE(ctx && T && Q && inv_evals && lvs, "ocm_cv_prefix: NULL argument");
  OCM_REQUIRE(k >= 1 && k <= CV_MAXK && nlv >= 1 && nlv <= CV_MAXK, "ocm_cv_prefix: 1 <= k, nlv <= 64");
  for (int l = 0; l < nlv; ++l) OCM_REQUIRE(lvs[l] >= 1 && lvs[l] <= k, "ocm_cv_prefix: LV outside [1, k]");
  hipStream_t st = (hipStream_t)stream;
  if (m <= 0) {
    if (stats_out) OCM_HIP(hipMemsetAsync(stats_out, 0, (size_t)nlv * 4 * sizeof(double), st));
    return OCM_OK;
  }
  const int64_t nblk = (m + 255) / 256;
  const size_t part_n = stats_out ? (size_t)nblk * nlv * 4 : 0;
  void* w = ocm::workspace(ctx, part_n * sizeof(double) + 512 + nlv * sizeof(int), st);
  if (!w) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(w)};
  double* part = stats_out ? cv.take<double>(part_n) : nullptr;
  int* dlv = cv.take<int>(nlv);
  OCM_HIP(hipMemcpyAsync(dlv, lvs, nlv * sizeof(int), hipMemcpyHostToDevice, st));
#define OCM_CV_PREFIX(KB)                                                                                        \
  hipLaunchKernelGGL(k_cv_prefix<KB>, dim3((unsigned)nblk), dim3(256), 0, st, T, m, k, Q, inv_evals, dlv, nlv, T2_out, \
                     Q_out, part)
  if (k <= 16) OCM_CV_PREFIX(16); else if (k <= 32) OCM_CV_PREFIX(32); else OCM_CV_PREFIX(64);
#undef OCM_CV_PREFIX
  OCM_CHECK_LAUNCH("k_cv_prefix");
  if (stats_out) {
    hipLaunchKernelGGL(k_cv_prefix_reduce, dim3(nlv), dim3(256), 0, st, part, nblk, nlv, stats_out);
    OCM_CHECK_LAUNCH("k_cv_prefix_reduce");
  }
  return OCM_OK;
}

int ocm_cv_counts(ocm_ctx* ctx, const float* T, int64_t m, int32_t k, const float* Q, const double* inv_evals,
                  const uint8_t* positive, int64_t m_split, const ocm_cv_config* cfg, int32_t ncfg,
                  uint64_t* counts_out, double* accept_out, void* stream) {
  OCM_REQUIRE(ctx && Q && inv_evals && positive && cfg && counts_out, "ocm_cv_counts: NULL argument");
  OCM_REQUIRE(k >= 1 && k <= CV_MAXK, "ocm_cv_counts: 1 <= k <= 64");
  OCM_REQUIRE(ncfg >= 1 && ncfg <= OCM_CV_MAXCFG, "ocm_cv_counts: 1 <= ncfg <= OCM_CV_MAXCFG");
  for (int c = 0; c < ncfg; ++c) {
    OCM_REQUIRE(cfg[c].lv >= 1 && cfg[c].lv <= k, "ocm_cv_counts: LV outside [1, k]");
    OCM_REQUIRE(cfg[c].type >= OCM_TYPE_SIM && cfg[c].type <= OCM_TYPE_DD, "ocm_cv_counts: bad decision type");
  }
  hipStream_t st = (hipStream_t)stream;
  OCM_HIP(hipMemsetAsync(counts_out, 0, (size_t)ncfg * 8 * sizeof(uint64_t), st));
  if (m <= 0) return OCM_OK;
  OCM_REQUIRE(T, "ocm_cv_counts: NULL T");
  void* w = ocm::workspace(ctx, (size_t)ncfg * sizeof(ocm_cv_config) + 256, st);
  if (!w) return OCM_ERR_NOMEM;
  auto* dcfg = static_cast<ocm_cv_config*>(w);
  // pageable source: the copy is staged before hipMemcpyAsync returns
  OCM_HIP(hipMemcpyAsync(dcfg, cfg, (size_t)ncfg * sizeof(ocm_cv_config), hipMemcpyHostToDevice, st));
  const int64_t want = (m + 255) / 256;
  const unsigned grid = (unsigned)std::min<int64_t>(want, (int64_t)ctx->num_cus * 8);
  auto* cnt = reinterpret_cast<unsigned long long*>(counts_out);
  const size_t lds = (size_t)ncfg * 8 * sizeof(unsigned);
#define OCM_CV_COUNTS(KB)                                                                                        \
  hipLaunchKernelGGL(k_cv_counts<KB>, dim3(grid), dim3(256), lds, st, T, m, k, Q, inv_evals, positive, m_split, dcfg, \
                     ncfg, cnt, accept_out)
  if (k <= 16) OCM_CV_COUNTS(16); else if (k <= 32) OCM_CV_COUNTS(32); else OCM_CV_COUNTS(64);
#undef OCM_CV_COUNTS
  OCM_CHECK_LAUNCH("k_cv_counts");
  return OCM_OK;
}

int ocm_confusion_counts(ocm_ctx* ctx, const double* accept, int64_t m, int64_t accept_stride,
                         const uint8_t* positive, uint64_t* counts_out, void* stream) {
  OCM_REQUIRE(ctx && counts_out, "ocm_confusion_counts: NULL argument");
  OCM_REQUIRE(m == 0 || (accept && positive), "ocm_confusion_counts: NULL argument");
  OCM_REQUIRE(m >= 0 && accept_stride >= 1, "ocm_confusion_counts: bad shape");
  hipStream_t st = (hipStream_t)stream;
  OCM_HIP(hipMemsetAsync(counts_out, 0, 4 * sizeof(uint64_t), st));
  if (m == 0) return OCM_OK;
  const unsigned grid = (unsigned)std::min<int64_t>((m + 255) / 256, (int64_t)ctx->num_cus * 4);
  hipLaunchKernelGGL(k_confusion, dim3(grid), dim3(256), 0, st, accept, m, accept_stride, positive,
                     reinterpret_cast<unsigned long long*>(counts_out));
  OCM_CHECK_LAUNCH("k_confusion");
  return OCM_OK;
}

}  // extern "C"
