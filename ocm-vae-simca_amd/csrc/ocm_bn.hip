// Training-mode BatchNorm1d for the VAE's narrow convolution stacks
// (vae_model.py:37-81: Conv1d/ConvTranspose1d → BatchNorm1d → ELU, 3-12
// channels × 512-2048 positions × B = 512).  MIOpen's spatial BN runs such
// shapes at a few GB/s (one workgroup per channel: 0.41 ms fwd + 0.19 ms bwd
// per layer at B=512, C=3, L=2048 — 63 % of the whole HIP-graph training step,
// profiles/r01_bench_i8x3_kernel_stats.md).  Here each channel's N·L
// reduction is split over many workgroups (f64 partials, fixed-order
// combine: deterministic), and the normalisation is one coalesced pass.
//
// x, y, dy, dx: (N, C, L) contiguous, bf16 (under autocast) or f32.
// Statistics f32 out (save_mean, save_invstd), math in f32/f64.
// Semantics = torch.nn.functional.batch_norm(training=True): biased variance
// for the normalisation, unbiased for running_var, momentum update.
#include <algorithm>

#include "ocm_internal.h"

namespace {

constexpr int BN_SPLIT = 64;       // workgroups per channel for the reductions, at least
constexpr int BN_SPLIT_MAX = 256;  // and at most
constexpr int BN_U = 8;            // elements per thread per pass of the reduction kernels (loads issued together)
constexpr int BN_T = 256;
// the 16-B-load reductions (k_bn_stats8 / k_bn_bwd_stats8) where the layout
// allows; OCM_BN_VEC_STATS=0 in the environment selects the scalar-load
// kernels (A/B runs, scripts/vae_ab.py)
// OCM_BN_FUSED=1: the one-launch forms below (off by default: they measured
// 1284-1287 against 1674-1678 steps/s for the two launches, the C4 step in one
// box, profiles/r06zq_vae_bn_fused_ab.jsonl — the channel's waiting workgroups
// and its last workgroup's reduction cost more than the launch they save)
bool bn_fused_on() {
  static const bool on = [] {
    const char* v = getenv("OCM_BN_FUSED");
    return v && v[0] == '1';
  }();
  return on;
}
bool bn_vec_stats() {
  static const bool on = [] {
    const char* v = getenv("OCM_BN_VEC_STATS");
    return !v || v[0] != '0';
  }();
  return on;
}

struct bf16_t {  // raw bfloat16 storage (torch.bfloat16 bit layout)
  uint16_t bits;
};
__device__ __forceinline__ float bn_ld(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float bn_ld(const bf16_t* p, int64_t i) { return __uint_as_float((uint32_t)p[i].bits << 16); }
__device__ __forceinline__ void bn_st(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void bn_st(bf16_t* p, int64_t i, float v) {
  // round to nearest even (NaN kept quiet), as torch's float → bfloat16 cast
  const uint32_t u = __float_as_uint(v);
  const uint32_t r = (u & 0x7fffffffu) > 0x7f800000u ? (u | 0x00400000u) : u + 0x7fffu + ((u >> 16) & 1u);
  p[i].bits = (uint16_t)(r >> 16);
}

// eight consecutive elements (16-B aligned: the row length is a multiple of 8)
__device__ __forceinline__ void bn_ld8(const float* p, int64_t i, float (&v)[8]) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p + i), b = *reinterpret_cast<const f32x4*>(p + i + 4);
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[e] = a[e];
    v[4 + e] = b[e];
  }
}
__device__ __forceinline__ void bn_ld8(const bf16_t* p, int64_t i, float (&v)[8]) {
  const uint4 q = *reinterpret_cast<const uint4*>(p + i);
  const uint32_t w[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    v[2 * e] = __uint_as_float(w[e] << 16);
    v[2 * e + 1] = __uint_as_float(w[e] & 0xffff0000u);
  }
}
__device__ __forceinline__ void bn_st8(float* p, int64_t i, const float (&v)[8]) {
  *reinterpret_cast<f32x4*>(p + i) = f32x4{v[0], v[1], v[2], v[3]};
  *reinterpret_cast<f32x4*>(p + i + 4) = f32x4{v[4], v[5], v[6], v[7]};
}
__device__ __forceinline__ void bn_st8(bf16_t* p, int64_t i, const float (&v)[8]) {
  uint32_t w[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    bf16_t lo, hi;
    bn_st(&lo, 0, v[2 * e]);
    bn_st(&hi, 0, v[2 * e + 1]);
    w[e] = (uint32_t)lo.bits | ((uint32_t)hi.bits << 16);
  }
  *reinterpret_cast<uint4*>(p + i) = uint4{w[0], w[1], w[2], w[3]};
}

__device__ __forceinline__ double block_sum_f64(double v, double* red) {
  v = wave_sum_f64(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) red[w] = v;
  __syncthreads();
  double t = 0.0;
  for (int i = 0; i < BN_T / 64; ++i) t += red[i];
  return t;
}

// split workgroups per channel for the reductions: enough to fill the chip when
// C is small (3-channel layers), at most BN_SPLIT_MAX
__host__ __device__ inline int bn_split(int C) {
  const int s = 2048 / (C > 0 ? C : 1);
  return s < BN_SPLIT ? BN_SPLIT : (s > BN_SPLIT_MAX ? BN_SPLIT_MAX : s);
}

// the n·L + l elements of channel c, BN_U per thread per pass, loads issued
// together (clamped index + select: no branch around a load)
template <typename T>
__device__ __forceinline__ float bn_ld_or0(const T* p, int C, int L, int c, int e, int total) {
  const bool ok = e < total;
  const int ec = ok ? e : 0;
  const int n = ec / L, l = ec - n * L;
  const float v = bn_ld(p, ((int64_t)n * C + c) * L + l);
  return ok ? v : 0.f;
}

// the split partials of channel c summed by one wave (lane-strided, then the
// fixed butterfly: deterministic)
__device__ __forceinline__ void bn_part_sum(const double* part, int c, int split, double& s1, double& s2) {
  const int lane = threadIdx.x & 63;
  // other workgroups' partials: write-through loads, eight per lane in flight
  s1 = wave_sum_f64(lane_sum_agent<double, double>(part + (size_t)c * split * 2, 2, split, lane));
  s2 = wave_sum_f64(lane_sum_agent<double, double>(part + (size_t)c * split * 2 + 1, 2, split, lane));
}

// The workgroup's partials → part (write-through); true in the last of channel
// c's split workgroups to arrive (ocm_internal.h last_arrival)
__device__ __forceinline__ bool bn_ticket(double s1, double s2, double* part, unsigned* ticket, int c, int sp,
                                          int split) {
  if (threadIdx.x == 0) {
    st_agent(part + ((size_t)c * split + sp) * 2 + 0, s1);
    st_agent(part + ((size_t)c * split + sp) * 2 + 1, s2);
  }
  return last_arrival2(ticket, c, (unsigned)split, (unsigned)sp);
}

constexpr int BN_U8 = 4;  // 16-B loads per thread and pass of the vectorised reductions

// the 8-element group e of channel c (e < total = N·L/8: row n = e / L8,
// positions 8·(e mod L8) …), loaded at a clamped index and zeroed past total
template <typename T>
__device__ __forceinline__ void bn_ld8_or0(const T* p, int C, int L8, int c, int e, int total, float (&v)[8]) {
  const bool ok = e < total;
  const int ec = ok ? e : 0;
  const int n = ec / L8, l = (ec - n * L8) * 8;
  bn_ld8(p, ((int64_t)n * C + c) * (int64_t)(8 * L8) + l, v);
#pragma unroll
  for (int k = 0; k < 8; ++k) v[k] = ok ? v[k] : 0.f;
}

__device__ __forceinline__ void bn_stats_tail(float a1, float a2, double* red, int N, int L, double* part,
                                              unsigned* ticket, float eps, float momentum, float* save_mean,
                                              float* save_invstd, float* running_mean, float* running_var,
                                              int64_t* nbt);

// grid (split, C): partial Σx, Σx² of channel c over its share of the N·L
// elements; the channel's last workgroup forms mean / invstd and the running
// statistics (and counts the batch in num_batches_tracked, channel 0)
template <typename T>
__global__ __launch_bounds__(BN_T) void k_bn_stats(const T* __restrict__ x, int N, int C, int L,
                                                   double* __restrict__ part, unsigned* __restrict__ ticket,
                                                   float eps, float momentum, float* __restrict__ save_mean,
                                                   float* __restrict__ save_invstd, float* __restrict__ running_mean,
                                                   float* __restrict__ running_var, int64_t* __restrict__ nbt) {
  __shared__ double red[BN_T / 64];
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x;
  const int total = N * L, step = split * BN_T;
  float a1 = 0.f, a2 = 0.f;  // ≤ N·L / (split·BN_T) terms per thread in f32, f64 across threads
  for (int e0 = sp * BN_T + threadIdx.x; e0 < total; e0 += BN_U * step) {
    float v[BN_U];
#pragma unroll
    for (int r = 0; r < BN_U; ++r) v[r] = bn_ld_or0(x, C, L, c, e0 + r * step, total);
#pragma unroll
    for (int r = 0; r < BN_U; ++r) {
      a1 += v[r];
      a2 = fmaf(v[r], v[r], a2);
    }
  }
  bn_stats_tail(a1, a2, red, N, L, part, ticket, eps, momentum, save_mean, save_invstd, running_mean, running_var,
                nbt);
}

// the same sums from 16-B loads, eight consecutive positions of one row each
// (L % 8 = 0, x 16-B aligned), BN_U8 of them in flight per thread: grid
// (bn_split8, C).  The scalar form issued 2-byte loads, one element per lane
// (8.4 µs per C4 layer, profiles/r06zj_vae_step_trace.md)
template <typename T>
__global__ __launch_bounds__(BN_T) void k_bn_stats8(const T* __restrict__ x, int N, int C, int L,
                                                    double* __restrict__ part, unsigned* __restrict__ ticket,
                                                    float eps, float momentum, float* __restrict__ save_mean,
                                                    float* __restrict__ save_invstd, float* __restrict__ running_mean,
                                                    float* __restrict__ running_var, int64_t* __restrict__ nbt) {
  __shared__ double red[BN_T / 64];
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x;
  const int L8 = L / 8, total = N * L8, step = split * BN_T;
  float a1 = 0.f, a2 = 0.f;
  for (int e0 = sp * BN_T + threadIdx.x; e0 < total; e0 += BN_U8 * step) {
    float v[BN_U8][8];
#pragma unroll
    for (int r = 0; r < BN_U8; ++r) bn_ld8_or0(x, C, L8, c, e0 + r * step, total, v[r]);
#pragma unroll
    for (int r = 0; r < BN_U8; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        a1 += v[r][k];
        a2 = fmaf(v[r][k], v[r][k], a2);
      }
  }
  bn_stats_tail(a1, a2, red, N, L, part, ticket, eps, momentum, save_mean, save_invstd, running_mean, running_var,
                nbt);
}

// the workgroup's sums → the channel's last workgroup forms mean / invstd and
// the running statistics (and counts the batch in num_batches_tracked, channel 0)
__device__ __forceinline__ void bn_stats_tail(float a1, float a2, double* red, int N, int L, double* part,
                                              unsigned* ticket, float eps, float momentum, float* save_mean,
                                              float* save_invstd, float* running_mean, float* running_var,
                                              int64_t* nbt) {
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x;
  const double s1 = block_sum_f64(a1, red);
  const double s2 = block_sum_f64(a2, red);
  if (!bn_ticket(s1, s2, part, ticket, c, sp, split) || threadIdx.x >= 64) return;
  double t1, t2;
  bn_part_sum(part, c, split, t1, t2);
  if (threadIdx.x != 0) return;
  const int64_t M = (int64_t)N * L;
  const double mean = t1 / (double)M;
  const double var = fmax(t2 / (double)M - mean * mean, 0.0);
  save_mean[c] = (float)mean;
  save_invstd[c] = (float)(1.0 / sqrt(var + (double)eps));
  if (running_mean) {
    const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
    running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
    running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
  }
  if (nbt && c == 0) *nbt += 1;
}

// grid (ceil(L / BN_T), N·C): y = (x − μ)·invstd·γ + β, then ELU (α = 1) when
// fused: z > 0 ? z : exp(z) − 1 (torch's elu, evaluated in float)
template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_apply(const T* __restrict__ x, int C, int L,
                                                   const float* __restrict__ mean, const float* __restrict__ invstd,
                                                   const float* __restrict__ gamma, const float* __restrict__ beta,
                                                   T* __restrict__ y) {
  const int row = blockIdx.y, c = row % C;
  const int l = blockIdx.x * BN_T + threadIdx.x;
  if (l >= L) return;
  const float a = invstd[c] * (gamma ? gamma[c] : 1.f);
  const float b = (beta ? beta[c] : 0.f) - mean[c] * a;
  const int64_t i = (int64_t)row * L + l;
  const float z = fmaf(bn_ld(x, i), a, b);
  bn_st(y, i, ELU ? (z > 0.f ? z : expf(z) - 1.f) : z);
}

// the same, eight consecutive positions per thread (L % 8 = 0): grid
// (ceil(L / (8·BN_T)), N·C), 16-B loads and stores
template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_apply8(const T* __restrict__ x, int C, int L,
                                                    const float* __restrict__ mean, const float* __restrict__ invstd,
                                                    const float* __restrict__ gamma, const float* __restrict__ beta,
                                                    T* __restrict__ y) {
  const int row = blockIdx.y, c = row % C;
  const int l = (blockIdx.x * BN_T + threadIdx.x) * 8;
  if (l >= L) return;
  const float a = invstd[c] * (gamma ? gamma[c] : 1.f);
  const float b = (beta ? beta[c] : 0.f) - mean[c] * a;
  const int64_t i = (int64_t)row * L + l;
  float v[8];
  bn_ld8(x, i, v);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float z = fmaf(v[e], a, b);
    v[e] = ELU ? (z > 0.f ? z : expf(z) - 1.f) : z;
  }
  bn_st8(y, i, v);
}

// eval mode (running statistics): y = (x − rm)·γ/√(rv + ε) + β (+ ELU), V
// consecutive values per thread over a flat (row, position) index — the
// latent-encoding batches are 8192 rows × C channels, past a 65535-row grid.y
// (MIOpen's inference kernel took 3.3 ms per call on them)
template <typename T, bool ELU, int V>
__global__ __launch_bounds__(BN_T) void k_bn_eval(const T* __restrict__ x, int C, int L, int64_t items,
                                                  const float* __restrict__ rm, const float* __restrict__ rv, float eps,
                                                  const float* __restrict__ gamma, const float* __restrict__ beta,
                                                  T* __restrict__ y) {
  const int64_t it = (int64_t)blockIdx.x * BN_T + threadIdx.x;
  if (it >= items) return;
  const int LV = L / V;
  const int64_t row = it / LV;
  const int c = (int)(row % C);
  const float inv = 1.f / sqrtf(rv[c] + eps);
  const float a = inv * (gamma ? gamma[c] : 1.f);
  const float b = (beta ? beta[c] : 0.f) - rm[c] * a;
  const int64_t i = row * L + (it - row * LV) * V;
  float v[V];
  if constexpr (V == 8) {
    bn_ld8(x, i, v);
  } else {
    v[0] = bn_ld(x, i);
  }
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const float z = fmaf(v[e], a, b);
    v[e] = ELU ? (z > 0.f ? z : expf(z) - 1.f) : z;
  }
  if constexpr (V == 8) {
    bn_st8(y, i, v);
  } else {
    bn_st(y, i, v[0]);
  }
}

// the gradient reaching the batch norm's output: with the fused ELU, dz = dy·(y > 0 ? 1 : y + 1)
// from the ELU output y (torch's elu_backward on the result)
template <bool ELU, typename T>
__device__ __forceinline__ float bn_grad(const T* dy, const T* ya, int64_t i) {
  const float g = bn_ld(dy, i);
  if (!ELU) return g;
  const float v = bn_ld(ya, i);
  return v > 0.f ? g : g * (v + 1.f);
}

__device__ __forceinline__ void bn_bwd_tail(float a1, float a2, double* red, double* part, unsigned* ticket,
                                            double* sums, float* dgamma, float* dbeta);

// grid (split, C): partial Σdz, Σdz·x̂; the channel's last workgroup forms
// the sums (and dβ, dγ)
template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_bwd_stats(const T* __restrict__ x, const T* __restrict__ dy,
                                                       const T* __restrict__ ya, int N,
                                                       int C, int L, const float* __restrict__ mean,
                                                       const float* __restrict__ invstd, double* __restrict__ part,
                                                       unsigned* __restrict__ ticket, double* __restrict__ sums,
                                                       float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ double red[BN_T / 64];
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x;
  const float mu = mean[c], is = invstd[c];
  const int total = N * L, step = split * BN_T;
  float a1 = 0.f, a2 = 0.f;
  for (int e0 = sp * BN_T + threadIdx.x; e0 < total; e0 += BN_U * step) {
    float g[BN_U], xv[BN_U], yv[BN_U];
#pragma unroll
    for (int r = 0; r < BN_U; ++r) {  // every load of the pass first
      g[r] = bn_ld_or0(dy, C, L, c, e0 + r * step, total);
      xv[r] = bn_ld_or0(x, C, L, c, e0 + r * step, total);
      if (ELU) yv[r] = bn_ld_or0(ya, C, L, c, e0 + r * step, total);
    }
#pragma unroll
    for (int r = 0; r < BN_U; ++r) {
      if (ELU) g[r] = yv[r] > 0.f ? g[r] : g[r] * (yv[r] + 1.f);
      a1 += g[r];
      // padded elements: g = 0, so the (0 − μ)·invstd term adds nothing
      a2 = fmaf(g[r], (xv[r] - mu) * is, a2);
    }
  }
  bn_bwd_tail(a1, a2, red, part, ticket, sums, dgamma, dbeta);
}

// the same sums from 16-B loads (L % 8 = 0, x / dy / ya 16-B aligned; see
// k_bn_stats8): grid (bn_split8, C)
template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_bwd_stats8(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const T* __restrict__ ya, int N, int C, int L,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd, double* __restrict__ part,
                                                        unsigned* __restrict__ ticket, double* __restrict__ sums,
                                                        float* __restrict__ dgamma, float* __restrict__ dbeta) {
  __shared__ double red[BN_T / 64];
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x;
  const float mu = mean[c], is = invstd[c];
  const int L8 = L / 8, total = N * L8, step = split * BN_T;
  constexpr int U = BN_U8 / 2;  // three tensors: two groups of each in flight
  float a1 = 0.f, a2 = 0.f;
  for (int e0 = sp * BN_T + threadIdx.x; e0 < total; e0 += U * step) {
    float g[U][8], xv[U][8], yv[ELU ? U : 1][8];
#pragma unroll
    for (int r = 0; r < U; ++r) {  // every load of the pass first
      bn_ld8_or0(dy, C, L8, c, e0 + r * step, total, g[r]);
      bn_ld8_or0(x, C, L8, c, e0 + r * step, total, xv[r]);
      if (ELU) bn_ld8_or0(ya, C, L8, c, e0 + r * step, total, yv[ELU ? r : 0]);
    }
#pragma unroll
    for (int r = 0; r < U; ++r)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float gz = g[r][k];
        if (ELU) gz = yv[ELU ? r : 0][k] > 0.f ? gz : gz * (yv[ELU ? r : 0][k] + 1.f);
        a1 += gz;
        // padded groups: g = 0, so the (0 − μ)·invstd term adds nothing
        a2 = fmaf(gz, (xv[r][k] - mu) * is, a2);
      }
  }
  bn_bwd_tail(a1, a2, red, part, ticket, sums, dgamma, dbeta);
}

__device__ __forceinline__ void bn_bwd_tail(float a1, float a2, double* red, double* part, unsigned* ticket,
                                            double* sums, float* dgamma, float* dbeta) {
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x;
  const double s1 = block_sum_f64(a1, red);
  const double s2 = block_sum_f64(a2, red);
  if (!bn_ticket(s1, s2, part, ticket, c, sp, split) || threadIdx.x >= 64) return;
  double t1, t2;
  bn_part_sum(part, c, split, t1, t2);
  if (threadIdx.x != 0) return;
  sums[2 * c] = t1;
  sums[2 * c + 1] = t2;
  if (dbeta) dbeta[c] = (float)t1;
  if (dgamma) dgamma[c] = (float)t2;
}

// dx = γ·invstd·(dz − Σdz/M − x̂·Σ(dz·x̂)/M)
template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_bwd_apply(const T* __restrict__ x, const T* __restrict__ dy,
                                                       const T* __restrict__ ya, int C,
                                                       int L, int64_t M, const float* __restrict__ mean,
                                                       const float* __restrict__ invstd,
                                                       const float* __restrict__ gamma,
                                                       const double* __restrict__ sums, T* __restrict__ dx) {
  const int row = blockIdx.y, c = row % C;
  const int l = blockIdx.x * BN_T + threadIdx.x;
  if (l >= L) return;
  const float is = invstd[c], mu = mean[c];
  const float k = is * (gamma ? gamma[c] : 1.f);
  const float m1 = (float)(sums[2 * c] / (double)M), m2 = (float)(sums[2 * c + 1] / (double)M);
  const int64_t i = (int64_t)row * L + l;
  const float xh = (bn_ld(x, i) - mu) * is;
  bn_st(dx, i, k * (bn_grad<ELU>(dy, ya, i) - m1 - xh * m2));
}

template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_bwd_apply8(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const T* __restrict__ ya, int C,
                                                        int L, int64_t M, const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma,
                                                        const double* __restrict__ sums, T* __restrict__ dx) {
  const int row = blockIdx.y, c = row % C;
  const int l = (blockIdx.x * BN_T + threadIdx.x) * 8;
  if (l >= L) return;
  const float is = invstd[c], mu = mean[c];
  const float k = is * (gamma ? gamma[c] : 1.f);
  const float m1 = (float)(sums[2 * c] / (double)M), m2 = (float)(sums[2 * c + 1] / (double)M);
  const int64_t i = (int64_t)row * L + l;
  float xv[8], g[8], yv[8];
  bn_ld8(x, i, xv);
  bn_ld8(dy, i, g);
  if (ELU) bn_ld8(ya, i, yv);
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float gz = ELU ? (yv[e] > 0.f ? g[e] : g[e] * (yv[e] + 1.f)) : g[e];
    const float xh = (xv[e] - mu) * is;
    xv[e] = k * (gz - m1 - xh * m2);
  }
  bn_st8(dx, i, xv);
}

// ---- one-launch forms (round 6): the statistics and the normalisation in
// one kernel, each thread's share of the channel held in registers between
// them (read once).  Every workgroup of channel c reads the channel's epoch
// word before it takes its ticket; the last to arrive forms the statistics,
// stores them and bumps the epoch; the others wait for the bump (s_sleep
// polls), then read them.  Opt-in (bn_fused_on).  The host launches this form only when the grid is
// co-resident (≤ the CUs' occupancy for the kernel, bn_fused_ok) and each
// thread's share fits one pass; a wait that still exceeds ≈ 1 s gives up (the
// outputs are then wrong) and counts in g_bn_wait_timeouts
// (ocm_bn_fused_timeouts) rather than hang the GPU.
__device__ unsigned long long g_bn_wait_timeouts;
constexpr unsigned BN_SPINS_1S = 1u << 22;  // ≈ 1 s of s_sleep(8) polls

// thread 0: wait until *epoch differs from e0 (acquire); false on timeout
__device__ __forceinline__ bool bn_wait_epoch(const unsigned* epoch, unsigned e0) {
  unsigned n = 0;
  while (__hip_atomic_load(const_cast<unsigned*>(epoch), __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) == e0 &&
         ++n < BN_SPINS_1S)
    __builtin_amdgcn_s_sleep(8);
  if (n < BN_SPINS_1S) return true;
  atomicAdd(&g_bn_wait_timeouts, 1ull);
  return false;
}
__device__ __forceinline__ void bn_bump_epoch(unsigned* epoch) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the statistics' write-through stores have left
  __hip_atomic_fetch_add(epoch, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
}

// forward: grid (split, C) with N·L/8 ≤ split·BN_T·BN_U8 (one pass)
template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_fused8(const T* __restrict__ x, int N, int C, int L,
                                                    double* __restrict__ part, unsigned* __restrict__ ticket,
                                                    unsigned* __restrict__ epoch, float eps, float momentum,
                                                    float* __restrict__ save_mean, float* __restrict__ save_invstd,
                                                    float* __restrict__ running_mean, float* __restrict__ running_var,
                                                    int64_t* __restrict__ nbt, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, T* __restrict__ y) {
  __shared__ double red[BN_T / 64];
  __shared__ unsigned e0s;
  __shared__ float ab[2];
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x, tid = threadIdx.x;
  const int L8 = L / 8, total = N * L8, step = split * BN_T;
  unsigned* ep = epoch + (size_t)c * TICKET_STRIDE;
  if (tid == 0) e0s = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // before the ticket
  float v[BN_U8][8];
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int r = 0; r < BN_U8; ++r) bn_ld8_or0(x, C, L8, c, sp * BN_T + tid + r * step, total, v[r]);
#pragma unroll
  for (int r = 0; r < BN_U8; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      a1 += v[r][k];
      a2 = fmaf(v[r][k], v[r][k], a2);
    }
  const double s1 = block_sum_f64(a1, red);
  const double s2 = block_sum_f64(a2, red);
  const bool last = bn_ticket(s1, s2, part, ticket, c, sp, split);  // (its vmcnt(0) orders the epoch read first)
  if (last) {
    if (tid < 64) {
      double t1, t2;
      bn_part_sum(part, c, split, t1, t2);
      if (tid == 0) {
        const int64_t M = (int64_t)N * L;
        const double mean = t1 / (double)M;
        const double var = fmax(t2 / (double)M - mean * mean, 0.0);
        const float mf = (float)mean, inv = (float)(1.0 / sqrt(var + (double)eps));
        st_agent(save_mean + c, mf);
        st_agent(save_invstd + c, inv);
        if (running_mean) {
          const double unb = M > 1 ? var * (double)M / (double)(M - 1) : var;
          running_mean[c] = (float)((1.0 - momentum) * running_mean[c] + momentum * mean);
          running_var[c] = (float)((1.0 - momentum) * running_var[c] + momentum * unb);
        }
        if (nbt && c == 0) *nbt += 1;
        const float a = inv * (gamma ? gamma[c] : 1.f);
        ab[0] = a;
        ab[1] = (beta ? beta[c] : 0.f) - mf * a;
        bn_bump_epoch(ep);
      }
    }
  } else if (tid == 0) {
    bn_wait_epoch(ep, e0s);
    const float mf = ld_agent(save_mean + c), inv = ld_agent(save_invstd + c);
    const float a = inv * (gamma ? gamma[c] : 1.f);
    ab[0] = a;
    ab[1] = (beta ? beta[c] : 0.f) - mf * a;
  }
  __syncthreads();
  const float a = ab[0], b = ab[1];
#pragma unroll
  for (int r = 0; r < BN_U8; ++r) {
    const int e = sp * BN_T + tid + r * step;
    if (e >= total) continue;
    const int n = e / L8, l = (e - n * L8) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float z = fmaf(v[r][k], a, b);
      v[r][k] = ELU ? (z > 0.f ? z : expf(z) - 1.f) : z;
    }
    bn_st8(y, ((int64_t)n * C + c) * L + l, v[r]);
  }
}

// backward: the sums Σdz, Σdz·x̂ and dx = γ·invstd·(dz − Σdz/M − x̂·Σ(dz·x̂)/M) in one launch
template <typename T, bool ELU>
__global__ __launch_bounds__(BN_T) void k_bn_bwd_fused8(const T* __restrict__ x, const T* __restrict__ dy,
                                                        const T* __restrict__ ya, int N, int C, int L,
                                                        const float* __restrict__ mean,
                                                        const float* __restrict__ invstd,
                                                        const float* __restrict__ gamma, double* __restrict__ part,
                                                        unsigned* __restrict__ ticket, unsigned* __restrict__ epoch,
                                                        double* __restrict__ sums, float* __restrict__ dgamma,
                                                        float* __restrict__ dbeta, T* __restrict__ dx) {
  __shared__ double red[BN_T / 64];
  __shared__ unsigned e0s;
  __shared__ double m12[2];
  const int c = blockIdx.y, sp = blockIdx.x, split = gridDim.x, tid = threadIdx.x;
  const float mu = mean[c], is = invstd[c];
  const int L8 = L / 8, total = N * L8, step = split * BN_T;
  unsigned* ep = epoch + (size_t)c * TICKET_STRIDE;
  if (tid == 0) e0s = __hip_atomic_load(ep, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  float g[BN_U8][8], xv[BN_U8][8];
  {
    float yv[ELU ? BN_U8 : 1][8];
#pragma unroll
    for (int r = 0; r < BN_U8; ++r) {
      bn_ld8_or0(dy, C, L8, c, sp * BN_T + tid + r * step, total, g[r]);
      bn_ld8_or0(x, C, L8, c, sp * BN_T + tid + r * step, total, xv[r]);
      if (ELU) bn_ld8_or0(ya, C, L8, c, sp * BN_T + tid + r * step, total, yv[ELU ? r : 0]);
    }
    if (ELU) {
#pragma unroll
      for (int r = 0; r < BN_U8; ++r)
#pragma unroll
        for (int k = 0; k < 8; ++k) g[r][k] = yv[ELU ? r : 0][k] > 0.f ? g[r][k] : g[r][k] * (yv[ELU ? r : 0][k] + 1.f);
    }
  }
  float a1 = 0.f, a2 = 0.f;
#pragma unroll
  for (int r = 0; r < BN_U8; ++r)
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      xv[r][k] = (xv[r][k] - mu) * is;  // x̂ (padded groups: g = 0 adds nothing)
      a1 += g[r][k];
      a2 = fmaf(g[r][k], xv[r][k], a2);
    }
  const double s1 = block_sum_f64(a1, red);
  const double s2 = block_sum_f64(a2, red);
  const bool last = bn_ticket(s1, s2, part, ticket, c, sp, split);
  if (last) {
    if (tid < 64) {
      double t1, t2;
      bn_part_sum(part, c, split, t1, t2);
      if (tid == 0) {
        st_agent(sums + 2 * c, t1);
        st_agent(sums + 2 * c + 1, t2);
        if (dbeta) dbeta[c] = (float)t1;
        if (dgamma) dgamma[c] = (float)t2;
        m12[0] = t1;
        m12[1] = t2;
        bn_bump_epoch(ep);
      }
    }
  } else if (tid == 0) {
    bn_wait_epoch(ep, e0s);
    m12[0] = ld_agent(sums + 2 * c);
    m12[1] = ld_agent(sums + 2 * c + 1);
  }
  __syncthreads();
  const double M = (double)N * L;
  const float m1 = (float)(m12[0] / M), m2 = (float)(m12[1] / M);
  const float kk = is * (gamma ? gamma[c] : 1.f);
#pragma unroll
  for (int r = 0; r < BN_U8; ++r) {
    const int e = sp * BN_T + tid + r * step;
    if (e >= total) continue;
    const int n = e / L8, l = (e - n * L8) * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) g[r][k] = kk * (g[r][k] - m1 - xv[r][k] * m2);
    bn_st8(dx, ((int64_t)n * C + c) * L + l, g[r]);
  }
}

// scratch of the forward / backward calls: per-(channel, split) partials, the
// backward's channel sums, then one completion counter per channel (zero
// before the first call; every call leaves them zero)
// workgroups per channel of the vectorised reductions: BN_U8 16-B groups per
// thread in one pass (≥ 1, ≤ bn_split(C): the scratch is laid out for that)
int bn_split8(int N, int C, int L) {
  const int64_t g8 = (int64_t)N * (L / 8);
  const int64_t s = (g8 + (int64_t)BN_T * BN_U8 - 1) / ((int64_t)BN_T * BN_U8);
  return (int)std::max<int64_t>(1, std::min<int64_t>(s, bn_split(C)));
}

size_t bn_part_doubles(int C) { return (size_t)C * bn_split(C) * 2 + 2 * (size_t)C; }
size_t bn_ticket_words(int C) { return (size_t)C * tickets_per_slot(bn_split(C)) * TICKET_STRIDE; }
// + one epoch word per channel (128-B apart) for the one-launch forms
size_t bn_scratch(int C) {
  return bn_part_doubles(C) * sizeof(double) + (bn_ticket_words(C) + (size_t)C * TICKET_STRIDE) * sizeof(unsigned);
}

// the one-launch form applies (opted in): one pass per thread, the whole grid resident
// at once (the occupancy of the kernel × the CUs, queried once per kernel)
template <class K>
bool bn_fused_ok(ocm_ctx* ctx, K kernel, int N, int C, int L, int split) {
  if (!bn_fused_on()) return false;
  if ((int64_t)N * (L / 8) > (int64_t)split * BN_T * BN_U8) return false;
  static const void* keys[16];  // occupancy per kernel, queried once (benign race: the same value)
  static int vals[16], used = 0;
  const void* key = reinterpret_cast<const void*>(kernel);
  int per_cu = -1;
  for (int i = 0; i < used; ++i)
    if (keys[i] == key) per_cu = vals[i];
  if (per_cu < 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, kernel, BN_T, 0) != hipSuccess) nb = 0;
    per_cu = nb;
    if (used < 16) {
      keys[used] = key;
      vals[used] = nb;
      ++used;
    }
  }
  return per_cu > 0 && (int64_t)split * C <= (int64_t)per_cu * ctx->num_cus;
}

template <typename T>
int bn_fwd(ocm_ctx* ctx, const void* x, int N, int C, int L, const float* gamma, const float* beta, float eps,
           float momentum, float* rmean, float* rvar, int64_t* nbt, void* y, float* smean, float* sinv,
           void* scratch, int act, hipStream_t st) {
  auto* part = static_cast<double*>(scratch);
  auto* ticket = reinterpret_cast<unsigned*>(part + bn_part_doubles(C));
  unsigned* epoch = ticket + bn_ticket_words(C);
  const bool v8 = L % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
  if (v8 && bn_vec_stats()) {
    const int s8 = bn_split8(N, C, L);
#define OCM_BN_FUSED_L(E_)                                                                                           \
  if (bn_fused_ok(ctx, k_bn_fused8<T, E_>, N, C, L, s8)) {                                                          \
    hipLaunchKernelGGL((k_bn_fused8<T, E_>), dim3(s8, C), dim3(BN_T), 0, st, static_cast<const T*>(x), N, C, L, part, \
                       ticket, epoch, eps, momentum, smean, sinv, rmean, rvar, nbt, gamma, beta, static_cast<T*>(y)); \
    OCM_CHECK_LAUNCH("k_bn_fused8");                                                                                  \
    return OCM_OK;                                                                                                    \
  }
    if (act == OCM_ACT_ELU) {
      OCM_BN_FUSED_L(true)
    } else {
      OCM_BN_FUSED_L(false)
    }
#undef OCM_BN_FUSED_L
  }
  if (v8 && bn_vec_stats())
    hipLaunchKernelGGL(k_bn_stats8<T>, dim3(bn_split8(N, C, L), C), dim3(BN_T), 0, st, static_cast<const T*>(x), N, C,
                       L, part, ticket, eps, momentum, smean, sinv, rmean, rvar, nbt);
  else
    hipLaunchKernelGGL(k_bn_stats<T>, dim3(bn_split(C), C), dim3(BN_T), 0, st, static_cast<const T*>(x), N, C, L,
                       part, ticket, eps, momentum, smean, sinv, rmean, rvar, nbt);
  const dim3 ga(v8 ? (L / 8 + BN_T - 1) / BN_T : (L + BN_T - 1) / BN_T, N * C);
#define OCM_BN_APPLY(K_, E_) \
  hipLaunchKernelGGL((K_<T, E_>), ga, dim3(BN_T), 0, st, static_cast<const T*>(x), C, L, smean, sinv, gamma, beta, \
                     static_cast<T*>(y))
  if (act == OCM_ACT_ELU) {
    if (v8) OCM_BN_APPLY(k_bn_apply8, true); else OCM_BN_APPLY(k_bn_apply, true);
  } else {
    if (v8) OCM_BN_APPLY(k_bn_apply8, false); else OCM_BN_APPLY(k_bn_apply, false);
  }
#undef OCM_BN_APPLY
  OCM_CHECK_LAUNCH("k_bn_fwd");
  return OCM_OK;
}

template <typename T, bool ELU>
int bn_bwd(ocm_ctx* ctx, const void* x, const void* dy, const void* ya, int N, int C, int L, const float* gamma,
           const float* smean, const float* sinv, void* dx, float* dgamma, float* dbeta, void* scratch,
           hipStream_t st) {
  auto* part = static_cast<double*>(scratch);
  auto* ticket = reinterpret_cast<unsigned*>(part + bn_part_doubles(C));
  const int split = bn_split(C);
  double* sums = part + (size_t)C * split * 2;
  unsigned* epoch = ticket + bn_ticket_words(C);
  const auto al = [](const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; };
  if (bn_vec_stats() && L % 8 == 0 && al(x) && al(dy) && (!ELU || al(ya)) && al(dx) &&
      bn_fused_ok(ctx, k_bn_bwd_fused8<T, ELU>, N, C, L, bn_split8(N, C, L))) {
    hipLaunchKernelGGL((k_bn_bwd_fused8<T, ELU>), dim3(bn_split8(N, C, L), C), dim3(BN_T), 0, st,
                       static_cast<const T*>(x), static_cast<const T*>(dy), static_cast<const T*>(ya), N, C, L, smean,
                       sinv, gamma, part, ticket, epoch, sums, dgamma, dbeta, static_cast<T*>(dx));
    OCM_CHECK_LAUNCH("k_bn_bwd_fused8");
    return OCM_OK;
  }
  if (bn_vec_stats() && L % 8 == 0 && al(x) && al(dy) && (!ELU || al(ya)))
    hipLaunchKernelGGL((k_bn_bwd_stats8<T, ELU>), dim3(bn_split8(N, C, L), C), dim3(BN_T), 0, st,
                       static_cast<const T*>(x), static_cast<const T*>(dy), static_cast<const T*>(ya), N, C, L, smean,
                       sinv, part, ticket, sums, dgamma, dbeta);
  else
    hipLaunchKernelGGL((k_bn_bwd_stats<T, ELU>), dim3(split, C), dim3(BN_T), 0, st, static_cast<const T*>(x),
                       static_cast<const T*>(dy), static_cast<const T*>(ya), N, C, L, smean, sinv, part, ticket, sums,
                       dgamma, dbeta);
  if (L % 8 == 0 && al(x) && al(dy) && (!ELU || al(ya)) && al(dx))
    hipLaunchKernelGGL((k_bn_bwd_apply8<T, ELU>), dim3((L / 8 + BN_T - 1) / BN_T, N * C), dim3(BN_T), 0, st,
                       static_cast<const T*>(x), static_cast<const T*>(dy), static_cast<const T*>(ya), C, L,
                       (int64_t)N * L, smean, sinv, gamma, sums, static_cast<T*>(dx));
  else
    hipLaunchKernelGGL((k_bn_bwd_apply<T, ELU>), dim3((L + BN_T - 1) / BN_T, N * C), dim3(BN_T), 0, st,
                       static_cast<const T*>(x), static_cast<const T*>(dy), static_cast<const T*>(ya), C, L,
                       (int64_t)N * L, smean, sinv, gamma, sums, static_cast<T*>(dx));
  OCM_CHECK_LAUNCH("k_bn_bwd");
  return OCM_OK;
}

}  // namespace

extern "C" {

size_t ocm_bn_scratch_bytes(int32_t C) { return C > 0 ? bn_scratch(C) : 0; }

int ocm_bn_fused_timeouts(int64_t* count_out) {
  OCM_REQUIRE(count_out, "ocm_bn_fused_timeouts: NULL argument");
  unsigned long long v = 0;
  OCM_HIP(hipMemcpyFromSymbol(&v, HIP_SYMBOL(g_bn_wait_timeouts), sizeof(v)));
  *count_out = (int64_t)v;
  return OCM_OK;
}

int ocm_bn_fwd_train(ocm_ctx* ctx, int32_t dtype, const void* x, int32_t N, int32_t C, int32_t L,
                     const float* gamma, const float* beta, float eps, float momentum, float* running_mean,
                     float* running_var, int64_t* num_batches_tracked, int32_t act, void* y, float* save_mean,
                     float* save_invstd, void* scratch, void* stream) {
  OCM_REQUIRE(ctx && x && y && save_mean && save_invstd && scratch, "ocm_bn_fwd_train: NULL argument");
  OCM_REQUIRE(N > 0 && C > 0 && L > 0 && (int64_t)N * L < INT32_MAX, "ocm_bn_fwd_train: bad shape");
  OCM_REQUIRE(!running_mean == !running_var, "ocm_bn_fwd_train: running_mean and running_var go together");
  OCM_REQUIRE(act == OCM_ACT_NONE || act == OCM_ACT_ELU, "ocm_bn_fwd_train: act must be OCM_ACT_NONE or OCM_ACT_ELU");
  hipStream_t st = (hipStream_t)stream;
  if (dtype == OCM_DTYPE_F32)
    return bn_fwd<float>(ctx, x, N, C, L, gamma, beta, eps, momentum, running_mean, running_var, num_batches_tracked,
                         y, save_mean, save_invstd, scratch, act, st);
  if (dtype == OCM_DTYPE_BF16)
    return bn_fwd<bf16_t>(ctx, x, N, C, L, gamma, beta, eps, momentum, running_mean, running_var,
                          num_batches_tracked, y, save_mean, save_invstd, scratch, act, st);
  return ocm::fail(OCM_ERR_ARG, "ocm_bn_fwd_train: dtype must be OCM_DTYPE_F32 or OCM_DTYPE_BF16");
}

int ocm_bn_fwd_eval(ocm_ctx* ctx, int32_t dtype, const void* x, int32_t N, int32_t C, int32_t L,
                    const float* running_mean, const float* running_var, float eps, const float* gamma,
                    const float* beta, int32_t act, void* y, void* stream) {
  OCM_REQUIRE(ctx && x && y && running_mean && running_var, "ocm_bn_fwd_eval: NULL argument");
  OCM_REQUIRE(N > 0 && C > 0 && L > 0, "ocm_bn_fwd_eval: bad shape");
  OCM_REQUIRE(act == OCM_ACT_NONE || act == OCM_ACT_ELU, "ocm_bn_fwd_eval: act must be OCM_ACT_NONE or OCM_ACT_ELU");
  OCM_REQUIRE(dtype == OCM_DTYPE_F32 || dtype == OCM_DTYPE_BF16, "ocm_bn_fwd_eval: dtype must be OCM_DTYPE_F32 or OCM_DTYPE_BF16");
  hipStream_t st = (hipStream_t)stream;
  const bool v8 = L % 8 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0 && (reinterpret_cast<uintptr_t>(y) & 15) == 0;
  const int64_t items = (int64_t)N * C * (v8 ? L / 8 : L);
  const dim3 g((unsigned)((items + BN_T - 1) / BN_T));
#define OCM_BN_EV(T, E, V)                                                                                          \
  hipLaunchKernelGGL((k_bn_eval<T, E, V>), g, dim3(BN_T), 0, st, static_cast<const T*>(x), C, L, items, running_mean, \
                     running_var, eps, gamma, beta, static_cast<T*>(y))
#define OCM_BN_EV2(T, E) \
  do {                   \
    if (v8) OCM_BN_EV(T, E, 8); else OCM_BN_EV(T, E, 1); \
  } while (0)
  const bool elu = act == OCM_ACT_ELU;
  if (dtype == OCM_DTYPE_F32) {
    if (elu) OCM_BN_EV2(float, true); else OCM_BN_EV2(float, false);
  } else {
    if (elu) OCM_BN_EV2(bf16_t, true); else OCM_BN_EV2(bf16_t, false);
  }
#undef OCM_BN_EV2
#undef OCM_BN_EV
  OCM_CHECK_LAUNCH("k_bn_eval");
  return OCM_OK;
}

int ocm_bn_bwd(ocm_ctx* ctx, int32_t dtype, const void* x, const void* dy, int32_t N, int32_t C, int32_t L,
               const float* gamma, const float* save_mean, const float* save_invstd, int32_t act, const void* y,
               void* dx, float* dgamma, float* dbeta, void* scratch, void* stream) {
  OCM_REQUIRE(ctx && x && dy && dx && save_mean && save_invstd && scratch, "ocm_bn_bwd: NULL argument");
  OCM_REQUIRE(N > 0 && C > 0 && L > 0 && (int64_t)N * L < INT32_MAX, "ocm_bn_bwd: bad shape");
  OCM_REQUIRE(act == OCM_ACT_NONE || (act == OCM_ACT_ELU && y), "ocm_bn_bwd: the fused ELU needs its output y");
  hipStream_t st = (hipStream_t)stream;
  const bool elu = act == OCM_ACT_ELU;
  if (dtype == OCM_DTYPE_F32)
    return elu ? bn_bwd<float, true>(ctx, x, dy, y, N, C, L, gamma, save_mean, save_invstd, dx, dgamma, dbeta,
                                     scratch, st)
               : bn_bwd<float, false>(ctx, x, dy, y, N, C, L, gamma, save_mean, save_invstd, dx, dgamma, dbeta,
                                      scratch, st);
  if (dtype == OCM_DTYPE_BF16)
    return elu ? bn_bwd<bf16_t, true>(ctx, x, dy, y, N, C, L, gamma, save_mean, save_invstd, dx, dgamma, dbeta,
                                      scratch, st)
               : bn_bwd<bf16_t, false>(ctx, x, dy, y, N, C, L, gamma, save_mean, save_invstd, dx, dgamma, dbeta,
                                       scratch, st);
  return ocm::fail(OCM_ERR_ARG, "ocm_bn_bwd: dtype must be OCM_DTYPE_F32 or OCM_DTYPE_BF16");
}

}  // extern "C"
