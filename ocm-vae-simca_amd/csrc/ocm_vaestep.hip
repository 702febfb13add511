// The small tensors of the VAE training step (vae_model.py:136-158,
// vae_bce_nut.py:178-203; utils/final_vaesimca.py:198-224, 362-375) fused
// into a few launches: the graphed C4 step is bound by its kernel count (each
// torch elementwise kernel costs ≈ 4.5 µs of the replay however small its
// tensor, profiles/r03n_vae_step_trace_by_grid.md), not by its bytes.
//
//   ocm_vae_bottleneck_fwd   z = μ + ε·exp(½ logσ²)  and  kl = −½ mean_B Σ_d (1 + logσ² − μ² − σ²)
//   ocm_vae_bottleneck_bwd   dμ = dz + dkl·μ/B,  dlogσ² = dz·ε·½exp(½logσ²) − ½dkl·(1 − σ²)/B
//   ocm_vae_recon_fwd        x̂ = xs·std + mean (the de-standardisation), the reconstruction term
//                            (BCE-with-logits vs the per-sample min–max scaled x, or MSE), total =
//                            recon + β·kl, and d total/d xs kept for the backward
//   ocm_vae_recon_bwd        dxs = dtotal·(d total/d xs), dkl = β·dtotal
//   ocm_adam_step            torch.optim.Adam (L2 weight decay, no amsgrad) over a table of tensors
//
// Sums are fp64 with per-workgroup partials combined in a fixed order by the
// last workgroup (a ticket counter): deterministic, graph-capturable (all
// scratch is caller-owned).
#include "ocm_internal.h"

namespace {

constexpr int VT = 256;

__device__ __forceinline__ float ld_act(const void* p, int dt, int64_t i) {
  if (dt == OCM_DTYPE_BF16) {
    const uint16_t h = static_cast<const uint16_t*>(p)[i];
    return __uint_as_float((uint32_t)h << 16);
  }
  return static_cast<const float*>(p)[i];
}

__device__ __forceinline__ void st_act(void* p, int dt, int64_t i, float v) {
  if (dt == OCM_DTYPE_BF16) {  // round to nearest even
    uint32_t u = __float_as_uint(v);
    if ((u & 0x7f800000u) != 0x7f800000u) u += 0x7fffu + ((u >> 16) & 1u);
    static_cast<uint16_t*>(p)[i] = (uint16_t)(u >> 16);
  } else {
    static_cast<float*>(p)[i] = v;
  }
}

__device__ __forceinline__ double block_sum_d(double v, double* red) {
  v = wave_sum_f64(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  double s = 0.0;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) s += red[w];
  return s;
}

__device__ __forceinline__ float block_minmax(float v, bool is_max, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float u = __shfl_xor(v, o, 64);
    v = is_max ? fmaxf(v, u) : fminf(v, u);
  }
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  float r = red[0];
  for (int w = 1; w < (int)(blockDim.x >> 6); ++w) r = is_max ? fmaxf(r, red[w]) : fminf(r, red[w]);
  return r;
}

// z and the KL: one element per thread, the workgroups' KL partials summed
// by the last one (ocm_internal.h last_arrival2)
// μ / logσ² (and their gradients) are rows of stride ld (ld = d: separate
// tensors; ld = 2d, logσ² = μ + d: the packed output of one [fc_mu; fc_logvar]
// product); z, ε, dz are B×d
__global__ __launch_bounds__(VT) void k_bottleneck_fwd(const void* mu, const void* lv, int ld, const void* eps, int dt,
                                                        int64_t n, int B, int d, void* z, float* kl, double* part,
                                                        unsigned* ticket) {
  __shared__ double red[VT / 64];
  const int64_t i = (int64_t)blockIdx.x * VT + threadIdx.x;
  double s = 0.0;
  if (i < n) {
    const int64_t r = i / d, j = r * ld + (i - r * d);
    const float m = ld_act(mu, dt, j), l = ld_act(lv, dt, j), e = ld_act(eps, dt, i);
    st_act(z, dt, i, m + e * expf(0.5f * l));
    s = 1.0 + (double)l - (double)m * m - exp((double)l);
  }
  const double ps = block_sum_d(s, red);
  if (threadIdx.x == 0) st_agent(part + blockIdx.x, ps);
  if (!last_arrival2(ticket, 0, gridDim.x, blockIdx.x)) return;
  const double t = threadIdx.x < 64 ? lane_sum_agent<double, double>(part, 1, (int)gridDim.x, threadIdx.x) : 0.0;
  const double tot = block_sum_d(t, red);
  if (threadIdx.x == 0) *kl = (float)(-0.5 * tot / B);
}

__global__ __launch_bounds__(VT) void k_bottleneck_bwd(const void* dz, const float* dkl, const void* mu,
                                                        const void* lv, int ld, const void* eps, int dt, int64_t n,
                                                        int B, int d, void* dmu, void* dlv) {
  const int64_t i = (int64_t)blockIdx.x * VT + threadIdx.x;
  if (i >= n) return;
  const int64_t r = i / d, j = r * ld + (i - r * d);
  const float g = dz ? ld_act(dz, dt, i) : 0.f;
  const float k = dkl ? *dkl : 0.f;
  const float m = ld_act(mu, dt, j), l = ld_act(lv, dt, j), e = ld_act(eps, dt, i);
  st_act(dmu, dt, j, g + k * m / B);
  st_act(dlv, dt, j, g * e * 0.5f * expf(0.5f * l) - 0.5f * k * (1.f - expf(l)) / B);
}

// one workgroup per row: x̂ = xs·std + mean; BCE-with-logits against t =
// clamp((x − lo)/(hi − lo + eps), 0, 1) (torch's stable form) or MSE; the
// gradient (d recon/d xs) into gxs; row partials → the last workgroup sums
// them in order and writes {total, recon}.
__global__ __launch_bounds__(VT) void k_recon_fwd(int kind, const float* __restrict__ x, const void* xs, int dt,
                                                   int B, int L, const float* __restrict__ mean,
                                                   const float* __restrict__ sd, float eps, const float* kl,
                                                   float beta, float* __restrict__ gxs, double* __restrict__ part,
                                                   unsigned* __restrict__ ticket, float* __restrict__ out) {
  __shared__ float redf[VT / 64];
  __shared__ double red[VT / 64];
  const int b = blockIdx.x;
  const float* xr = x + (int64_t)b * L;
  const double inv = 1.0 / ((double)B * L);
  // the row's values in registers, every load of a pass issued together (RP
  // per thread covers L ≤ RP·VT; longer rows stream through the same code in
  // RP·VT pieces, each loaded twice)
  constexpr int RP = 8;
  float lo = 0.f, den = 1.f;
  if (kind == OCM_VAE_LOSS_BCE) {
    float mn = __builtin_inff(), mx = -__builtin_inff();
    for (int j0 = threadIdx.x; j0 < L; j0 += RP * VT) {
      float v[RP];
#pragma unroll
      for (int r = 0; r < RP; ++r) {
        const int j = j0 + r * VT;
        v[r] = xr[j < L ? j : 0];
      }
#pragma unroll
      for (int r = 0; r < RP; ++r)
        if (j0 + r * VT < L) {
          mn = fminf(mn, v[r]);
          mx = fmaxf(mx, v[r]);
        }
    }
    lo = block_minmax(mn, false, redf);
    const float hi = block_minmax(mx, true, redf);
    den = hi - lo + eps;
  }
  double s = 0.0;
  for (int j0 = threadIdx.x; j0 < L; j0 += RP * VT) {
    float xv[RP], zv[RP], sv[RP];
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      const int j = j0 + r * VT, jc = j < L ? j : 0;
      xv[r] = xr[jc];
      sv[r] = sd[jc];
      zv[r] = ld_act(xs, dt, (int64_t)b * L + jc) * sv[r] + mean[jc];
    }
#pragma unroll
    for (int r = 0; r < RP; ++r) {
      const int j = j0 + r * VT;
      if (j >= L) continue;
      const float z = zv[r];
      float g;
      if (kind == OCM_VAE_LOSS_BCE) {
        const float t = fminf(fmaxf((xv[r] - lo) / den, 0.f), 1.f);
        s += (double)(fmaxf(z, 0.f) - z * t + log1pf(expf(-fabsf(z))));
        const float sg = 1.f / (1.f + expf(-z));
        g = (float)((double)(sg - t) * inv);
      } else {  // MSE
        const float d = z - xv[r];
        s += (double)d * d;
        g = (float)(2.0 * d * inv);
      }
      gxs[(int64_t)b * L + j] = g * sv[r];
    }
  }
  const double ps = block_sum_d(s, red);
  if (threadIdx.x == 0) st_agent(part + b, ps);  // write-through (ocm_internal.h last_arrival)
  // two-level counter: B = 512 arrivals at one counter queue up at the atomic unit
  if (!last_arrival2(ticket, 0, gridDim.x, blockIdx.x)) return;
  const double t = threadIdx.x < 64 ? lane_sum_agent<double, double>(part, 1, (int)gridDim.x, threadIdx.x) : 0.0;
  const double tot = block_sum_d(t, red);
  if (threadIdx.x == 0) {
    const float recon = (float)(tot * inv);
    out[1] = recon;
    out[0] = recon + beta * (kl ? *kl : 0.f);
  }
}

__global__ __launch_bounds__(VT) void k_recon_bwd(const float* __restrict__ dtotal, const float* __restrict__ gxs,
                                                   int64_t n, int dt, void* dxs, float beta, float* dkl) {
  const int64_t i = (int64_t)blockIdx.x * VT + threadIdx.x;
  const float g = *dtotal;
  if (i < n) st_act(dxs, dt, i, g * gxs[i]);
  if (i == 0 && dkl) *dkl = beta * g;
}

// Adam over a table of tensors: each thread takes ADAM_U elements of the
// concatenation (the prefix of element counts in the table), all their loads
// before any arithmetic; the tensor of an element is found by binary search
// in an LDS copy of the offsets (a linear walk through the table in global
// memory cost one memory latency per step); the step counter (f32, on the
// device) is read as t − 1 and advanced by the last workgroup.
constexpr int ADAM_U = 4, ADAM_TMAX = 256;
__global__ __launch_bounds__(VT) void k_adam(const ocm_adam_tensor* __restrict__ tab, int nt, int64_t total,
                                              float* __restrict__ step, float lr, float b1, float b2, float eps,
                                              float wd, unsigned* __restrict__ ticket) {
  __shared__ int64_t offs[ADAM_TMAX];
  for (int k = threadIdx.x; k < nt; k += VT) offs[k] = tab[k].offset;
  __syncthreads();
  const float t = *step + 1.f;
  const float bc1 = 1.f - powf(b1, t), bc2 = 1.f - powf(b2, t);
  const float step_size = lr / bc1, bc2s = sqrtf(bc2);
  const int64_t stride = (int64_t)gridDim.x * VT;
  for (int64_t i0 = (int64_t)blockIdx.x * VT + threadIdx.x; i0 < total; i0 += ADAM_U * stride) {
    float* pp[ADAM_U];
    float* mp[ADAM_U];
    float* vp[ADAM_U];
    float g[ADAM_U], pv[ADAM_U], m[ADAM_U], v[ADAM_U];
#pragma unroll
    for (int r = 0; r < ADAM_U; ++r) {
      const int64_t i = i0 + r * stride;
      const int64_t ic = i < total ? i : total - 1;
      int lo = 0, hi = nt - 1;  // the last tensor whose offset ≤ ic
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (offs[mid] <= ic) lo = mid; else hi = mid - 1;
      }
      const ocm_adam_tensor& T = tab[lo];
      const int64_t j = ic - offs[lo];
      pp[r] = T.param + j;
      mp[r] = T.exp_avg + j;
      vp[r] = T.exp_avg_sq + j;
      g[r] = T.grad[j];
      pv[r] = *pp[r];
      m[r] = *mp[r];
      v[r] = *vp[r];
    }
#pragma unroll
    for (int r = 0; r < ADAM_U; ++r) {
      if (i0 + r * stride >= total) continue;
      float gr = g[r];
      if (wd != 0.f) gr += wd * pv[r];
      const float mm = b1 * m[r] + (1.f - b1) * gr;
      const float vv = b2 * v[r] + (1.f - b2) * gr * gr;
      *mp[r] = mm;
      *vp[r] = vv;
      *pp[r] = pv[r] - step_size * mm / (sqrtf(vv) / bc2s + eps);
    }
  }
  // the last workgroup advances the counter: every workgroup read it before
  // its own arrival (no data hand-off, so no fence); two-level counters (≈ 800
  // arrivals at one counter queue up at the atomic unit)
  if (last_arrival2(ticket, 0, gridDim.x, blockIdx.x) && threadIdx.x == 0) *step = t;
}

// up to CAST_MAX tensors converted in one launch (the arguments by value:
// graph-capturable without a device table)
constexpr int CAST_MAX = 32;
struct CastArgs {
  const void* src[CAST_MAX];
  void* dst[CAST_MAX];
  int64_t end[CAST_MAX];  // prefix sums of the element counts
  int n;
};
__global__ __launch_bounds__(VT) void k_cast_multi(CastArgs a, int sdt, int ddt) {
  const int64_t total = a.end[a.n - 1];
  int cur = 0;
  for (int64_t i = (int64_t)blockIdx.x * VT + threadIdx.x; i < total; i += (int64_t)gridDim.x * VT) {
    while (i >= a.end[cur]) ++cur;
    const int64_t j = i - (cur ? a.end[cur - 1] : 0);
    st_act(a.dst[cur], ddt, j, ld_act(a.src[cur], sdt, j));
  }
}

// xs = (x − mean) / std, per column of a B×L float32 matrix, written in dtype
__global__ __launch_bounds__(VT) void k_standardise(const float* __restrict__ x, const float* __restrict__ mean,
                                                     const float* __restrict__ sd, int64_t n, int L, int dt,
                                                     void* out) {
  const int64_t i = (int64_t)blockIdx.x * VT + threadIdx.x;
  if (i >= n) return;
  const int j = (int)(i % L);
  st_act(out, dt, i, (x[i] - mean[j]) / sd[j]);
}

// A Linear layer's backward tail (vae_model.py:80-84, fc / fc_dec: Linear →
// ELU, and fc_mu / fc_logvar: Linear alone), bf16: gy = g·elu'(y) (torch's
// elu_backward on the pre-activation y, in float32, rounded to bf16) and the
// bias gradient Σ_rows gy (float32 over the rounded gy, fixed order, rounded
// to bf16) in one pass, instead of torch's elu_backward and sum kernels.
// Workgroup: 32 columns × 256 row lanes (N = 6144: 192 workgroups); a thread
// takes 8 contiguous columns (one 16-byte load per row) of rows rl, rl + 256,
// …; the 16 row lanes of a wave that share a column group are summed by
// shuffles, the 16 waves in LDS.
constexpr int AB_T = 1024, AB_CG = 4, AB_RL = AB_T / AB_CG, AB_U = 2;
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }
__device__ __forceinline__ uint32_t bf_rne(float v) {  // the bf16 bits of v, round to nearest even
  uint32_t u = __float_as_uint(v);
  if ((u & 0x7f800000u) != 0x7f800000u) u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}
template <int ACT>
__global__ __launch_bounds__(AB_T) void k_act_bias_bwd(const uint16_t* __restrict__ g, const uint16_t* __restrict__ y,
                                                       int B, int N, uint16_t* __restrict__ gy,
                                                       uint16_t* __restrict__ gb) {
  __shared__ float red[AB_T / 64][AB_CG * 8];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int cg = lane & (AB_CG - 1);
  const int rl = wave * (64 / AB_CG) + lane / AB_CG;
  const int c0 = (blockIdx.x * AB_CG + cg) * 8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c0 < N) {
    // AB_U rows per pass, their loads issued together (B = 512: one pass)
    for (int rb = rl; rb < B; rb += AB_U * AB_RL) {
      uint4 gv[AB_U], yv[AB_U];
#pragma unroll
      for (int u = 0; u < AB_U; ++u) {
        const int r = rb + u * AB_RL;
        gv[u] = r < B ? *reinterpret_cast<const uint4*>(g + (int64_t)r * N + c0) : make_uint4(0, 0, 0, 0);
        if (ACT) yv[u] = r < B ? *reinterpret_cast<const uint4*>(y + (int64_t)r * N + c0) : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < AB_U; ++u) {
        const int r = rb + u * AB_RL;
        const uint32_t gw[4] = {gv[u].x, gv[u].y, gv[u].z, gv[u].w};
        float v[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[2 * k] = bf_lo(gw[k]);
          v[2 * k + 1] = bf_hi(gw[k]);
        }
        if (ACT) {
          const uint32_t yw[4] = {yv[u].x, yv[u].y, yv[u].z, yv[u].w};
          uint32_t o[4];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const float y0 = bf_lo(yw[k]), y1 = bf_hi(yw[k]);
            const uint32_t r0 = bf_rne(y0 > 0.f ? v[2 * k] : v[2 * k] * expf(y0));
            const uint32_t r1 = bf_rne(y1 > 0.f ? v[2 * k + 1] : v[2 * k + 1] * expf(y1));
            v[2 * k] = __uint_as_float(r0 << 16);
            v[2 * k + 1] = __uint_as_float(r1 << 16);
            o[k] = r0 | (r1 << 16);
          }
          if (r < B) *reinterpret_cast<uint4*>(gy + (int64_t)r * N + c0) = make_uint4(o[0], o[1], o[2], o[3]);
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) s[k] += v[k];  // rows past B loaded as zeros
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
#pragma unroll
    for (int o = AB_CG; o < 64; o <<= 1) s[k] += __shfl_xor(s[k], o, 64);
  }
  if (lane < AB_CG) {
#pragma unroll
    for (int k = 0; k < 8; ++k) red[wave][lane * 8 + k] = s[k];
  }
  __syncthreads();
  if (threadIdx.x < AB_CG * 8) {
    const int c = blockIdx.x * AB_CG * 8 + threadIdx.x;
    if (c < N) {
      float t = 0.f;
      for (int w = 0; w < AB_T / 64; ++w) t += red[w][threadIdx.x];
      gb[c] = (uint16_t)bf_rne(t);
    }
  }
}

// Split-K bf16 GEMM for the bottleneck's long-K products (vae_model.py:80-84):
// C (M×N, bf16) = A (M×K) · B (+ bias), B given as N×K (BT: a Linear weight in
// the forward, y = x·Wᵀ) or as K×N (BN: the weight in the input gradient,
// gx = gy·W); M and N multiples of 64, K of 256.  hipBLASLt runs these shapes
// with a few workgroups that each walk all of K (fc_dec[3]'s input gradient,
// 512×64 over K = 6144: 20.6 µs; fc[0]'s forward 8.5 µs,
// profiles/r06zf_vae_gemm_calls.txt).  Here one workgroup takes a 64×64 tile
// and one 256-deep chunk of K on v_mfma_f32_16x16x32_bf16 (wave w: rows
// 16w..16w+15, four 16-column tiles; A fragments straight from memory, BN's
// chunk staged transposed in LDS), the accumulators flushed into f32 running
// sums every 128 products; the f32 partial tiles go to caller-owned scratch and
// k_gemm_sk_reduce sums them in chunk order, adds the bias and rounds to bf16.
constexpr int SK_KC = 256, SK_PAD = 8;
using sk_bf16x8 = __attribute__((ext_vector_type(8))) short;
template <bool BT>
__global__ __launch_bounds__(256) void k_gemm_sk(const uint16_t* __restrict__ A, const uint16_t* __restrict__ B, int M,
                                                 int N, int K, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) uint16_t Bs[BT ? 1 : 64][SK_KC + SK_PAD];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n16 = lane & 15, kg = lane >> 4;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64, k0 = blockIdx.z * SK_KC;
  if (!BT) {  // B[k0 .. k0 + 255][n0 .. n0 + 63] → Bs[n][k]
#pragma unroll
    for (int r = 0; r < SK_KC * 64 / 8 / 256; ++r) {
      const int e = tid + 256 * r, k = e >> 3, nn = (e & 7) * 8;
      const uint4 v = *reinterpret_cast<const uint4*>(B + (int64_t)(k0 + k) * N + n0 + nn);
      const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        Bs[nn + 2 * j][k] = (uint16_t)(wv[j] & 0xffffu);
        Bs[nn + 2 * j + 1][k] = (uint16_t)(wv[j] >> 16);
      }
    }
    __syncthreads();
  }
  f32x4 acc[4], run[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) acc[nt] = run[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  const uint16_t* arow = A + (int64_t)(m0 + 16 * w + n16) * K + k0 + 8 * kg;
#pragma unroll
  for (int ks = 0; ks < SK_KC / 32; ++ks) {
    const sk_bf16x8 a = __builtin_bit_cast(sk_bf16x8, *reinterpret_cast<const f32x4*>(arow + 32 * ks));
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const int kk = 32 * ks + 8 * kg;
      const f32x4 bv = BT ? *reinterpret_cast<const f32x4*>(B + (int64_t)(n0 + 16 * nt + n16) * K + k0 + kk)
                          : *reinterpret_cast<const f32x4*>(&Bs[BT ? 0 : 16 * nt + n16][kk]);
      acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, __builtin_bit_cast(sk_bf16x8, bv), acc[nt], 0, 0, 0);
    }
    if ((ks & 3) == 3) {
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        run[nt] += acc[nt];
        acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
  // D layout: column 16·nt + (lane & 15), rows 4·(lane >> 4) + r
  float* P = part + (int64_t)blockIdx.z * M * N;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) P[(int64_t)(m0 + 16 * w + 4 * kg + r) * N + n0 + 16 * nt + n16] = run[nt][r];
}

__global__ __launch_bounds__(VT) void k_gemm_sk_reduce(const float* __restrict__ part, int S, int64_t MN, int N,
                                                       const uint16_t* __restrict__ bias, uint16_t* __restrict__ C) {
  const int64_t i = (int64_t)blockIdx.x * VT + threadIdx.x;
  if (i >= MN) return;
  float t = 0.f;
  int s = 0;
  for (; s + 8 <= S; s += 8) {  // eight loads in flight, added in chunk order
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(int64_t)(s + u) * MN + i];
#pragma unroll
    for (int u = 0; u < 8; ++u) t += v[u];
  }
  for (; s < S; ++s) t += part[(int64_t)s * MN + i];
  if (bias) t += __uint_as_float((uint32_t)bias[i % N] << 16);
  C[i] = (uint16_t)bf_rne(t);
}

// The bottleneck's short-K Linear layers with their ELU (vae_model.py:83-84,
// fc_dec: K = 32 and 64): y = x·Wᵀ + b and a = ELU(y) in one launch, where
// hipBLASLt's GEMM + torch's ELU took two (≈ 5 + 4.5 µs each,
// profiles/r06zj_vae_step_trace.md).  One 64×64 tile per workgroup on
// v_mfma_f32_16x16x32_bf16 (wave w: rows 16w..16w+15, four 16-column tiles),
// the whole K in registers; y is rounded to bf16 (as the GEMM's output) and
// the ELU — torch's expm1 form — is taken of the rounded value, so a matches
// torch's elu of the bf16 y.  y (the backward's ELU input) and a are written.
template <int KS>
__global__ __launch_bounds__(256) void k_linear_act(const uint16_t* __restrict__ X, const uint16_t* __restrict__ W,
                                                    const uint16_t* __restrict__ bias, int N,
                                                    uint16_t* __restrict__ Y, uint16_t* __restrict__ Aout) {
  constexpr int K = 32 * KS;
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, n16 = lane & 15, kg = lane >> 4;
  const int m0 = blockIdx.x * 64, n0 = blockIdx.y * 64;
  const uint16_t* arow = X + (int64_t)(m0 + 16 * w + n16) * K + 8 * kg;
  sk_bf16x8 a[KS], b[4][KS];
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) a[ks] = __builtin_bit_cast(sk_bf16x8, *reinterpret_cast<const f32x4*>(arow + 32 * ks));
#pragma unroll
  for (int nt = 0; nt < 4; ++nt)
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
      b[nt][ks] = __builtin_bit_cast(
          sk_bf16x8, *reinterpret_cast<const f32x4*>(W + (int64_t)(n0 + 16 * nt + n16) * K + 32 * ks + 8 * kg));
  float bv[4];
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) bv[nt] = bias ? __uint_as_float((uint32_t)bias[n0 + 16 * nt + n16] << 16) : 0.f;
#pragma unroll
  for (int nt = 0; nt < 4; ++nt) {
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[ks], b[nt][ks], acc, 0, 0, 0);
    // D layout: column 16·nt + (lane & 15), rows 4·(lane >> 4) + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t o = (int64_t)(m0 + 16 * w + 4 * kg + r) * N + n0 + 16 * nt + n16;
      const uint32_t yb = bf_rne(acc[r] + bv[nt]);
      const float y = __uint_as_float(yb << 16);
      Y[o] = (uint16_t)yb;
      Aout[o] = (uint16_t)bf_rne(y > 0.f ? y : expm1f(y));
    }
  }
}

}  // namespace

extern "C" {

int ocm_vae_linear_act(ocm_ctx* ctx, const void* x, const void* W, const void* bias, int32_t M, int32_t N, int32_t K,
                       void* y_out, void* a_out, void* stream) {
  OCM_REQUIRE(ctx && x && W && y_out && a_out, "ocm_vae_linear_act: NULL argument");
  OCM_REQUIRE(M > 0 && N > 0 && M % 64 == 0 && N % 64 == 0 && (K == 32 || K == 64 || K == 128 || K == 256),
              "ocm_vae_linear_act: M, N multiples of 64, K ∈ {32, 64, 128, 256}");
  OCM_REQUIRE(((uintptr_t)x | (uintptr_t)W) % 16 == 0, "ocm_vae_linear_act: 16-byte aligned x and W");
  OCM_REQUIRE(M / 64 <= 65535 && N / 64 <= 65535, "ocm_vae_linear_act: M, N ≤ 64·65535");
  const dim3 g((unsigned)(M / 64), (unsigned)(N / 64));
  const auto* xp = static_cast<const uint16_t*>(x);
  const auto* wp = static_cast<const uint16_t*>(W);
  const auto* bp = static_cast<const uint16_t*>(bias);
  auto* yp = static_cast<uint16_t*>(y_out);
  auto* ap = static_cast<uint16_t*>(a_out);
  hipStream_t st = (hipStream_t)stream;
  if (K == 32) hipLaunchKernelGGL(k_linear_act<1>, g, dim3(256), 0, st, xp, wp, bp, N, yp, ap);
  else if (K == 64) hipLaunchKernelGGL(k_linear_act<2>, g, dim3(256), 0, st, xp, wp, bp, N, yp, ap);
  else if (K == 128) hipLaunchKernelGGL(k_linear_act<4>, g, dim3(256), 0, st, xp, wp, bp, N, yp, ap);
  else hipLaunchKernelGGL(k_linear_act<8>, g, dim3(256), 0, st, xp, wp, bp, N, yp, ap);
  OCM_CHECK_LAUNCH("k_linear_act");
  return OCM_OK;
}

size_t ocm_gemm_bf16_sk_scratch_bytes(int32_t M, int32_t N, int32_t K) {
  return (size_t)(K / SK_KC) * (size_t)M * (size_t)N * sizeof(float);
}

int ocm_gemm_bf16_sk(ocm_ctx* ctx, int32_t b_nk, const void* A, const void* B, const void* bias, int32_t M, int32_t N,
                     int32_t K, void* C, void* scratch, void* stream) {
  OCM_REQUIRE(ctx && A && B && C && scratch, "ocm_gemm_bf16_sk: NULL argument");
  OCM_REQUIRE(M > 0 && N > 0 && K > 0 && M % 64 == 0 && N % 64 == 0 && K % SK_KC == 0,
              "ocm_gemm_bf16_sk: M, N multiples of 64, K of 256");
  OCM_REQUIRE(((uintptr_t)A | (uintptr_t)B | (uintptr_t)C) % 16 == 0, "ocm_gemm_bf16_sk: 16-byte aligned operands");
  const int S = K / SK_KC;
  OCM_REQUIRE(S <= 65535, "ocm_gemm_bf16_sk: K ≤ 256·65535");
  const dim3 grid((unsigned)(M / 64), (unsigned)(N / 64), (unsigned)S);
  auto* part = static_cast<float*>(scratch);
  const auto* a = static_cast<const uint16_t*>(A);
  const auto* bm = static_cast<const uint16_t*>(B);
  if (b_nk)
    hipLaunchKernelGGL(k_gemm_sk<true>, grid, dim3(256), 0, (hipStream_t)stream, a, bm, M, N, K, part);
  else
    hipLaunchKernelGGL(k_gemm_sk<false>, grid, dim3(256), 0, (hipStream_t)stream, a, bm, M, N, K, part);
  OCM_CHECK_LAUNCH("k_gemm_sk");
  const int64_t MN = (int64_t)M * N;
  hipLaunchKernelGGL(k_gemm_sk_reduce, dim3((unsigned)((MN + VT - 1) / VT)), dim3(VT), 0, (hipStream_t)stream, part, S,
                     MN, N, static_cast<const uint16_t*>(bias), static_cast<uint16_t*>(C));
  OCM_CHECK_LAUNCH("k_gemm_sk_reduce");
  return OCM_OK;
}

int ocm_vae_act_bias_bwd(ocm_ctx* ctx, int32_t act, const void* g, const void* y, int32_t B, int32_t N, void* gy_out,
                         void* gbias_out, void* stream) {
  OCM_REQUIRE(ctx && g && gbias_out && (act == 0 || (y && gy_out)), "ocm_vae_act_bias_bwd: NULL argument");
  OCM_REQUIRE(act == 0 || act == 1, "ocm_vae_act_bias_bwd: act 0 (none) or 1 (ELU)");
  OCM_REQUIRE(B > 0 && N > 0 && N % 8 == 0, "ocm_vae_act_bias_bwd: B > 0, N a positive multiple of 8");
  OCM_REQUIRE(((uintptr_t)g | (uintptr_t)(act ? y : g) | (uintptr_t)(act ? gy_out : g)) % 16 == 0,
              "ocm_vae_act_bias_bwd: 16-byte aligned rows");
  const dim3 grid((unsigned)((N + AB_CG * 8 - 1) / (AB_CG * 8)));
  const auto* gp = static_cast<const uint16_t*>(g);
  if (act)
    hipLaunchKernelGGL(k_act_bias_bwd<1>, grid, dim3(AB_T), 0, (hipStream_t)stream, gp,
                       static_cast<const uint16_t*>(y), B, N, static_cast<uint16_t*>(gy_out),
                       static_cast<uint16_t*>(gbias_out));
  else
    hipLaunchKernelGGL(k_act_bias_bwd<0>, grid, dim3(AB_T), 0, (hipStream_t)stream, gp, nullptr, B, N, nullptr,
                       static_cast<uint16_t*>(gbias_out));
  OCM_CHECK_LAUNCH("k_act_bias_bwd");
  return OCM_OK;
}

int ocm_cast_multi(ocm_ctx* ctx, int32_t n, const void* const* src, int32_t src_dtype, void* const* dst,
                   int32_t dst_dtype, const int64_t* numel, void* stream) {
  OCM_REQUIRE(ctx && src && dst && numel, "ocm_cast_multi: NULL argument");
  OCM_REQUIRE(n >= 0 && n <= CAST_MAX, "ocm_cast_multi: at most 32 tensors");
  OCM_REQUIRE((src_dtype == OCM_DTYPE_F32 || src_dtype == OCM_DTYPE_BF16) &&
                  (dst_dtype == OCM_DTYPE_F32 || dst_dtype == OCM_DTYPE_BF16),
              "ocm_cast_multi: float32 / bfloat16");
  CastArgs a{};
  int64_t t = 0;
  int m = 0;
  for (int k = 0; k < n; ++k) {
    OCM_REQUIRE(numel[k] >= 0 && (numel[k] == 0 || (src[k] && dst[k])), "ocm_cast_multi: bad tensor");
    if (numel[k] == 0) continue;
    t += numel[k];
    a.src[m] = src[k];
    a.dst[m] = dst[k];
    a.end[m] = t;
    ++m;
  }
  a.n = m;
  if (m == 0) return OCM_OK;
  const int64_t blocks = std::min<int64_t>((t + VT - 1) / VT, 4 * (int64_t)ctx->num_cus);
  hipLaunchKernelGGL(k_cast_multi, dim3((unsigned)blocks), dim3(VT), 0, (hipStream_t)stream, a, src_dtype,
                     dst_dtype);
  OCM_CHECK_LAUNCH("k_cast_multi");
  return OCM_OK;
}

int ocm_vae_standardise(ocm_ctx* ctx, const float* x, int32_t B, int32_t L, const float* mean, const float* std_,
                        int32_t dtype, void* out, void* stream) {
  OCM_REQUIRE(ctx && x && mean && std_ && out, "ocm_vae_standardise: NULL argument");
  OCM_REQUIRE(B > 0 && L > 0 && (dtype == OCM_DTYPE_F32 || dtype == OCM_DTYPE_BF16), "ocm_vae_standardise: bad args");
  const int64_t n = (int64_t)B * L;
  hipLaunchKernelGGL(k_standardise, dim3((unsigned)((n + VT - 1) / VT)), dim3(VT), 0, (hipStream_t)stream, x, mean,
                     std_, n, L, dtype, out);
  OCM_CHECK_LAUNCH("k_standardise");
  return OCM_OK;
}

size_t ocm_vae_scratch_bytes(int32_t B) {
  // row partials (B + 32 doubles), then the two-level completion counters
  return (size_t)(B + 32) * sizeof(double) + (size_t)tickets_per_slot(B) * TICKET_STRIDE * sizeof(unsigned) + 256;
}
size_t ocm_vae_bottleneck_scratch_bytes() { return 4096 * sizeof(double) + tickets_per_slot(4096) * TICKET_STRIDE * sizeof(unsigned); }

int ocm_vae_bottleneck_fwd(ocm_ctx* ctx, int32_t dtype, const void* mu, const void* logvar, const void* eps, int32_t B,
                           int32_t d, void* z_out, float* kl_out, void* scratch, void* stream) {
  return ocm_vae_bottleneck_fwd_ld(ctx, dtype, mu, logvar, d, eps, B, d, z_out, kl_out, scratch, stream);
}

int ocm_vae_bottleneck_fwd_ld(ocm_ctx* ctx, int32_t dtype, const void* mu, const void* logvar, int32_t ld,
                              const void* eps, int32_t B, int32_t d, void* z_out, float* kl_out, void* scratch,
                              void* stream) {
  OCM_REQUIRE(ctx && mu && logvar && eps && z_out && kl_out && scratch, "ocm_vae_bottleneck_fwd: NULL argument");
  OCM_REQUIRE(B > 0 && d > 0 && ld >= d && (dtype == OCM_DTYPE_F32 || dtype == OCM_DTYPE_BF16),
              "ocm_vae_bottleneck_fwd: bad args");
  const int64_t n = (int64_t)B * d;
  const int64_t nb = (n + VT - 1) / VT;
  OCM_REQUIRE(nb <= 4096, "ocm_vae_bottleneck_fwd: B·d ≤ 2²⁰");
  auto* part = static_cast<double*>(scratch);
  auto* ticket = reinterpret_cast<unsigned*>(part + 4096);
  hipLaunchKernelGGL(k_bottleneck_fwd, dim3((unsigned)nb), dim3(VT), 0, (hipStream_t)stream, mu, logvar, ld, eps,
                     dtype, n, B, d, z_out, kl_out, part, ticket);
  OCM_CHECK_LAUNCH("k_bottleneck_fwd");
  return OCM_OK;
}

int ocm_vae_bottleneck_bwd(ocm_ctx* ctx, int32_t dtype, const void* dz, const float* dkl, const void* mu,
                           const void* logvar, const void* eps, int32_t B, int32_t d, void* dmu_out, void* dlogvar_out,
                           void* stream) {
  return ocm_vae_bottleneck_bwd_ld(ctx, dtype, dz, dkl, mu, logvar, d, eps, B, d, dmu_out, dlogvar_out, stream);
}

int ocm_vae_bottleneck_bwd_ld(ocm_ctx* ctx, int32_t dtype, const void* dz, const float* dkl, const void* mu,
                              const void* logvar, int32_t ld, const void* eps, int32_t B, int32_t d, void* dmu_out,
                              void* dlogvar_out, void* stream) {
  OCM_REQUIRE(ctx && mu && logvar && eps && dmu_out && dlogvar_out, "ocm_vae_bottleneck_bwd: NULL argument");
  OCM_REQUIRE(B > 0 && d > 0 && ld >= d && (dtype == OCM_DTYPE_F32 || dtype == OCM_DTYPE_BF16),
              "ocm_vae_bottleneck_bwd: bad args");
  const int64_t n = (int64_t)B * d;
  hipLaunchKernelGGL(k_bottleneck_bwd, dim3((unsigned)((n + VT - 1) / VT)), dim3(VT), 0, (hipStream_t)stream, dz, dkl,
                     mu, logvar, ld, eps, dtype, n, B, d, dmu_out, dlogvar_out);
  OCM_CHECK_LAUNCH("k_bottleneck_bwd");
  return OCM_OK;
}

int ocm_vae_recon_fwd(ocm_ctx* ctx, int32_t kind, const float* x, int32_t dtype, const void* xs, int32_t B, int32_t L,
                      const float* mean, const float* std, float eps, const float* kl, float beta, float* gxs_out,
                      float* out2, void* scratch, void* stream) {
  OCM_REQUIRE(ctx && x && xs && mean && std && gxs_out && out2 && scratch, "ocm_vae_recon_fwd: NULL argument");
  OCM_REQUIRE(kind == OCM_VAE_LOSS_BCE || kind == OCM_VAE_LOSS_MSE, "ocm_vae_recon_fwd: kind BCE or MSE");
  OCM_REQUIRE(B > 0 && L > 0 && (dtype == OCM_DTYPE_F32 || dtype == OCM_DTYPE_BF16), "ocm_vae_recon_fwd: bad args");
  auto* part = static_cast<double*>(scratch);
  auto* ticket = reinterpret_cast<unsigned*>(part + B + 32);
  hipLaunchKernelGGL(k_recon_fwd, dim3(B), dim3(VT), 0, (hipStream_t)stream, kind, x, xs, dtype, B, L, mean, std, eps,
                     kl, beta, gxs_out, part, ticket, out2);
  OCM_CHECK_LAUNCH("k_recon_fwd");
  return OCM_OK;
}

int ocm_vae_recon_bwd(ocm_ctx* ctx, const float* dtotal, const float* gxs, int64_t n, int32_t dtype, void* dxs_out,
                      float beta, float* dkl_out, void* stream) {
  OCM_REQUIRE(ctx && dtotal && gxs && dxs_out, "ocm_vae_recon_bwd: NULL argument");
  OCM_REQUIRE(n > 0 && (dtype == OCM_DTYPE_F32 || dtype == OCM_DTYPE_BF16), "ocm_vae_recon_bwd: bad args");
  hipLaunchKernelGGL(k_recon_bwd, dim3((unsigned)((n + VT - 1) / VT)), dim3(VT), 0, (hipStream_t)stream, dtotal, gxs, n,
                     dtype, dxs_out, beta, dkl_out);
  OCM_CHECK_LAUNCH("k_recon_bwd");
  return OCM_OK;
}

int ocm_adam_step(ocm_ctx* ctx, const ocm_adam_tensor* table, int32_t ntensors, int64_t total, float* step, float lr,
                  float beta1, float beta2, float eps, float weight_decay, void* scratch, void* stream) {
  OCM_REQUIRE(ctx && table && step && scratch && ntensors > 0 && ntensors <= ADAM_TMAX && total > 0,
              "ocm_adam_step: bad arguments (≤ 256 tensors)");
  const int grid = (int)std::min<int64_t>((total + ADAM_U * VT - 1) / (ADAM_U * VT), 4096);
  hipLaunchKernelGGL(k_adam, dim3(grid), dim3(VT), 0, (hipStream_t)stream, table, ntensors, total, step, lr, beta1,
                     beta2, eps, weight_decay, static_cast<unsigned*>(scratch));
  OCM_CHECK_LAUNCH("k_adam");
  return OCM_OK;
}

}  // extern "C"
