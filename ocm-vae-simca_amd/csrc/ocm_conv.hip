// Narrow 1-D convolutions of the VAE (vae_model.py:37-81: Conv1d /
// ConvTranspose1d with 1-12 channels, kernel 7, stride 1 or 2, B = 512 ×
// L = 2048).  MIOpen lowers these to implicit-GEMM kernels plus NCHW↔NHWC
// transposes: ≈ 19 kernels and ≈ 0.95 ms per graphed C4 training step,
// 36 % of it (profiles/r03g_vae_step_trace.md), for a few MB of activations per
// layer.  Here every pass is one direct kernel over the positions (the data is
// HBM/L2-streamed once; channels and taps are a handful of FMAs per element):
//
//   down  y[b][o][l] = bias[o] + Σ_i Σ_t w[o][i][t] · x[b][i][l·s + t − pad]
//         — Conv1d forward (w: [O][I][K]) and ConvTranspose1d's input gradient
//   up    y[b][o][j] = bias[o] + Σ_i Σ_t w[i][o][t] · x[b][i][(j + pad − t)/s]
//         (terms where s divides j + pad − t and the index is in range)
//         — ConvTranspose1d forward (w: [I][O][K]) and Conv1d's input gradient
//   wgrad G[o][i][t] = Σ_b Σ_l P[b][o][l] · Q[b][i][l·s + t − pad]
//         — Conv1d: P = dy, Q = x → dW[co][ci][t];  ConvTranspose1d: P = x,
//           Q = dy → dW[ci][co][t]; per-workgroup partials, summed in a fixed
//           order by a second launch (deterministic)
//   csum  Σ_b Σ_l dy[b][c][l] (the bias gradient), two-stage likewise.
//
// Activations (N, C, L) contiguous, float32 or bfloat16 (autocast); weights,
// bias and gradients of them float32; accumulation float32.  Each thread of
// down / up computes four output channels of one position (grid.y = channel
// groups); the four channels' weights sit in LDS, interleaved by channel.
#include <algorithm>

#include "ocm_internal.h"

namespace {

struct bf16_t {
  uint16_t bits;
};
__device__ __forceinline__ float cv_ld(const float* p, int64_t i) { return p[i]; }
__device__ __forceinline__ float cv_ld(const bf16_t* p, int64_t i) { return __uint_as_float((uint32_t)p[i].bits << 16); }
__device__ __forceinline__ void cv_st(float* p, int64_t i, float v) { p[i] = v; }
__device__ __forceinline__ void cv_st(bf16_t* p, int64_t i, float v) {
  // round to nearest even, NaN kept quiet (torch's float → bfloat16)
  const uint32_t u = __float_as_uint(v);
  const uint32_t r = (u & 0x7fffffffu) > 0x7f800000u ? (u | 0x00400000u) : u + 0x7fffu + ((u >> 16) & 1u);
  p[i].bits = (uint16_t)(r >> 16);
}

constexpr int CV_T = 256, CV_OG = 4, CV_KMAX = 15, CV_CMAX = 64;

// v = ok ? p[i] : 0 without a branch: the load always runs, at an index clamped into
// [0, n) — hipcc turns a guarded load into a branch with its own vmcnt(0) wait, so a
// row of guarded taps would cost one memory round trip per tap
template <typename T>
__device__ __forceinline__ float cv_ld_or0(const T* p, int i, int n, bool ok) {
  const float v = cv_ld(p, min(max(i, 0), n - 1));
  return ok ? v : 0.f;
}
constexpr int WG_SPLIT = 128;   // csum partial workgroups per channel
constexpr int WG_MAXSPLIT = 1024;  // wgrad partial workgroups per (o, i) pair, at most
constexpr int WG_PPT = 4;          // wgrad positions per thread and pass
// scratch layout: CV_TICKETS completion counter words (zero before the first
// call; every call leaves them zero), then the partials.  wgrad: groups ·
// tickets_per_slot(split) counters, ≤ 2·1024 + 8192/16; chan_sum: C·9
constexpr int CV_TICKETS = 2560 * TICKET_STRIDE;

// true in the last of the gridDim.x workgroups of slot `slot` to arrive
// (ocm_internal.h last_arrival; partials stored with st_agent)
__device__ __forceinline__ bool cv_last(unsigned* ticket, int slot) {
  return last_arrival2(ticket, slot, gridDim.x, blockIdx.x);
}

// down / up: grid (ceil(Lout / CV_T), ceil(O / OG), B).  KT ≥ K is the
// compile-time tap count, so the taps of one input channel unroll and their
// loads issue together (a runtime tap loop waits out one load latency per tap).
// Each thread computes OG output channels of its position (OG ≥ O for the C4
// layers: one pass over x per layer — with four channels per thread the
// 6 → 12 layers read every tap three times, 2-byte loads each)
template <bool UP, int KT, int OG, typename TI, typename TO>
__global__ __launch_bounds__(CV_T) void k_conv(const TI* __restrict__ x, int I, int Lin, const float* __restrict__ w,
                                              const float* __restrict__ bias, int O, int Lout, int K, int s, int pad,
                                              TO* __restrict__ y) {
  static_assert(OG % 4 == 0, "channel quads");
  constexpr int NQ = OG / 4;
  // the OG output channels' weights as [input channel][tap][channel quad]: one
  // ds_read_b128 serves four FMAs of a tap (CV_KMAX slots, zero past K)
  extern __shared__ f32x4 sw[];  // I · CV_KMAX · NQ (dynamic: only the layer's input channels)
  const int o0 = blockIdx.y * OG, b = blockIdx.z;
  const int l = blockIdx.x * CV_T + threadIdx.x;  // this thread's output position (≥ Lout: none)
  const TI* xb = x + (int64_t)b * I * Lin;
  // up: the taps that reach output l are t ≡ (l + pad) mod s, input l' = (l + pad − t)/s;
  // the t-th of them is tap t0 + t·s at input jb − t (one division per thread)
  const int q0 = l + pad;
  const int t0 = UP ? q0 % s : 0;
  const int jb = UP ? (q0 - t0) / s : 0;
  // the next input channel's taps are loaded before this channel's FMAs
  auto taps = [&](int i, float (&v)[KT]) __attribute__((always_inline)) {
    const TI* xr = xb + (int64_t)i * Lin;
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      int j;
      bool ok;
      if (UP) {
        const int tt = t0 + t * s;  // t-th tap of this output's residue class
        j = jb - t;
        ok = tt < K && j >= 0 && j < Lin;
      } else {
        j = l * s + t - pad;
        ok = t < K && j >= 0 && j < Lin;
      }
      v[t] = cv_ld_or0(xr, j, Lin, ok);
    }
  };
  // the first channel's taps are issued before the weights are staged (their
  // latencies overlap; the loads are clamped, so idle threads issue them too)
  float va[KT], vb[KT];
  taps(0, va);
  for (int e = threadIdx.x; e < I * CV_KMAX * NQ; e += CV_T) {
    const int qd = e % NQ, it = e / NQ, i = it / CV_KMAX, t = it - i * CV_KMAX;
    f32x4 wv;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int o = o0 + 4 * qd + u;
      wv[u] = (o < O && t < K) ? (UP ? w[((int64_t)i * O + o) * K + t] : w[((int64_t)o * I + i) * K + t]) : 0.f;
    }
    sw[e] = wv;
  }
  __syncthreads();
  if (l >= Lout) return;
  float acc[OG];
#pragma unroll
  for (int u = 0; u < OG; ++u) acc[u] = (bias && o0 + u < O) ? bias[o0 + u] : 0.f;
  auto fmas = [&](int i, const float (&v)[KT]) __attribute__((always_inline)) {
#pragma unroll
    for (int t = 0; t < KT; ++t) {
      // raw tap of v[t] (clamped into the slot row: v[t] = 0 there)
      const int tw = UP ? min(t0 + t * s, CV_KMAX - 1) : t;
#pragma unroll
      for (int qd = 0; qd < NQ; ++qd) {
        const f32x4 wv = sw[(i * CV_KMAX + tw) * NQ + qd];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[4 * qd + u] = fmaf(wv[u], v[t], acc[4 * qd + u]);
      }
    }
  };
  for (int i = 0; i < I; i += 2) {
    if (i + 1 < I) taps(i + 1, vb);
    fmas(i, va);
    if (i + 1 >= I) break;
    if (i + 2 < I) taps(i + 2, va);
    fmas(i + 1, vb);
  }
  TO* yb = y + (int64_t)b * O * Lout;
#pragma unroll
  for (int u = 0; u < OG; ++u)
    if (o0 + u < O) cv_st(yb, (int64_t)(o0 + u) * Lout + l, acc[u]);
}

// wgrad: grid (split, I · ⌈O/4⌉).  Consecutive threads take consecutive
// positions (b, l) of P (coalesced); a thread loads the K taps of Q[i] once and
// four P channels, and accumulates the 4·K products; with WB (the Conv1d case,
// P = dy) the i = 0 threads also sum P, the bias gradient, as tap K.  The
// workgroup's partial sums go to part[((o·I + i)·split + x)·KS + t], KS = K + WB.
template <int KT, bool WB, typename TP, typename TQ>
__global__ __launch_bounds__(CV_T) void k_conv_wgrad(const TP* __restrict__ P, int O, int Lp, const TQ* __restrict__ Q,
                                                    int I, int Lq, int B, int K, int s, int pad,
                                                    float* __restrict__ part, unsigned* __restrict__ ticket,
                                                    float* __restrict__ G, float* __restrict__ db) {
  constexpr int NA = KT + (WB ? 1 : 0);
  __shared__ float red[CV_T / 64][CV_OG][NA];
  const int i = blockIdx.y % I, o0 = (blockIdx.y / I) * CV_OG;
  const int total = B * Lp;  // < 2³¹ (checked by the host): 32-bit position arithmetic
  float acc[CV_OG][NA];  // KT ≥ K: the taps unroll with compile-time indices
#pragma unroll
  for (int u = 0; u < CV_OG; ++u)
#pragma unroll
    for (int t = 0; t < NA; ++t) acc[u][t] = 0.f;
  // WG_PPT positions per thread and pass, all their loads issued before any
  // FMA (a position at a time waited out one memory latency per position:
  // 16 in a row, ≈ 40 µs for a 5-MB layer, round 4)
  const int stride = gridDim.x * CV_T;
  for (int e0 = blockIdx.x * CV_T + threadIdx.x; e0 < total; e0 += WG_PPT * stride) {
    float qv[WG_PPT][KT], pv[WG_PPT][CV_OG];
#pragma unroll
    for (int r = 0; r < WG_PPT; ++r) {
      const int e = e0 + r * stride;
      const bool in = e < total;
      const int ec = in ? e : 0;  // clamped: a valid position, its products dropped
      const int b = ec / Lp, l = ec - b * Lp;
      const TQ* qr = Q + ((int64_t)b * I + i) * Lq;
      const int j0 = l * s - pad;
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        const int j = j0 + t;
        qv[r][t] = cv_ld_or0(qr, j, Lq, in && t < K && j >= 0 && j < Lq);
      }
      // channels past O read channel O − 1 (valid memory) and are dropped
      const TP* pb = P + (int64_t)b * O * Lp + l;
#pragma unroll
      for (int u = 0; u < CV_OG; ++u) {
        const float v = cv_ld(pb, (int64_t)min(o0 + u, O - 1) * Lp);
        pv[r][u] = in && o0 + u < O ? v : 0.f;
      }
    }
#pragma unroll
    for (int r = 0; r < WG_PPT; ++r)
#pragma unroll
      for (int u = 0; u < CV_OG; ++u) {
#pragma unroll
        for (int t = 0; t < KT; ++t) acc[u][t] = fmaf(pv[r][u], qv[r][t], acc[u][t]);
        if (WB) acc[u][NA - 1] += pv[r][u];
      }
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int u = 0; u < CV_OG; ++u)
#pragma unroll
    for (int t = 0; t < NA; ++t) {
      const float v = wave_sum_f32(acc[u][t]);
      if (lane == 0) red[wv][u][t] = v;
    }
  __syncthreads();
  const int KS = K + (WB ? 1 : 0);
  for (int e = threadIdx.x; e < CV_OG * KS; e += CV_T) {
    const int u = e / KS, t = e % KS, o = o0 + u;
    const int ts = (WB && t == K) ? NA - 1 : t;
    if (o < O)
      st_agent(part + (((int64_t)o * I + i) * gridDim.x + blockIdx.x) * KS + t,
               (red[0][u][ts] + red[1][u][ts]) + (red[2][u][ts] + red[3][u][ts]));
  }
  // the group's last workgroup: G[(o·I + i)·K + t] = Σ_x part[((o·I + i)·split + x)·KS + t],
  // one wave per output (lane-strided partials, then the wave sum: a fixed
  // order); with WB the i = 0 slot t = K of each o is its bias gradient, db[o]
  if (!cv_last(ticket, blockIdx.y)) return;
  const int split = gridDim.x;
  for (int e = wv; e < CV_OG * KS; e += CV_T / 64) {
    const int u = e / KS, t = e % KS, o = o0 + u;
    if (o >= O) continue;
    const int64_t pair = (int64_t)o * I + i;
    float v = lane_sum_agent<float, float>(part + pair * split * KS + t, KS, split, lane);
    v = wave_sum_f32(v);
    if (lane) continue;
    if (t < K) G[pair * K + t] = v;
    else if (i == 0) db[o] = v;
  }
}

// wgrad on the matrix cores (bf16 activations, the autocast training step):
// G[o][c] = Σ_pos P[o][pos] · Qc[pos] is a (O × ncol) GEMM over B·Lp positions,
// columns c = i·K + t (Qc[pos] = Q[b][i][l·s + t − pad], zero outside the row)
// plus, with WB, a column of ones whose sum is the bias gradient.  One
// v_mfma_f32_16x16x32_bf16 per 32 positions and 16 columns: A = P (16 channel
// rows × 32 positions, one 16-B load per lane), B = the Q windows, built from
// an LDS copy of the chunk's Q rows (all input channels, one wide load per 8
// values).  A workgroup takes chunks of WM_CH positions of one row b, loading
// the next chunk into registers while the MFMAs of this one run; products are
// exact in f32, and every WM_FL chunks the MFMA accumulators (16 products
// deep) are added into f32 running sums on the VALU (the bf16 MFMA truncates
// its internal sum).  The workgroups' partials are summed in a fixed order by
// the last workgroup of each 16 and then by the last of those (deterministic).
// The VALU kernel above gave each (input channel, 4 outputs) group its own
// pass over the positions: the C4 layers took 34–39 µs per call for a few MB.
using bf16x8 = __attribute__((ext_vector_type(8))) short;
// ≤ WM_WG workgroups, four per CU (37.5 KB of LDS each): each loads one chunk
// ahead, so the chunks in flight per CU — the memory-level parallelism of a
// few-MB layer — come from the resident workgroups
constexpr int WM_CH = 256, WM_NT = 6, WM_IMAX = 12, WM_OMAX = 16, WM_FL = 8, WM_WG = 1024;
constexpr int WM_NOUT = 768;  // partial floats per workgroup (O · ncol), at most
constexpr int WM_LEVELS = 3;  // 16-way partial-sum levels: 1024 → 64 → 4 → 1
template <int S>
__host__ __device__ constexpr int wm_qwp() {  // LDS row of one input channel (bf16 values): window + alignment slack
  return ((7 + (WM_CH - 1) * S + CV_KMAX + 7) / 8) * 8;
}

// QB (ConvTranspose1d, P = x, Q = dy): P gains a row of ones (A row O), whose
// products G[O][i·K + t] = Σ Q[b][i][l·s + t − pad] sum Q over the positions
// ≡ t − pad (mod s); for Lq = s·Lp and pad + s ≤ K the s taps t = pad …
// pad + s − 1 cover every position of Q once, so their sum is Σ_b Σ_j Q[b][i][j]
// (the bias gradient) at no extra MFMA: A had 16 rows and O ≤ 12 used.
template <bool WB, bool QB, int S, int NTT>
__global__ __launch_bounds__(256, 4) void k_conv_wgrad_mfma(const bf16_t* __restrict__ P, int O, int Lp,
                                                         const bf16_t* __restrict__ Q, int I, int Lq, int B, int K,
                                                         int pad, float* __restrict__ part,
                                                         unsigned* __restrict__ ticket, float* __restrict__ G,
                                                         float* __restrict__ db) {
  static_assert(!(WB && QB), "one sum per launch");
  constexpr int QWP = wm_qwp<S>(), N8 = QWP / 8;
  constexpr int QI = (WM_IMAX * N8 + 255) / 256;  // staged 16-B pieces per thread
  __shared__ __attribute__((aligned(16))) uint16_t Qs[WM_IMAX * QWP];
  __shared__ float red[4][WM_OMAX][WM_NT * 16];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int n = lane & 15, kg = lane >> 4;
  const int ncol = I * K + (WB ? 1 : 0);
  const int NT = (ncol + 15) / 16;
  const int OR = O + (QB ? 1 : 0);  // G rows (QB: the ones row O last)
  const int NOUT = OR * ncol;
  const int cpr = Lp / WM_CH, nch = B * cpr;
  // this lane's column of each N tile: LDS offset i·QWP + t (≥ 0), ones (−2), zero (−1)
  int cb[NTT];
#pragma unroll
  for (int nt = 0; nt < NTT; ++nt) {
    const int c = 16 * nt + n;
    cb[nt] = c < I * K ? (c / K) * QWP + c % K : (WB && c == I * K ? -2 : -1);
  }
  f32x4 qv[QI];
  bf16x8 av[2];
  auto window = [&](int ch, int& b, int& l0, int& base) __attribute__((always_inline)) {
    b = ch / cpr;
    l0 = (ch - b * cpr) * WM_CH;
    const int a = l0 * S - pad;
    base = a >= 0 ? (a & ~7) : -((7 - a) & ~7);  // ⌊a / 8⌋ · 8
  };
  auto load_chunk = [&](int ch) __attribute__((always_inline)) {
    int b, l0, base;
    window(ch, b, l0, base);
#pragma unroll
    for (int r = 0; r < QI; ++r) {
      const int e = tid + 256 * r, i = e / N8, j0 = base + 8 * (e - i * N8);
      // Lq % 8 == 0: an aligned piece lies wholly inside the row or wholly outside
      const bool ok = e < I * N8 && j0 >= 0 && j0 + 8 <= Lq;
      const f32x4 v = *reinterpret_cast<const f32x4*>(Q + ((int64_t)b * I + (i < I ? i : I - 1)) * Lq + (ok ? j0 : 0));
      qv[r] = ok ? v : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int pos = l0 + 64 * w + 32 * ks + 8 * kg;
      const f32x4 v = *reinterpret_cast<const f32x4*>(P + ((int64_t)b * O + (n < O ? n : O - 1)) * Lp + pos);
      const bf16x8 ones = {0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80, 0x3F80};  // bf16 1.0
      av[ks] = n < O ? __builtin_bit_cast(bf16x8, v)
                     : (QB && n == O ? ones : __builtin_bit_cast(bf16x8, f32x4{0.f, 0.f, 0.f, 0.f}));
    }
  };
  f32x4 acc[NTT], run[NTT];
#pragma unroll
  for (int nt = 0; nt < NTT; ++nt) acc[nt] = run[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  int done = 0;
  int ch = blockIdx.x;
  if (ch < nch) load_chunk(ch);
  for (; ch < nch; ch += gridDim.x) {
    int b, l0, base;
    window(ch, b, l0, base);
    const int off = l0 * S - pad - base;
    __syncthreads();  // the previous chunk's windows are read
#pragma unroll
    for (int r = 0; r < QI; ++r) {
      const int e = tid + 256 * r;
      if (e < I * N8) *reinterpret_cast<f32x4*>(&Qs[(e / N8) * QWP + 8 * (e % N8)]) = qv[r];
    }
    const bf16x8 a0 = av[0], a1 = av[1];
    __syncthreads();
    if (ch + (int)gridDim.x < nch) load_chunk(ch + gridDim.x);  // in flight under this chunk's MFMAs
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int p0 = (64 * w + 32 * ks + 8 * kg) * S + off;
#pragma unroll
      for (int nt = 0; nt < NTT; ++nt) {
        if (nt >= NT) break;
        const int c0 = cb[nt];
        const int ix = c0 >= 0 ? c0 + p0 : 0;
        const short fill = c0 == -2 ? (short)0x3F80 : (short)0;  // bf16 1.0 / 0
        bf16x8 bf;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const short v = (short)Qs[ix + j * S];
          bf[j] = c0 >= 0 ? v : fill;
        }
        acc[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ks ? a1 : a0, bf, acc[nt], 0, 0, 0);
      }
    }
    if (++done == WM_FL) {
      done = 0;
#pragma unroll
      for (int nt = 0; nt < NTT; ++nt) {
        run[nt] += acc[nt];
        acc[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  }
#pragma unroll
  for (int nt = 0; nt < NTT; ++nt) run[nt] += acc[nt];
  // D layout: column 16·nt + (lane & 15), rows 4·(lane >> 4) + r
#pragma unroll
  for (int nt = 0; nt < NTT; ++nt)
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][4 * kg + r][16 * nt + n] = run[nt][r];
  __syncthreads();
  for (int e = tid; e < NOUT; e += 256) {
    const int o = e / ncol, c = e - o * ncol;
    st_agent(part + (int64_t)blockIdx.x * NOUT + e, (red[0][o][c] + red[1][o][c]) + (red[2][o][c] + red[3][o][c]));
  }
  // the last of each 16 workgroups sums their partials, the last of each 16 of
  // those the group sums, … (fixed membership and order: deterministic)
  constexpr int EPT = WM_NOUT / 256;
  __shared__ bool last_;
  int idx = blockIdx.x, cnt = gridDim.x;
  const float* src = part;
  float* dst = part + (int64_t)gridDim.x * NOUT;
  unsigned* tk = ticket;
  for (int lvl = 0; lvl < WM_LEVELS; ++lvl) {
    const int g = idx / 16, ng = (cnt + 15) / 16, gsize = min(16, cnt - 16 * g);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have left
    __syncthreads();
    if (tid == 0) {
      unsigned* sub = tk + (int64_t)g * TICKET_STRIDE;
      const bool l = __hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)gsize - 1;
      if (l) __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      last_ = l;
    }
    __syncthreads();
    if (!last_) return;
    float v[EPT][16];
    const float* gs = src + (int64_t)16 * g * NOUT;
#pragma unroll
    for (int r = 0; r < EPT; ++r) {
      const int e = tid + 256 * r, ec = e < NOUT ? e : 0;
#pragma unroll
      for (int k = 0; k < 16; ++k) v[r][k] = ld_agent(gs + (int64_t)(k < gsize ? k : 0) * NOUT + ec);
    }
#pragma unroll
    for (int r = 0; r < EPT; ++r) {
      const int e = tid + 256 * r;
      float sm = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) sm += k < gsize ? v[r][k] : 0.f;
      if (e >= NOUT) continue;
      if (ng > 1) {
        st_agent(dst + (int64_t)g * NOUT + e, sm);
      } else {
        const int o = e / ncol, c = e - o * ncol;
        if (QB && o == O) red[0][0][c] = sm;  // the ones row, staged (the red tiles are read)
        else if (c < I * K) G[(int64_t)o * I * K + c] = sm;
        else db[o] = sm;
      }
    }
    if (ng == 1) {
      if constexpr (QB) {  // db[i] = Σ_{t = pad}^{pad + S − 1} G[O][i·K + t]
        __syncthreads();
        for (int i = tid; i < I; i += 256) {
          float sm = 0.f;
#pragma unroll
          for (int r = 0; r < S; ++r) sm += red[0][0][i * K + pad + r];
          db[i] = sm;
        }
      }
      return;
    }
    tk += (int64_t)ng * TICKET_STRIDE;
    src = dst;
    dst += (int64_t)ng * NOUT;
    idx = g;
    cnt = ng;
  }
}

// per-channel sums of (B, C, L): grid (WG_SPLIT, C) partials; the channel's
// last workgroup sums them in order (fp64)
template <typename T>
__global__ __launch_bounds__(CV_T) void k_chan_sum(const T* __restrict__ v, int B, int C, int L,
                                                  float* __restrict__ part, unsigned* __restrict__ ticket,
                                                  float* __restrict__ out) {
  __shared__ float red[CV_T / 64];
  const int c = blockIdx.y;
  const int total = B * L;  // < 2³¹ (checked by the host)
  float a = 0.f;
  // eight positions per thread and pass, their loads issued together
  constexpr int U = 8;
  for (int e0 = blockIdx.x * CV_T + threadIdx.x; e0 < total; e0 += U * WG_SPLIT * CV_T) {
    float t[U];
#pragma unroll
    for (int r = 0; r < U; ++r) {
      const int e = e0 + r * WG_SPLIT * CV_T;
      const int ec = e < total ? e : 0;
      const int b = ec / L, l = ec - b * L;
      const float x = cv_ld(v, ((int64_t)b * C + c) * L + l);
      t[r] = e < total ? x : 0.f;
    }
#pragma unroll
    for (int r = 0; r < U; ++r) a += t[r];
  }
  a = wave_sum_f32(a);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = a;
  __syncthreads();
  if (threadIdx.x == 0) st_agent(part + (int64_t)c * WG_SPLIT + blockIdx.x, (red[0] + red[1]) + (red[2] + red[3]));
  if (!cv_last(ticket, c) || threadIdx.x >= 64) return;
  const double s = wave_sum_f64(lane_sum_agent<float, double>(part + (int64_t)c * WG_SPLIT, 1, WG_SPLIT, threadIdx.x));
  if (threadIdx.x == 0) out[c] = (float)s;
}

template <bool UP, int KT, int OG>
int launch_conv_k(int dti, int dto, const void* x, int B, int I, int Lin, const float* w, const float* bias, int O,
                  int Lout, int K, int s, int pad, void* y, hipStream_t st) {
  dim3 g((unsigned)((Lout + CV_T - 1) / CV_T), (unsigned)((O + OG - 1) / OG), (unsigned)B);
#define OCM_CONV_L(TI, TO)                                                                                        \
  hipLaunchKernelGGL((k_conv<UP, KT, OG, TI, TO>), g, dim3(CV_T), (size_t)I * CV_KMAX * (OG / 4) * sizeof(f32x4), st, \
                     static_cast<const TI*>(x), I, Lin, w, bias, O, Lout, K, s, pad, static_cast<TO*>(y))
  if (dti == OCM_DTYPE_F32 && dto == OCM_DTYPE_F32) OCM_CONV_L(float, float);
  else if (dti == OCM_DTYPE_F32) OCM_CONV_L(float, bf16_t);
  else if (dto == OCM_DTYPE_F32) OCM_CONV_L(bf16_t, float);
  else OCM_CONV_L(bf16_t, bf16_t);
#undef OCM_CONV_L
  OCM_CHECK_LAUNCH("k_conv");
  return OCM_OK;
}

template <bool UP, int KT>
int launch_conv_og(int dti, int dto, const void* x, int B, int I, int Lin, const float* w, const float* bias, int O,
                   int Lout, int K, int s, int pad, void* y, hipStream_t st) {
  // output channels per thread: all of them up to 12, else groups of 16
  if (O <= 4) return launch_conv_k<UP, KT, 4>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
  if (O <= 8) return launch_conv_k<UP, KT, 8>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
  if (O <= 12) return launch_conv_k<UP, KT, 12>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
  return launch_conv_k<UP, KT, 16>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
}

template <bool UP>
int launch_conv(int dti, int dto, const void* x, int B, int I, int Lin, const float* w, const float* bias, int O,
                int Lout, int K, int s, int pad, void* y, hipStream_t st) {
  // up: KT counts the taps of one residue class, ⌈K / s⌉
  const int kt = UP ? (K + s - 1) / s : K;
  if (kt == 1) return launch_conv_og<UP, 1>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
  if (kt <= 4) return launch_conv_og<UP, 4>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
  if (kt <= 7) return launch_conv_og<UP, 7>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
  return launch_conv_og<UP, CV_KMAX>(dti, dto, x, B, I, Lin, w, bias, O, Lout, K, s, pad, y, st);
}

}  // namespace

extern "C" {

size_t ocm_conv1d_scratch_bytes(int32_t O, int32_t I, int32_t K) {
  // VALU wgrad: ≤ WG_MAXSPLIT partials of O·I·(K + 1) (+ the channel sums);
  // matrix-core wgrad: WM_WG + 64 + 4 partials of O·(I·K + 1)
  const int64_t valu = ((int64_t)O * I * (K + 1) + (int64_t)(O > I ? O : I)) * WG_MAXSPLIT;
  // (the ones column of the Conv1d bias, or the ones row of the ConvTranspose1d bias)
  const int64_t mfma = std::max((int64_t)O * (I * K + 1), (int64_t)(O + 1) * I * K) * (WM_WG + 64 + 4);
  return CV_TICKETS * sizeof(unsigned) + (size_t)(valu > mfma ? valu : mfma) * sizeof(float) + 256;
}

int ocm_conv1d(ocm_ctx* ctx, int32_t mode, int32_t dtype_in, const void* x, int32_t B, int32_t I, int32_t Lin,
               const float* w, const float* bias, int32_t O, int32_t Lout, int32_t K, int32_t stride, int32_t pad,
               int32_t dtype_out, void* y, void* stream) {
  OCM_REQUIRE(ctx && x && w && y, "ocm_conv1d: NULL argument");
  OCM_REQUIRE(mode == OCM_CONV_DOWN || mode == OCM_CONV_UP, "ocm_conv1d: mode must be OCM_CONV_DOWN or OCM_CONV_UP");
  OCM_REQUIRE(B > 0 && I > 0 && O > 0 && Lin > 0 && Lout > 0 && B <= 65535, "ocm_conv1d: bad shape");
  OCM_REQUIRE(I <= CV_CMAX && K >= 1 && K <= CV_KMAX && stride >= 1 && pad >= 0,
              "ocm_conv1d: channels ≤ 64, kernel ≤ 15, stride ≥ 1");
  OCM_REQUIRE((dtype_in == OCM_DTYPE_F32 || dtype_in == OCM_DTYPE_BF16) &&
                  (dtype_out == OCM_DTYPE_F32 || dtype_out == OCM_DTYPE_BF16),
              "ocm_conv1d: float32 / bfloat16 activations");
  hipStream_t st = (hipStream_t)stream;
  return mode == OCM_CONV_DOWN ? launch_conv<false>(dtype_in, dtype_out, x, B, I, Lin, w, bias, O, Lout, K, stride, pad, y, st)
                               : launch_conv<true>(dtype_in, dtype_out, x, B, I, Lin, w, bias, O, Lout, K, stride, pad, y, st);
}

}  // extern "C"

namespace {
// ocm_conv1d_wgrad (qsum_out = nullptr) and ocm_conv1d_wgrad_qsum (psum_out = nullptr)
int conv_wgrad(ocm_ctx* ctx, int32_t dtype_p, const void* P, int32_t O, int32_t Lp, int32_t dtype_q, const void* Q,
               int32_t I, int32_t Lq, int32_t B, int32_t K, int32_t stride, int32_t pad, float* G_out,
               float* psum_out, float* qsum_out, void* scratch, void* stream) {
  OCM_REQUIRE(ctx && P && Q && G_out && scratch, "ocm_conv1d_wgrad: NULL argument");
  OCM_REQUIRE(B > 0 && O > 0 && I > 0 && Lp > 0 && Lq > 0 && (int64_t)I * ((O + CV_OG - 1) / CV_OG) <= 1024,
              "ocm_conv1d_wgrad: bad shape");
  OCM_REQUIRE(K >= 1 && K <= CV_KMAX && stride >= 1 && pad >= 0, "ocm_conv1d_wgrad: kernel ≤ 15, stride ≥ 1");
  OCM_REQUIRE((dtype_p == OCM_DTYPE_F32 || dtype_p == OCM_DTYPE_BF16) &&
                  (dtype_q == OCM_DTYPE_F32 || dtype_q == OCM_DTYPE_BF16),
              "ocm_conv1d_wgrad: float32 / bfloat16 activations");
  hipStream_t st = (hipStream_t)stream;
  auto* ticket = static_cast<unsigned*>(scratch);
  float* part = reinterpret_cast<float*>(ticket + CV_TICKETS);
  OCM_REQUIRE((int64_t)B * Lp < (1LL << 31), "ocm_conv1d_wgrad: B·Lp must be < 2^31");
  const int groups = I * ((O + CV_OG - 1) / CV_OG);
  // ≈ 1024 workgroups in all (a one-group layer must fill the chip), between
  // one and four passes of WG_PPT positions per thread; ≤ 8192 workgroups in
  // all and ≤ WG_MAXSPLIT per group (the completion counters fit CV_TICKETS)
  const int64_t pos = (int64_t)B * Lp;
  const int one = (int)((pos + WG_PPT * CV_T - 1) / (WG_PPT * CV_T));
  const int four = (int)((pos + 4 * WG_PPT * CV_T - 1) / (4 * WG_PPT * CV_T));
  const int want = std::min(one, std::max(four, (1024 + groups - 1) / groups));
  const int split = std::max(1, std::min({WG_MAXSPLIT, std::max(1, 8192 / groups), want}));
  const bool wb = psum_out != nullptr;
  const int ncol = I * K + (wb ? 1 : 0);
  // Σ Q rides on the matrix-core launch as a ones row of P when Q's positions
  // are covered once by the taps pad … pad + s − 1 (k_conv_wgrad_mfma QB)
  const bool qb = qsum_out != nullptr && Lq == stride * Lp && pad + stride <= K && O + 1 <= WM_OMAX &&
                  (O + 1) * ncol <= WM_NOUT;
  if (dtype_p == OCM_DTYPE_BF16 && dtype_q == OCM_DTYPE_BF16 && O <= WM_OMAX && I <= WM_IMAX && ncol <= 16 * WM_NT &&
      O * ncol <= WM_NOUT &&
      (stride == 1 || stride == 2) && Lp % WM_CH == 0 && Lq % 8 == 0 && pad <= 7 &&
      (reinterpret_cast<uintptr_t>(P) & 15) == 0 && (reinterpret_cast<uintptr_t>(Q) & 15) == 0) {
    // the matrix-core path (bf16): ≤ WM_WG workgroups, two-level partial sums
    const int nch = (int)((int64_t)B * Lp / WM_CH);
    const int nwg = std::min(WM_WG, nch);
    const int nt = (ncol + 15) / 16;
#define OCM_WM3(WB, S, NTT)                                                                                        \
  do {                                                                                                             \
    if (qb)                                                                                                        \
      hipLaunchKernelGGL((k_conv_wgrad_mfma<false, true, S, NTT>), dim3((unsigned)nwg), dim3(256), 0, st,          \
                         static_cast<const bf16_t*>(P), O, Lp, static_cast<const bf16_t*>(Q), I, Lq, B, K, pad,   \
                         part, ticket, G_out, qsum_out);                                                           \
    else                                                                                                           \
      hipLaunchKernelGGL((k_conv_wgrad_mfma<WB, false, S, NTT>), dim3((unsigned)nwg), dim3(256), 0, st,            \
                         static_cast<const bf16_t*>(P), O, Lp, static_cast<const bf16_t*>(Q), I, Lq, B, K, pad,   \
                         part, ticket, G_out, psum_out);                                                           \
  } while (0)
#define OCM_WM(WB, S)                    \
  do {                                   \
    if (nt == 1) OCM_WM3(WB, S, 1);      \
    else if (nt == 2) OCM_WM3(WB, S, 2); \
    else if (nt == 3) OCM_WM3(WB, S, 3); \
    else OCM_WM3(WB, S, 6);              \
  } while (0)
    if (wb && stride == 1) OCM_WM(true, 1);
    else if (wb) OCM_WM(true, 2);
    else if (stride == 1) OCM_WM(false, 1);
    else OCM_WM(false, 2);
#undef OCM_WM
#undef OCM_WM3
    OCM_CHECK_LAUNCH("k_conv_wgrad_mfma");
    if (qsum_out && !qb) return ocm_chan_sum(ctx, dtype_q, Q, B, I, Lq, qsum_out, scratch, stream);
    return OCM_OK;
  }
  dim3 g((unsigned)split, (unsigned)groups);
#define OCM_WG_K(KT, WB, TP, TQ)                                                                            \
  hipLaunchKernelGGL((k_conv_wgrad<KT, WB, TP, TQ>), g, dim3(CV_T), 0, st, static_cast<const TP*>(P), O, Lp,   \
                     static_cast<const TQ*>(Q), I, Lq, B, K, stride, pad, part, ticket, G_out, psum_out)
#define OCM_WG_L(TP, TQ)                                  \
  do {                                                    \
    if (K <= 7 && wb) OCM_WG_K(7, true, TP, TQ);          \
    else if (K <= 7) OCM_WG_K(7, false, TP, TQ);          \
    else if (wb) OCM_WG_K(CV_KMAX, true, TP, TQ);         \
    else OCM_WG_K(CV_KMAX, false, TP, TQ);                \
  } while (0)
  if (dtype_p == OCM_DTYPE_F32 && dtype_q == OCM_DTYPE_F32) OCM_WG_L(float, float);
  else if (dtype_p == OCM_DTYPE_F32) OCM_WG_L(float, bf16_t);
  else if (dtype_q == OCM_DTYPE_F32) OCM_WG_L(bf16_t, float);
  else OCM_WG_L(bf16_t, bf16_t);
#undef OCM_WG_L
#undef OCM_WG_K
  OCM_CHECK_LAUNCH("k_conv_wgrad");
  if (qsum_out)  // the layer's scratch again: stream-ordered, its counters left zero
    return ocm_chan_sum(ctx, dtype_q, Q, B, I, Lq, qsum_out, scratch, stream);
  return OCM_OK;
}
}  // namespace

extern "C" {

int ocm_conv1d_wgrad(ocm_ctx* ctx, int32_t dtype_p, const void* P, int32_t O, int32_t Lp, int32_t dtype_q,
                     const void* Q, int32_t I, int32_t Lq, int32_t B, int32_t K, int32_t stride, int32_t pad,
                     float* G_out, float* psum_out, void* scratch, void* stream) {
  return conv_wgrad(ctx, dtype_p, P, O, Lp, dtype_q, Q, I, Lq, B, K, stride, pad, G_out, psum_out, nullptr, scratch,
                    stream);
}

int ocm_conv1d_wgrad_qsum(ocm_ctx* ctx, int32_t dtype_p, const void* P, int32_t O, int32_t Lp, int32_t dtype_q,
                          const void* Q, int32_t I, int32_t Lq, int32_t B, int32_t K, int32_t stride, int32_t pad,
                          float* G_out, float* qsum_out, void* scratch, void* stream) {
  OCM_REQUIRE(qsum_out, "ocm_conv1d_wgrad_qsum: NULL argument");
  return conv_wgrad(ctx, dtype_p, P, O, Lp, dtype_q, Q, I, Lq, B, K, stride, pad, G_out, nullptr, qsum_out, scratch,
                    stream);
}

int ocm_chan_sum(ocm_ctx* ctx, int32_t dtype, const void* v, int32_t B, int32_t C, int32_t L, float* out,
                 void* scratch, void* stream) {
  OCM_REQUIRE(ctx && v && out && scratch, "ocm_chan_sum: NULL argument");
  OCM_REQUIRE(B > 0 && C > 0 && L > 0 && C * tickets_per_slot(WG_SPLIT) * TICKET_STRIDE <= CV_TICKETS &&
                  (int64_t)B * L < (1LL << 31),
              "ocm_chan_sum: bad shape (C ≤ 284)");
  OCM_REQUIRE(dtype == OCM_DTYPE_F32 || dtype == OCM_DTYPE_BF16, "ocm_chan_sum: float32 / bfloat16");
  hipStream_t st = (hipStream_t)stream;
  auto* ticket = static_cast<unsigned*>(scratch);
  float* part = reinterpret_cast<float*>(ticket + CV_TICKETS);
  dim3 g(WG_SPLIT, (unsigned)C);
  if (dtype == OCM_DTYPE_F32)
    hipLaunchKernelGGL(k_chan_sum<float>, g, dim3(CV_T), 0, st, static_cast<const float*>(v), B, C, L, part, ticket,
                       out);
  else
    hipLaunchKernelGGL(k_chan_sum<bf16_t>, g, dim3(CV_T), 0, st, static_cast<const bf16_t*>(v), B, C, L, part,
                       ticket, out);
  OCM_CHECK_LAUNCH("k_chan_sum");
  return OCM_OK;
}

}  // extern "C"
