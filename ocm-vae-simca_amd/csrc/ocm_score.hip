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

#include <utility>

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
                                               double* T2_out, float* __restrict__ Q_out, DecArgs dec,
                                               double* __restrict__ acc_out, int64_t acc_stride,
                                               double* __restrict__ stat_part, int ldt = 0,
                                               const double* T2_in = nullptr) {
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
  if (ldt <= 0) ldt = k;
  if (own) {
    if (T2_in) T2 = T2_in[grow];  // earlier component blocks (k > 64)
    const double* trow = Tt + l31 * (KP + 1);
    if (a_diag) {  // A holds the diagonal only
      for (int a = 0; a < k; ++a) T2 += trow[a] * trow[a] * A[a];
    } else {
      for (int a = 0; a < k; ++a) {
        double s = 0.0;
        for (int b = 0; b < k; ++b) s += A[a * k + b] * trow[b];
        T2 += trow[a] * s;
      }
    }
    if (T_out)
      for (int a = 0; a < k; ++a) T_out[grow * ldt + a] = (float)trow[a];
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
// X and R_out (and T2_in / T2_out) alias for the component blocks after the
// first (k > 64: the residual is projected in place), so they carry no
// __restrict__
__global__ __launch_bounds__(256, 2) void k_score_direct(const float* X, int64_t ldx,
                                                         const int64_t* __restrict__ rows, int64_t m, int p,
                                                         const float* __restrict__ P, const float* __restrict__ mu,
                                                         const double* __restrict__ A, int k, int a_diag,
                                                         float* __restrict__ T_out, double* T2_out,
                                                         float* __restrict__ Q_out, DecArgs dec,
                                                         double* __restrict__ acc_out, int64_t acc_stride,
                                                         double* __restrict__ stat_part, int ldt,
                                                         const double* T2_in, float* R_out,
                                                         int64_t ldr) {
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
      f32x4 rv;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float cm = col + e < p ? 1.f : 0.f;  // clamped loads beyond p carry data
        const float r = ((S.d[g][e] - u[e]) - accR[4 * g + e]) * cm;
        rv[e] = r;
        qc += r * r;
      }
      if (R_out && grow < m) {  // the residual feeds the next component block (k > 64)
        float* rr = R_out + grow * ldr;
        if (VEC && col + 3 < p) {
          *reinterpret_cast<f32x4*>(rr + col) = rv;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e)
            if (col + e < p) rr[col + e] = rv[e];
        }
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
                         Q_out, dec, acc_out, acc_stride, stat_part, ldt, T2_in);
}

// ---------------------------------------------------------------------------
// k_score_1p — single HBM pass over X (p ∈ {256, 512, 1024, 2048}, k ≤ 20,
// diagonal A = diag(1/λ) as every SIMCA fit produces).  The default scoring
// kernel for those shapes; k_score_direct covers the rest.
//
// One workgroup of four waves per CU (one wave per SIMD), persistent over
// 16-row tiles.  Wave w owns columns [w·p/4, (w+1)·p/4) of a tile's 16 rows.
// The raw rows stay in AGPRs from the HBM read to the residual (X is read
// once), in two tile buffers: while tile t is finished (sweep 2) and tile
// t + G (G = grid) starts (sweep 1), tile t + 2G streams into the registers
// tile t frees, block by block — a whole tile (the 128 KiB per CU an HBM
// stream needs in flight at full rate) is always outstanding and each load
// has a full tile of compute to arrive.  The MFMAs read x straight from the
// AGPRs: no VALU touches the data.
//   sweep 1  tᵀ += P₀·xᵀ (comps 0..15) on v_mfma_f32_16x16x4_f32, lane (row =
//            l&15, q = l>>4) feeding column 16j+4q+e of its row as B; comps
//            16..19 on v_mfma_f32_4x4x1_16b_f32 (16 4×4 blocks, a quarter of
//            the cycles: block l/4 = (q, row group), so lane (row, q) sums its
//            own columns, reduced over q once per tile; the A operands come
//            from one register per block by ds_bpermute); the mean is applied
//            once per tile, t = P·x − P·μ (fp64);
//   reduce   the four waves' partial t meet in LDS (one barrier per tile);
//   sweep 2  rᵀ = xᵀ + Pᵀ·(−t)ᵀ − μ per 16-column block: a chain of MFMAs from
//            the AGPR tile as accumulator input (comps as K; one more step
//            with the −μ column); q += r²;
//   epilogue the wave partials of Q meet after the next barrier; T², Q, T,
//            the fused decision and the moment partials.
// Nothing but X (and the row indices of a gather, through the scalar cache) is
// read from global memory inside the tile loop and the waves synchronise by
// LDS + s_barrier only: vmcnt is in order, so any wait on another global
// access would also wait for the tile in flight.  Rows past m are clamped to
// row m−1 (a valid row) and their outputs dropped.  P₀ is stored
// [comp][16-B chunk ^ sw(comp)]: conflict-free ds_read_b128 in sweep 1 and
// ds_read_b32 in sweep 2.  Numerics: f32 MFMA products, f32 partials over ≤ 64
// columns per chain flushed to f64; r is formed in the f32 accumulator as the
// reference forms X − (T·P + μ) in float32 (utils/SIMCA.py:67, 105).
// ---------------------------------------------------------------------------
namespace s1p {
constexpr int R = 16;  // rows per tile (the waves per workgroup are k_score_1p's WV)
// compile-time loop: f(std::integral_constant<int, I>) for I = 0 .. N-1
template <class F, int... I>
__device__ __forceinline__ void sfor_(F&& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  sfor_(f, std::make_integer_sequence<int, N>{});
}
__device__ __forceinline__ int sw(int m) { return ((4 * m) ^ (2 * (m >> 2))) & 15; }

// 16 B of row data into an AGPR quad, not tracked by the compiler's waitcnt:
// the consumer waits with wait_vm (vmcnt is in order)
template <int OFF>
__device__ __forceinline__ void load_a(f32x4& a, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off offset:%2" : "=a"(a) : "v"(p), "n"(OFF) : "memory");
}
// diagnostic builds only (make exp): the refill loads of sweep 2 are skipped
template <int OFF>
__device__ __forceinline__ void refill_a(f32x4& a, const float* p) {
#ifdef OCM_S1P_DIAG_NOLOAD
  asm volatile("" : "+a"(a) : "v"(p));
#else
  load_a<OFF>(a, p);
#endif
}
template <int N>
__device__ __forceinline__ void wait_vm(f32x4& a) {
  asm volatile("s_waitcnt vmcnt(%1)" : "+a"(a) : "n"(N));
}
// the halo quad of a lazy view's row tile: a VGPR, loaded and waited the same way
__device__ __forceinline__ void load_v(f32x4& h, const float* p) {
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(h) : "v"(p) : "memory");
}
template <int N>
__device__ __forceinline__ void wait_vv(f32x4& h) {
  asm volatile("s_waitcnt vmcnt(%1)" : "+v"(h) : "n"(N));
}
// lane `src` (a byte address: 4·lane) of v
__device__ __forceinline__ float xlane(int src, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(src, __builtin_bit_cast(int, v)));
}

// Sweep-1 block: acc[A..D] += a[e] · x[e] (comps 0..15), and for EX acc[E,F]
// += b[e] ⊗ x[e] on 4x4x1 blocks (comps 16..19 of this lane's row over its
// columns).  B operands straight from the AGPR tile; four (six) interleaved
// chains, none waits on its predecessor.  The s_nop covers a VALU/LDS write
// of a or b right before.
#ifdef OCM_S1P_DIAG_NOMFMA  // diagnostic builds only (make exp): both sweeps' MFMAs removed, timing only
#define OCM_MF(ACC, A, B) ""
#define OCM_M4(ACC, A, B) ""
#else
#define OCM_MF(ACC, A, B) "v_mfma_f32_16x16x4_f32 %[" #ACC "], %[" #A "], %[" #B "], %[" #ACC "]\n\t"
#define OCM_M4(ACC, A, B) "v_mfma_f32_4x4x1_16b_f32 %[" #ACC "], %[" #A "], %[" #B "], %[" #ACC "]\n\t"
#endif
template <bool EX>
__device__ __forceinline__ void s1_block(f32x4& acA, f32x4& acB, f32x4& acC, f32x4& acD, f32x4& acE, f32x4& acF,
                                         const f32x4& a, const float (&b)[4], const f32x4& x) {
  if constexpr (EX)
    asm("s_nop 1\n\t" OCM_M4(cE, b0, x0) OCM_MF(cA, a0, x0) OCM_M4(cF, b1, x1) OCM_MF(cB, a1, x1)
            OCM_M4(cE, b2, x2) OCM_MF(cC, a2, x2) OCM_M4(cF, b3, x3) OCM_MF(cD, a3, x3)
        : [cA] "+v"(acA), [cB] "+v"(acB), [cC] "+v"(acC), [cD] "+v"(acD), [cE] "+v"(acE), [cF] "+v"(acF)
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [b0] "v"(b[0]), [b1] "v"(b[1]),
          [b2] "v"(b[2]), [b3] "v"(b[3]), [x0] "a"(x[0]), [x1] "a"(x[1]), [x2] "a"(x[2]), [x3] "a"(x[3]));
  else
    asm("s_nop 1\n\t" OCM_MF(cA, a0, x0) OCM_MF(cB, a1, x1) OCM_MF(cC, a2, x2) OCM_MF(cD, a3, x3)
        : [cA] "+v"(acA), [cB] "+v"(acB), [cC] "+v"(acC), [cD] "+v"(acD)
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [x0] "a"(x[0]), [x1] "a"(x[1]),
          [x2] "a"(x[2]), [x3] "a"(x[3]));
}

// Sweep-2 block pair (j, j+1): r_u = x_u − μ_u + Σ_s a_u[s]·tB[s], two MFMA
// chains interleaved, in place on the AGPR tile (an MFMA's C input and result
// share a register file).  The −μ step comes first, on a 4x4x1 MFMA (block
// l/4, row l&3 = this lane's column 4q + (l&3); B = 1), then NS = 4 or 5 comp
// steps.  QW: the q += r² work of the PREVIOUS pair (p0, p1, finished a whole
// pair ago) rides in the gaps of this pair's MFMAs as groups of four
// independent VALU ops (a dependent VALU op would stall the in-order issue
// and with it the next MFMA); the caller refills p0, p1 afterwards.  No
// trailing wait: the next reader of x0, x1 is the next pair's statement or
// the drain, which opens with its own s_nop.
#ifdef OCM_S1P_DIAG_NOMFMA
#define OCM_M2(R, A, T) ""
#else
#define OCM_M2(R, A, T) "v_mfma_f32_16x16x4_f32 %[" #R "], %[" #A "], %[" #T "], %[" #R "]\n\t"
#endif
#define OCM_RD(S, P) "v_accvgpr_read_b32 %[" #S "], %[" #P "]\n\t"
#define OCM_FM(Q, S) "v_fmac_f32_e32 %[" #Q "], %[" #S "], %[" #S "]\n\t"
template <bool EX, bool QW>
__device__ __forceinline__ void s2_pair(f32x4& x0, f32x4& x1, const float (&a0)[5], const float (&a1)[5], float m0,
                                        float m1, const float (&tB)[5], float one, const f32x4& p0, const f32x4& p1,
                                        float (&q)[4]) {
  float s[4];
  if constexpr (EX && QW)
    asm volatile("s_nop 1\n\t" OCM_M4(x0, m0, on) OCM_M4(x1, m1, on) "s_nop 4\n\t" OCM_M2(x0, u0, t0) OCM_M2(x1, w0, t0) OCM_RD(s0, p00) OCM_RD(s1, p10) OCM_RD(s2, p01) OCM_RD(s3, p11) OCM_M2(x0, u1, t1) OCM_FM(q0, s0) OCM_FM(q1, s1) OCM_FM(q2, s2) OCM_FM(q3, s3) OCM_M2(x1, w1, t1) OCM_RD(s0, p02) OCM_RD(s1, p12) OCM_RD(s2, p03) OCM_RD(s3, p13) OCM_M2(x0, u2, t2) OCM_FM(q0, s0) OCM_FM(q1, s1) OCM_FM(q2, s2) OCM_FM(q3, s3) OCM_M2(x1, w2, t2) OCM_M2(x0, u3, t3) OCM_M2(x1, w3, t3) OCM_M2(x0, u4, t4) OCM_M2(x1, w4, t4)
        : [x0] "+a"(x0), [x1] "+a"(x1), [q0] "+v"(q[0]), [q1] "+v"(q[1]), [q2] "+v"(q[2]), [q3] "+v"(q[3]), [s0] "=&v"(s[0]), [s1] "=&v"(s[1]), [s2] "=&v"(s[2]), [s3] "=&v"(s[3])
        : [u0] "v"(a0[0]), [u1] "v"(a0[1]), [u2] "v"(a0[2]), [u3] "v"(a0[3]), [u4] "v"(a0[4]), [w0] "v"(a1[0]), [w1] "v"(a1[1]), [w2] "v"(a1[2]), [w3] "v"(a1[3]), [w4] "v"(a1[4]), [m0] "v"(m0), [m1] "v"(m1), [t0] "v"(tB[0]), [t1] "v"(tB[1]), [t2] "v"(tB[2]), [t3] "v"(tB[3]), [t4] "v"(tB[4]), [on] "v"(one), [p00] "a"(p0[0]), [p01] "a"(p0[1]), [p02] "a"(p0[2]), [p03] "a"(p0[3]), [p10] "a"(p1[0]), [p11] "a"(p1[1]), [p12] "a"(p1[2]), [p13] "a"(p1[3]));
  else if constexpr (EX)
    asm volatile("s_nop 1\n\t" OCM_M4(x0, m0, on) OCM_M4(x1, m1, on) "s_nop 4\n\t" OCM_M2(x0, u0, t0) OCM_M2(x1, w0, t0) OCM_M2(x0, u1, t1) OCM_M2(x1, w1, t1) OCM_M2(x0, u2, t2) OCM_M2(x1, w2, t2) OCM_M2(x0, u3, t3) OCM_M2(x1, w3, t3) OCM_M2(x0, u4, t4) OCM_M2(x1, w4, t4)
        : [x0] "+a"(x0), [x1] "+a"(x1)
        : [u0] "v"(a0[0]), [u1] "v"(a0[1]), [u2] "v"(a0[2]), [u3] "v"(a0[3]), [u4] "v"(a0[4]), [w0] "v"(a1[0]), [w1] "v"(a1[1]), [w2] "v"(a1[2]), [w3] "v"(a1[3]), [w4] "v"(a1[4]), [m0] "v"(m0), [m1] "v"(m1), [t0] "v"(tB[0]), [t1] "v"(tB[1]), [t2] "v"(tB[2]), [t3] "v"(tB[3]), [t4] "v"(tB[4]), [on] "v"(one));
  else if constexpr (QW)
    asm volatile("s_nop 1\n\t" OCM_M4(x0, m0, on) OCM_M4(x1, m1, on) "s_nop 4\n\t" OCM_M2(x0, u0, t0) OCM_M2(x1, w0, t0) OCM_RD(s0, p00) OCM_RD(s1, p10) OCM_RD(s2, p01) OCM_RD(s3, p11) OCM_M2(x0, u1, t1) OCM_FM(q0, s0) OCM_FM(q1, s1) OCM_FM(q2, s2) OCM_FM(q3, s3) OCM_M2(x1, w1, t1) OCM_RD(s0, p02) OCM_RD(s1, p12) OCM_RD(s2, p03) OCM_RD(s3, p13) OCM_M2(x0, u2, t2) OCM_FM(q0, s0) OCM_FM(q1, s1) OCM_FM(q2, s2) OCM_FM(q3, s3) OCM_M2(x1, w2, t2) OCM_M2(x0, u3, t3) OCM_M2(x1, w3, t3)
        : [x0] "+a"(x0), [x1] "+a"(x1), [q0] "+v"(q[0]), [q1] "+v"(q[1]), [q2] "+v"(q[2]), [q3] "+v"(q[3]), [s0] "=&v"(s[0]), [s1] "=&v"(s[1]), [s2] "=&v"(s[2]), [s3] "=&v"(s[3])
        : [u0] "v"(a0[0]), [u1] "v"(a0[1]), [u2] "v"(a0[2]), [u3] "v"(a0[3]), [w0] "v"(a1[0]), [w1] "v"(a1[1]), [w2] "v"(a1[2]), [w3] "v"(a1[3]), [m0] "v"(m0), [m1] "v"(m1), [t0] "v"(tB[0]), [t1] "v"(tB[1]), [t2] "v"(tB[2]), [t3] "v"(tB[3]), [on] "v"(one), [p00] "a"(p0[0]), [p01] "a"(p0[1]), [p02] "a"(p0[2]), [p03] "a"(p0[3]), [p10] "a"(p1[0]), [p11] "a"(p1[1]), [p12] "a"(p1[2]), [p13] "a"(p1[3]));
  else
    asm volatile("s_nop 1\n\t" OCM_M4(x0, m0, on) OCM_M4(x1, m1, on) "s_nop 4\n\t" OCM_M2(x0, u0, t0) OCM_M2(x1, w0, t0) OCM_M2(x0, u1, t1) OCM_M2(x1, w1, t1) OCM_M2(x0, u2, t2) OCM_M2(x1, w2, t2) OCM_M2(x0, u3, t3) OCM_M2(x1, w3, t3)
        : [x0] "+a"(x0), [x1] "+a"(x1)
        : [u0] "v"(a0[0]), [u1] "v"(a0[1]), [u2] "v"(a0[2]), [u3] "v"(a0[3]), [w0] "v"(a1[0]), [w1] "v"(a1[1]), [w2] "v"(a1[2]), [w3] "v"(a1[3]), [m0] "v"(m0), [m1] "v"(m1), [t0] "v"(tB[0]), [t1] "v"(tB[1]), [t2] "v"(tB[2]), [t3] "v"(tB[3]), [on] "v"(one));
  (void)s, (void)p0, (void)p1, (void)q;
}
// s1_block with the B operands in VGPRs (a lazy view's tile, transformed in registers)
template <bool EX>
__device__ __forceinline__ void s1_block_v(f32x4& acA, f32x4& acB, f32x4& acC, f32x4& acD, f32x4& acE, f32x4& acF,
                                           const f32x4& a, const float (&b)[4], const f32x4& x) {
  if constexpr (EX)
    asm("s_nop 1\n\t" OCM_M4(cE, b0, x0) OCM_MF(cA, a0, x0) OCM_M4(cF, b1, x1) OCM_MF(cB, a1, x1)
            OCM_M4(cE, b2, x2) OCM_MF(cC, a2, x2) OCM_M4(cF, b3, x3) OCM_MF(cD, a3, x3)
        : [cA] "+v"(acA), [cB] "+v"(acB), [cC] "+v"(acC), [cD] "+v"(acD), [cE] "+v"(acE), [cF] "+v"(acF)
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [b0] "v"(b[0]), [b1] "v"(b[1]),
          [b2] "v"(b[2]), [b3] "v"(b[3]), [x0] "v"(x[0]), [x1] "v"(x[1]), [x2] "v"(x[2]), [x3] "v"(x[3]));
  else
    asm("s_nop 1\n\t" OCM_MF(cA, a0, x0) OCM_MF(cB, a1, x1) OCM_MF(cC, a2, x2) OCM_MF(cD, a3, x3)
        : [cA] "+v"(acA), [cB] "+v"(acB), [cC] "+v"(acC), [cD] "+v"(acD)
        : [a0] "v"(a[0]), [a1] "v"(a[1]), [a2] "v"(a[2]), [a3] "v"(a[3]), [x0] "v"(x[0]), [x1] "v"(x[1]),
          [x2] "v"(x[2]), [x3] "v"(x[3]));
}
#undef OCM_MF
#undef OCM_M4
#undef OCM_M2
#undef OCM_RD
#undef OCM_FM
}  // namespace s1p

#ifdef OCM_S1P_W8  // make exp A/B: OCM_S1P_W8_ON=0 selects the four-wave kernel in the same process
static bool s1p_w8_enabled() {
  const char* v = getenv("OCM_S1P_W8_ON");
  return !v || v[0] != '0';
}
#endif

// HH ≥ 0: a lazy view (include/ocm.h ocm_prep, window 2·HH + 1, or SNV only
// at HH = 0).  Each raw tile is transformed in registers inside sweep 1, block
// by block one block behind its loads: the quads of the neighbouring lanes of
// a row (and of the block before / after) arrive by ds_bpermute, each tile
// brings one more quad per lane — the HH columns beyond the wave's slice on
// either side (lanes lq ≥ 2: virtual block −1, lq ≤ 1: virtual block NJ) —
// and loads it first, the rows' (m_r, s_r) come through the scalar cache.
// y replaces x in the AGPR tile, so sweep 2 and the epilogue are unchanged;
// sweep 1 takes y from VGPRs.  The first / last HH columns of the row (wave 0
// block 0, wave 3 block NJ − 1) use the least-squares edge rows.
// WV: waves per workgroup.  4 (the default) = one wave per SIMD with two row
// tiles in AGPRs; 8 = two waves per SIMD, each with half the columns (NJ
// halves at the same p) and the same two tiles (half the AGPRs), so one wave's
// MFMA stream can run under the other's loads and waits.  WV = 8 keeps one
// tpart buffer (P₀ takes 128 KiB of the 160 KiB of LDS at p = 2048) and adds a
// barrier before sweep 1 writes it.
template <int NJ, bool EX, int HH = -1, int WV = 4>
__global__ __launch_bounds__(64 * WV, 1) void k_score_1p(const float* __restrict__ X, int64_t ldx,
                                                     const int64_t* __restrict__ rows, int64_t m,
                                                     const double* __restrict__ P, const double* __restrict__ mu,
                                                     const double* __restrict__ adiag, int k,
                                                     float* __restrict__ T_out, double* __restrict__ T2_out,
                                                     float* __restrict__ Q_out, DecArgs dec,
                                                     double* __restrict__ acc_out, int64_t acc_stride,
                                                     double* __restrict__ stat_part, int64_t ntiles,
                                                     PrepArgs pa, const float* __restrict__ ptaps,
                                                     const float* __restrict__ prow) {
  using namespace s1p;
  constexpr int W = WV;             // waves (column slices) per workgroup
  constexpr int NT = 64 * WV;       // threads
  constexpr int TPB = WV == 4 ? 2 : 1;  // tpart buffers
  constexpr bool PREP = HH >= 0;
  constexpr int GL = NJ + (HH > 0 ? 1 : 0);  // loads per tile group (the halo quad first)
  constexpr int PW = 16 * NJ;  // columns per wave
  constexpr int PP = W * PW;   // p
  constexpr int NCH = PP / 4;  // 16-B chunks per component row
  static_assert(NJ % 4 == 0 && 2 * NJ - 1 <= 63, "64-column wave slices, vmcnt range");
  __shared__ f32x4 P0s[16 * NCH];
  __shared__ float nmuL[PP];               // −μ (the sweep-2 μ step's A operand)
  __shared__ double pmuL[20];              // P·μ (fp64)
  __shared__ double tpart[TPB][W * 20 * R];  // [buffer][wave][comp][row]
  __shared__ double qpart[2][W * R];       // [buffer][wave][row]
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ln = lane & 15, lq = lane >> 4;

  // ---- prologue: loadings (f64 → f32) and −μ into LDS, P·μ (fp64), comps
  // 16..19 and diag(A) into registers.  Every load is unconditional (rows
  // c ≥ k clamped to row 0, zeroed by a select after the load) and issued in
  // batches ahead of its use: with per-element branches each load was waited
  // for before the next issued — ≈220 L2 round trips per workgroup, 40 µs of
  // every launch (profiles/r05s1_score_prologue_ab.jsonl)
  {
    constexpr int PE = 16 * NCH / NT;  // chunks per thread (= NJ)
    constexpr int UB = PE < 8 ? PE : 8;
    static_assert(PE % UB == 0, "prologue batches");
#pragma unroll
    for (int i0 = 0; i0 < PE; i0 += UB) {
      double v[UB][4];
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int e = tid + (i0 + u) * NT, c = e / NCH, ch = e - c * NCH;
        const double* src = P + (int64_t)(c < k ? c : 0) * PP + 4 * ch;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[u][q] = src[q];
      }
#pragma unroll
      for (int u = 0; u < UB; ++u) {
        const int e = tid + (i0 + u) * NT, c = e / NCH, ch = e - c * NCH;
        f32x4 x;
#pragma unroll
        for (int q = 0; q < 4; ++q) x[q] = c < k ? (float)v[u][q] : 0.f;
        P0s[c * NCH + (ch ^ sw(c))] = x;
      }
    }
    constexpr int ME = PP / NT;  // −μ entries per thread
    float nm[ME];
#pragma unroll
    for (int i = 0; i < ME; ++i) nm[i] = -(float)mu[tid + i * NT];
#pragma unroll
    for (int i = 0; i < ME; ++i) nmuL[tid + i * NT] = nm[i];
    // P·μ: lane l sums columns l, l + 64, ... in that order (fma chain), then
    // the wave sum; μ's lane columns loaded once for the wave's comps
    constexpr int CL = PP / 64;
    double muv[CL];
#pragma unroll
    for (int i = 0; i < CL; ++i) muv[i] = mu[lane + 64 * i];
    for (int c = w; c < 20; c += W) {  // wave w: comps w, w + W, ...
      double s = 0.0;
      if (c < k) {
        double pv[CL];
#pragma unroll
        for (int i = 0; i < CL; ++i) pv[i] = P[(int64_t)c * PP + lane + 64 * i];
#pragma unroll
        for (int i = 0; i < CL; ++i) s += pv[i] * muv[i];
      }
      s = wave_sum_f64(s);
      if (lane == 0) pmuL[c] = s;
    }
  }
  float p1a[EX ? NJ : 1];  // comps 16..19: lane (ln, lq) holds P[16 + lq][w·PW + 16j + ln] (sweep 2)
  // the same values with the column of lanes lq ≥ 2 XOR 8 (lane (x, c) holds
  // column x ^ 8·(c >> 1)): the sources one half-wave's ds_bpermute reads in
  // sweep 1 then sit on 8 distinct banks (lane mod 32) instead of 4 — with p1a
  // as the source, lanes 16c + col and 16(c + 2) + col met on one bank: a 2-way
  // conflict on every bpermute, 256 extra LDS cycles per wave and tile, the
  // whole SQ_LDS_BANK_CONFLICT count of round 2 (profiles/r02n_pmc_score.json)
  // (the widest lazy-view variant, HH = 7 at NJ = 32, has no VGPRs to spare for
  // p1b: its sweep 1 reads p1a at the equivalent lane, 16c + 4lq + e, and takes
  // the 2-way conflicts back — round 3 measured them at no cost in time)
  constexpr bool NOP1B = EX && ((NJ == 32 && HH > 4) || WV == 8);  // WV = 8: no registers to spare either
  float p1b[EX && !NOP1B ? NJ : 1];
  if constexpr (EX) {
    const bool p1v = 16 + lq < k;  // rows ≥ k: row 0 loaded, zeroed after
    const double* p1r = P + (int64_t)(p1v ? 16 + lq : 0) * PP + w * PW;
    double pa_[NJ], pb_[NOP1B ? 1 : NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      pa_[j] = p1r[16 * j + ln];
      if constexpr (!NOP1B) pb_[j] = p1r[16 * j + (ln ^ (8 * (lq >> 1)))];
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      p1a[j] = p1v ? (float)pa_[j] : 0.f;
      if constexpr (!NOP1B) p1b[j] = p1v ? (float)pb_[j] : 0.f;
    }
  }
  // diag(A) of this lane's comps lq + 4s: registers at WV = 4, LDS at WV = 8
  // (read once per tile, in compute_t; the registers went to the tiles)
  __shared__ double adL[WV == 8 ? 20 : 1];
  double ad[WV == 8 ? 1 : 5];
  if constexpr (WV == 8) {
    if (tid < 20) adL[tid] = tid < k ? adiag[tid] : 0.0;
  } else {
#pragma unroll
    for (int s = 0; s < 5; ++s) ad[s] = lq + 4 * s < k ? adiag[lq + 4 * s] : 0.0;
  }
  // sweep-1 A operand: chunk (w·PW/4 + 4j + lq) ^ sw(ln) of comp ln; the XOR
  // only touches the low 4 bits, so j = 4a + b reads b1[b] + 16a chunks
  int b1[4];
#pragma unroll
  for (int b = 0; b < 4; ++b) b1[b] = ln * NCH + w * (PW / 4) + ((4 * b + lq) ^ sw(ln));
  // sweep-2 A operand: P[c = 4s + lq][w·PW + 16j + ln] at float index
  // 4·(c·NCH + w·PW/4 + ((4j + ln/4) ^ sw(c))) + ln%4; j = 4a + b → b2[s][b] + 64a
  int b2[4][4];
#pragma unroll
  for (int s = 0; s < 4; ++s)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int c = 4 * s + lq;
      b2[s][b] = 4 * (c * NCH + w * (PW / 4) + ((4 * b + (ln >> 2)) ^ sw(c))) + (ln & 3);
    }
  const float* p0f = reinterpret_cast<const float*>(P0s);
  // sweep-1 comps 16..19 operand of MFMA e: P[16 + (ln&3)][16j + 4lq + e], which
  // p1b[j] holds on lane 16c + ((4lq) ^ 8(c >> 1)) + e, c = ln&3 (ds_bpermute
  // address, bytes)
  const int bperm = 4 * (16 * (ln & 3) + ((4 * lq) ^ (8 * ((ln & 3) >> 1))));
  const int bpermA = 4 * (16 * (ln & 3) + 4 * lq);  // the same operands from p1a (NOP1B)
  const float one = 1.f;  // B of the −μ step
  __syncthreads();

  const int64_t G = gridDim.x;
  // base of this lane's 16-B pieces in row `row` of the wave's column slice
  auto col_base = [&](int64_t row) { return X + row * ldx + w * PW + 4 * lq; };
  // row index of lane row ln in tile tt (clamped: always a valid row).  For a
  // gather the 16 indices are read through the scalar cache (uniform
  // addresses, lgkmcnt): a vector load would wait, in order, for the tile in flight
  auto index_of = [&](int64_t tt) -> int64_t {
    if (!rows) {
      const int64_t r = tt * R + ln;
      return r < m ? r : m - 1;
    }
    int64_t v = 0;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t r = tt * R + i;
      const int64_t ri = rows[r < m ? r : m - 1];
      v = ln == i ? ri : v;
    }
    return v;
  };

  f32x4 XA[NJ], XB[NJ];  // two raw row tiles (AGPRs, loaded by asm, waited with wait_vm)
  double st[4] = {0.0, 0.0, 0.0, 0.0};
  double tt[5];
  float tB[5];
  double T2 = 0.0, T2prev = 0.0;

  // ---- sweep 1 on tile Y: partial t (uncentred) → tpart[buf] ----------------
  // ---- lazy view.  The fused forms (score_diag_impl routes the rest through a
  // materialised copy): SNV alone (HH = 0), y = (x − m_r)·s_r, and an
  // odd-derivative filter (HH > 0), y = s_r·Σ_t c_t (x_{j+t} − x_{j−t}), s_r = 1
  // without SNV (a·1 = a exactly: one formula, no per-element selects).
  float ctap[HH > 0 ? HH + 1 : 1];  // interior taps c_1 .. c_HH (wave-uniform)
  if constexpr (HH > 0)
#pragma unroll
    for (int t = 1; t <= HH; ++t) ctap[t] = ptaps[HH + t];
  // (m_r, s_r) of lane row ln of tile tt (scalar loads, selects)
  auto rowstat_of = [&](int64_t tt, float& mr, float& sr) {
    mr = 0.f;
    sr = 1.f;
    if (!PREP || !pa.snv) return;
#pragma unroll
    for (int i = 0; i < R; ++i) {
      const int64_t r = tt * R + i;
      const int64_t rr = r < m ? r : m - 1;
      const int64_t xi = rows ? rows[rr] : rr;
      const float mi = prow[2 * xi], si = prow[2 * xi + 1];
      mr = ln == i ? mi : mr;
      sr = ln == i ? si : sr;
    }
  };
  // y of this lane's four columns of block j from the window u[c0 − HH .. c0 + 3 + HH]
  auto stencil_e = [&](const float* win, float sr, int e) __attribute__((always_inline)) -> float {
    const int o = (HH > 0 ? HH : 0) + e;
    float a;
    if constexpr (HH <= 0) {
      a = win[o];  // x − m_r (the window is mean-subtracted at HH = 0)
    } else {
      a = 0.f;
#pragma unroll
      for (int t = 1; t <= HH; ++t) a = fmaf(ctap[t], __fsub_rn(win[o + t], win[o - t]), a);
    }
    return ocm::mul_nc(a, sr);
  };
  auto stencil = [&](const float* win, float sr) __attribute__((always_inline)) -> f32x4 {
    f32x4 y;
#pragma unroll
    for (int e = 0; e < 4; ++e) y[e] = stencil_e(win, sr, e);
    return y;
  };
  // the first (LEFT) / last HH columns of the row: block 0 of wave 0 or block
  // NJ − 1 of wave 3; the 16 u values of the block's row gathered from its
  // four lanes, the edge rows from the scalar cache
  auto edge_fix = [&](f32x4& y, const f32x4& ucur, float sr, bool left) __attribute__((always_inline)) {  // y: this lane's edge outputs
    if constexpr (HH > 0) {
      f32x4 q1, q2, q3;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        q1[e] = xlane(4 * (lane ^ 16), ucur[e]);
        q2[e] = xlane(4 * (lane ^ 32), ucur[e]);
        q3[e] = xlane(4 * (lane ^ 48), ucur[e]);
      }
      float row16[16];
#pragma unroll
      for (int sq = 0; sq < 4; ++sq)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int kk = lq ^ sq;  // the round that brought quad sq
          row16[4 * sq + e] = kk == 0 ? ucur[e] : kk == 1 ? q1[e] : kk == 2 ? q2[e] : q3[e];
        }
      const int Wn = 2 * HH + 1;
#pragma unroll
      for (int i = 0; i < HH; ++i) {
        const float* et = ptaps + Wn + (left ? i : HH + i) * Wn;
        const int s0 = left ? 0 : 16 - Wn;           // window start within the block
        const int cl = left ? i : 16 - HH + i;       // the output's column within the block
        const float ref = row16[cl];  // deriv ≥ 1
        float a = 0.f;
#pragma unroll
        for (int t = 0; t < Wn; ++t) a = fmaf(et[t], __fsub_rn(row16[s0 + t], ref), a);
        const float yv = ocm::mul_nc(a, sr);
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (4 * lq + e == cl) y[e] = yv;
      }
    }
  };

  // the window u[c0 − HH .. c0 + 3 + HH] of this lane's quad in one block:
  // the neighbouring quads of the row by ds_bpermute (lanes ±16, ±32; the
  // quad before / after the block from the providing lanes' prev / next)
  auto exchange = [&](const f32x4& uprev, const f32x4& ucur, const f32x4& unext, float* win)
      __attribute__((always_inline)) {
    constexpr int H_ = HH > 0 ? HH : 0;
    constexpr int NL1 = H_ < 4 ? H_ : 4;
#pragma unroll
    for (int e = 4 - NL1; e < 4; ++e) {  // quad lq − 1 (block j − 1 for lq = 0)
      win[H_ - 4 + e] = xlane(4 * ((lane + 48) & 63), lq == 3 ? uprev[e] : ucur[e]);
      win[H_ + 4 + (e - (4 - NL1))] =
          xlane(4 * ((lane + 16) & 63), lq == 0 ? unext[e - (4 - NL1)] : ucur[e - (4 - NL1)]);
    }
    if constexpr (H_ > 4) {
#pragma unroll
      for (int e = 8 - H_; e < 4; ++e)  // quad lq − 2
        win[H_ - 8 + e] = xlane(4 * (lane ^ 32), lq >= 2 ? uprev[e] : ucur[e]);
#pragma unroll
      for (int e = 0; e < H_ - 4; ++e)  // quad lq + 2
        win[H_ + 8 + e] = xlane(4 * (lane ^ 32), lq <= 1 ? unext[e] : ucur[e]);
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) win[H_ + e] = ucur[e];
  };

  // XG: vector-memory ops issued after Y's group (the other tile's group in
  // the loop; none for the first tile, whose sweep runs before the second
  // tile's loads are issued — two tiles' loads in flight around the first
  // sweep made the compiler stage some through VGPRs, copying them before
  // they landed: scripts/tile_hazard_check.py)
  auto sweep1 = [&](f32x4 (&Y)[NJ], f32x4& hy, int buf, int64_t tile, auto XGc) __attribute__((always_inline)) {
    constexpr int XG = decltype(XGc)::value;
    f32x4 acA = {0.f, 0.f, 0.f, 0.f}, acB = acA, acC = acA, acD = acA, acE = acA, acF = acA;
    double t64[4] = {0.0, 0.0, 0.0, 0.0}, x164[4] = {0.0, 0.0, 0.0, 0.0};
    f32x4 aN = P0s[b1[0]];  // LDS / crossbar operands one block ahead
    float bN[4] = {0.f, 0.f, 0.f, 0.f};
    if constexpr (EX)
#pragma unroll
      for (int e = 0; e < 4; ++e)
        bN[e] = NOP1B ? xlane(bpermA + 4 * e, p1a[0])
                      : __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(bperm + 4 * e, __builtin_bit_cast(int, p1b[0])));
    // the A / B operands of block j (taken from the prefetch) and block j + 1's prefetch
    auto operands = [&](auto J, f32x4& a, float (&b)[4]) __attribute__((always_inline)) {
      constexpr int j = decltype(J)::value;
      a = aN;
#pragma unroll
      for (int e = 0; e < 4; ++e) b[e] = bN[e];
      if constexpr (j + 1 < NJ) {
        aN = P0s[b1[(j + 1) & 3] + 16 * ((j + 1) >> 2)];
        if constexpr (EX)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            bN[e] = __builtin_bit_cast(float,
                                       __builtin_amdgcn_ds_bpermute(NOP1B ? bpermA + 4 * e : bperm + 4 * e,
                                                                    __builtin_bit_cast(int, NOP1B ? p1a[j + 1] : p1b[NOP1B ? 0 : j + 1])));
      }
    };
    // f32 partials over ≤ 64 columns per chain, flushed to f64.  The MFMAs are
    // asm (hipcc pads no hazard of theirs): the s_nop covers MFMA result →
    // VALU read, and ties the accumulators so no read is scheduled above it
    // (a "memory" clobber orders loads and stores only — with it, the reads of
    // the last MFMA's first elements had moved up and read stale values)
    auto flush = [&]() __attribute__((always_inline)) {
      asm volatile("s_nop 11" : "+v"(acA), "+v"(acB), "+v"(acC), "+v"(acD), "+v"(acE), "+v"(acF));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        t64[i] += ((double)acA[i] + (double)acB[i]) + ((double)acC[i] + (double)acD[i]);
        x164[i] += (double)acE[i] + (double)acF[i];
        acA[i] = acB[i] = acC[i] = acD[i] = acE[i] = acF[i] = 0.f;
      }
    };
    if constexpr (!PREP) {
      static_for<NJ>([&](auto J) {
        constexpr int j = decltype(J)::value;
        f32x4 a;
        float b[4];
        operands(J, a, b);
        // Y[j] was issued before the rest of its tile (NJ − 1 − j loads) and
        // the NJ refills of the other tile (stores issued since only make the
        // wait earlier)
        wait_vm<NJ - 1 - j + XG>(Y[j]);
        s1_block<EX>(acA, acB, acC, acD, acE, acF, a, b, Y[j]);
        __builtin_amdgcn_sched_barrier(0);  // keep the scheduler from hoisting every block's reads
        if constexpr ((j & 15) == 15 || j == NJ - 1) {
          flush();
        }
      });
    } else {
      // Lazy view, two blocks in flight: block j's MFMAs (compiler builtins,
      // so the scheduler can fill their issue gaps) run beside the stencil of
      // block j + 1 (its window was exchanged during block j − 1) and the
      // ds_bpermute exchange of block j + 2's window.  y_j replaces x_j in the
      // AGPR tile once its MFMAs are issued (sweep 2 and the epilogue read it
      // there).
      constexpr int H_ = HH > 0 ? HH : 0;
      float win[4 + 2 * H_];
      float mr, sr;
      rowstat_of(tile, mr, sr);
      // hy, Y[0..2] (the oldest loads of the tile's group) have landed: the
      // rest of this group and the other tile's whole group may be in flight
      constexpr int W0 = NJ - 3 + XG < 63 ? NJ - 3 + XG : 63;
      wait_vm<W0>(Y[2]);
      wait_vm<W0>(Y[1]);
      wait_vm<W0>(Y[0]);
      wait_vv<W0>(hy);
      auto raw = [&](const f32x4& v) __attribute__((always_inline)) {
        f32x4 u = v;
        if constexpr (HH == 0)  // SNV alone subtracts the row mean first
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = __fsub_rn(u[e], mr);
        return u;
      };
      f32x4 uprev = raw(hy), ucur = raw(Y[0]), unext = raw(Y[1]);
      // the row ends first (wave 0: block 0, wave 3: block NJ − 1)
      f32x4 yE = {0.f, 0.f, 0.f, 0.f};  // this lane's outputs among the row's first / last HH columns
      if constexpr (HH > 0) {
        // every wave waits (the tile's group landed during the last sweep 2):
        // a tied wait inside the branch would make the compiler merge two
        // versions of Y[NJ − 1] with register copies, and copying a tile
        // register whose load is in flight reads garbage
        wait_vm<XG>(Y[NJ - 1]);
        if (w == 0) edge_fix(yE, ucur, sr, true);
        if (w == W - 1) edge_fix(yE, raw(Y[NJ - 1]), sr, false);
      }
      auto patch = [&](f32x4& y, bool right) __attribute__((always_inline)) {
        if constexpr (HH > 0)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int cl = 4 * lq + e;  // column within the block
            const bool ed = right ? (w == W - 1) & (cl >= 16 - HH) : (w == 0) & (cl < HH);
            y[e] = ed ? yE[e] : y[e];
          }
      };
      auto advance = [&](const f32x4& nx) __attribute__((always_inline)) {
        unext = raw(nx);
        exchange(uprev, ucur, unext, win);
        uprev = ucur;
        ucur = unext;
      };
      exchange(uprev, ucur, unext, win);  // block 0's window
      uprev = ucur;
      ucur = unext;
      f32x4 y = stencil(win, sr);
      patch(y, false);
      if constexpr (NJ == 1) patch(y, true);
      advance(Y[2]);  // block 1's window
      static_for<NJ>([&](auto J) {
        constexpr int j = decltype(J)::value;
        f32x4 a;
        float b[4];
        operands(J, a, b);
        // block j's MFMAs as compiler builtins (it pads their hazards — an asm
        // MFMA's sources were rewritten by the next VALU while it still read
        // them — and fills their issue gaps with block j + 1's stencil; the
        // accumulators stay in VGPRs, -amdgpu-mfma-vgpr-form, Makefile: the
        // AGPRs are the tiles, whose in-flight loads must never be copied)
        f32x4 yn = y;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (EX)
            (e & 1 ? acF : acE) = __builtin_amdgcn_mfma_f32_4x4x1f32(b[e], y[e], e & 1 ? acF : acE, 0, 0, 0);
          f32x4& c = e == 0 ? acA : e == 1 ? acB : e == 2 ? acC : acD;
          c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[e], y[e], c, 0, 0, 0);
          if constexpr (j + 1 < NJ) yn[e] = stencil_e(win, sr, e);
        }
        asm volatile("" : "=a"(Y[j]) : "0"(y));  // y into the AGPR tile
        if constexpr (j + 1 < NJ) {
          y = yn;
          if constexpr (j + 1 == NJ - 1) patch(y, true);
          if constexpr (j + 2 < NJ) {  // block j + 2's window: Y[j + 3] (or the halo) has landed
            if constexpr (j + 3 < NJ) {
              wait_vm<NJ - 4 - j + XG>(Y[j + 3]);
              advance(Y[j + 3]);
            } else {
              advance(hy);  // lanes lq <= 1: virtual block NJ
            }
          }
        }
        __builtin_amdgcn_sched_barrier(0);
        if constexpr ((j & 15) == 15 || j == NJ - 1) {
          flush();
        }
      });
    }
    if constexpr (TPB == 1) {
      // one buffer: every wave has read the previous tile's t (compute_t,
      // right after the last barrier) before any wave overwrites it
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
    }
    double* tp = tpart[TPB == 1 ? 0 : buf];
#pragma unroll
    for (int i = 0; i < 4; ++i) tp[(w * 20 + 4 * lq + i) * R + ln] = t64[i];
    if constexpr (EX) {  // comps 16..19: lane (ln, lq) holds the partial over its column quarter lq
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        x164[u] += __shfl_xor(x164[u], 16, 64);
        x164[u] += __shfl_xor(x164[u], 32, 64);
      }
      if (lq == 0)
#pragma unroll
        for (int u = 0; u < 4; ++u) tp[(w * 20 + 16 + u) * R + ln] = x164[u];
    }
  };
  // ---- full t of this lane's comps lq + 4s (row ln) from tpart[buf]; T², T --
  auto compute_t = [&](int64_t t, int buf) {
    const double* tp = tpart[TPB == 1 ? 0 : buf];
#pragma unroll
    for (int s = 0; s < 5; ++s) {
      double v = 0.0;
      if (s < 4 || EX) {
#pragma unroll
        for (int ww = 0; ww < W; ++ww) v += tp[(ww * 20 + lq + 4 * s) * R + ln];
        v -= pmuL[lq + 4 * s];  // t = P·x − P·μ
      }
      tt[s] = v;
    }
    T2 = 0.0;
#pragma unroll
    for (int s = 0; s < 5; ++s) T2 += tt[s] * tt[s] * (WV == 8 ? adL[lq + 4 * s] : ad[s < (WV == 8 ? 1 : 5) ? s : 0]);
    T2 += __shfl_xor(T2, 16, 64);
    T2 += __shfl_xor(T2, 32, 64);
    const int64_t row = t * R + ln;
    if (T_out && w == 0 && row < m)
#pragma unroll
      for (int s = 0; s < 5; ++s)
        if (lq + 4 * s < k) T_out[row * k + lq + 4 * s] = (float)tt[s];
#pragma unroll
    for (int s = 0; s < 5; ++s) tB[s] = -(float)tt[s];  // r = x − μ + Pᵀ(−t)
  };
  // ---- sweep 2 on tile Z (raw x of the tile being scored): Q partials →
  // qpart[buf]; each consumed block pair of Z is refilled from `pre`
  // a lazy view's halo quad of the tile whose row pointer is `pre`: lanes
  // lq ≥ 2 the quad of virtual block −1, lanes lq ≤ 1 of virtual block NJ (an
  // in-row address at the row's ends, where the edge rows replace the stencil)
  auto halo_ptr = [&](const float* pre) -> const float* {
    const bool left = lq >= 2;
    return left ? (w > 0 ? pre - 16 : pre) : (w < W - 1 ? pre + 16 * NJ : pre);
  };
  auto sweep2 = [&](f32x4 (&Z)[NJ], f32x4& hz, const float* pre, int buf) __attribute__((always_inline)) {
    if constexpr (HH > 0) load_v(hz, halo_ptr(pre));  // first load of the refilled tile's group
    float q[4] = {0.f, 0.f, 0.f, 0.f};
    double q64 = 0.0;
    float aN[2][5], mN[2];  // A operands of the next block pair (one pair ahead)
    auto read_a = [&](auto J, float (&dst)[5], float& mdst) {
      constexpr int j = decltype(J)::value;
#pragma unroll
      for (int s = 0; s < 4; ++s) dst[s] = p0f[b2[s][j & 3] + 64 * (j >> 2)];
      dst[4] = EX ? p1a[j] : 0.f;
      mdst = nmuL[w * PW + 16 * j + 4 * lq + (ln & 3)];  // 4x4x1 A: block l/4, row l&3
    };
    read_a(std::integral_constant<int, 0>{}, aN[0], mN[0]);
    read_a(std::integral_constant<int, 1>{}, aN[1], mN[1]);
    static_for<NJ / 2>([&](auto H) {
      constexpr int j = 2 * decltype(H)::value;
      float a0[5], a1[5];
#pragma unroll
      for (int s = 0; s < 5; ++s) {
        a0[s] = aN[0][s];
        a1[s] = aN[1][s];
      }
      const float m0 = mN[0], m1 = mN[1];
      if constexpr (j + 2 < NJ) {
        read_a(std::integral_constant<int, j + 2>{}, aN[0], mN[0]);
        read_a(std::integral_constant<int, j + 3>{}, aN[1], mN[1]);
      }
      // r is formed in place of x (the tile registers are all the AGPRs there
      // are at NJ = 32; a separate result would push tile quads into VGPRs and
      // the compiler would copy them before their loads had landed); the
      // previous pair's r is squared into q inside this pair's MFMA stream and
      // only then refilled
      if constexpr (j == 0) {
        s2_pair<EX, false>(Z[0], Z[1], a0, a1, m0, m1, tB, one, Z[0], Z[1], q);
      } else {
        s2_pair<EX, true>(Z[j], Z[j + 1], a0, a1, m0, m1, tB, one, Z[j - 2], Z[j - 1], q);
        __builtin_amdgcn_sched_barrier(0);
        refill_a<64 * (j - 2)>(Z[j - 2], pre);
        refill_a<64 * (j - 1)>(Z[j - 1], pre);
        if constexpr (((j - 2) & 15) == 14) {  // f32 q partials over ≤ 16 columns each per lane
          q64 += ((double)q[0] + (double)q[1]) + ((double)q[2] + (double)q[3]);
          q[0] = q[1] = q[2] = q[3] = 0.f;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    });
    // the last pair: its MFMA results → VALU reads, then its refill
    asm volatile("s_nop 11" : "+a"(Z[NJ - 2]), "+a"(Z[NJ - 1]));
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      q[e & 1] = fmaf(Z[NJ - 2][e], Z[NJ - 2][e], q[e & 1]);
      q[2 + (e & 1)] = fmaf(Z[NJ - 1][e], Z[NJ - 1][e], q[2 + (e & 1)]);
    }
    __builtin_amdgcn_sched_barrier(0);
    refill_a<64 * (NJ - 2)>(Z[NJ - 2], pre);
    refill_a<64 * (NJ - 1)>(Z[NJ - 1], pre);
    q64 += ((double)q[0] + (double)q[1]) + ((double)q[2] + (double)q[3]);
    q64 += __shfl_xor(q64, 16, 64);
    q64 += __shfl_xor(q64, 32, 64);
    if (lq == 0) qpart[buf][w * R + ln] = q64;
  };
  // outputs of tile t from qpart[buf] (T² of t was kept in T2prev)
  auto finish = [&](int64_t t, int buf) {
    double Q = 0.0;
#pragma unroll
    for (int ww = 0; ww < W; ++ww) Q += qpart[buf][ww * R + ln];
    const int64_t row = t * R + ln;
    if (w == 0 && lq == 0 && row < m) {
      const float Qf = (float)Q;
      if (T2_out) T2_out[row] = T2prev;
      if (Q_out) Q_out[row] = Qf;
      if (dec.enabled) {
        const double dr = ocm::dred_of(dec.type, T2prev * dec.t2_scale, (double)Qf * dec.q_scale);
        acc_out[row * acc_stride] = dr < dec.dlim ? 1.0 : 0.0;
      }
      st[0] += T2prev;
      st[1] += T2prev * T2prev;
      st[2] += (double)Qf;
      st[3] += (double)Qf * (double)Qf;
    }
  };
  // LDS hand-off between the waves: no global access is waited for
  auto lds_barrier = [&]() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  };

  // ---- tile pipeline: tiles t_i = blockIdx.x + i·G.  step(X, Y) scores t (in
  // X, sweep 2) while t + 2G streams into X, then sweep 1 of t + G (in Y);
  // unrolled by two so X / Y swap roles.  Past the last tile the refills
  // re-read a valid tile.
  int64_t t = blockIdx.x;
  auto clamp_tile = [&](int64_t tt) { return tt < ntiles ? tt : t; };
  f32x4 hA = {0.f, 0.f, 0.f, 0.f}, hB = hA;  // lazy view: the tiles' halo quads
  {
    const float* p0 = col_base(index_of(t));
    if constexpr (HH > 0) load_v(hA, halo_ptr(p0));
    static_for<NJ>([&](auto J) { load_a<64 * decltype(J)::value>(XA[decltype(J)::value], p0); });
  }
  sweep1(XA, hA, 0, t, std::integral_constant<int, 0>{});
  {
    const float* p1 = col_base(index_of(clamp_tile(t + G)));
    if constexpr (HH > 0) load_v(hB, halo_ptr(p1));
    static_for<NJ>([&](auto J) { load_a<64 * decltype(J)::value>(XB[decltype(J)::value], p1); });
  }
  lds_barrier();
  compute_t(t, 0);
  int buf = 0;
#ifdef OCM_S1P_STAMPS  // diagnostic build (make exp): Σ cycles per phase replace the moment partials
  double cyc[4] = {0.0, 0.0, 0.0, 0.0};
  uint64_t c_last = __builtin_readcyclecounter();
#define OCM_STAMP(I)                                    \
  {                                                     \
    const uint64_t c_now = __builtin_readcyclecounter(); \
    cyc[I] += (double)(c_now - c_last);                  \
    c_last = c_now;                                      \
  }
#else
#define OCM_STAMP(I)
#endif
  auto step = [&](f32x4 (&Xc)[NJ], f32x4& hc, f32x4 (&Yn)[NJ], f32x4& hn) __attribute__((always_inline)) -> bool {
    const int64_t tn = t + G;
    const bool more = tn < ntiles;
    OCM_STAMP(3)
    sweep2(Xc, hc, col_base(index_of(clamp_tile(tn + G))), buf);
    OCM_STAMP(0)
    if (more || PREP) sweep1(Yn, hn, buf ^ 1, tn, std::integral_constant<int, GL>{});  // lazy view: unconditional (a tile past the end is a clamped valid one), so Yn never merges raw and transformed values
    OCM_STAMP(1)
    lds_barrier();
    OCM_STAMP(2)
    T2prev = T2;
    finish(t, buf);
    if (!more) return false;
    t = tn;
    buf ^= 1;
    compute_t(t, buf);
    return true;
  };
#undef OCM_STAMP
  for (;;) {
    if (!step(XA, hA, XB, hB)) break;
    if (!step(XB, hB, XA, hA)) break;
  }
  // drain the refills past the last tile before the wave ends
#pragma unroll
  for (int j = 0; j < NJ; ++j) {
    wait_vm<0>(XA[j]);
    wait_vm<0>(XB[j]);
  }
  if constexpr (HH > 0) {
    wait_vv<0>(hA);
    wait_vv<0>(hB);
  }
#ifdef OCM_S1P_STAMPS
#pragma unroll
  for (int i = 0; i < 4; ++i) st[i] = cyc[i] / 64.0;  // the wave sum below restores the wave's total
#endif
  if (stat_part) {
#pragma unroll
    for (int i = 0; i < 4; ++i) st[i] = wave_sum_f64(st[i]);
    if (w == 0 && lane == 0)
#pragma unroll
      for (int i = 0; i < 4; ++i) stat_part[(int64_t)blockIdx.x * 4 + i] = st[i];
  }
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

// q_i = Σ_j (s(x_ij) − s(x̂_ij))² with s(v) = clamp((v − min_j x_ij)/(max_j x_ij − min_j x_ij + eps), 0, 1):
// the per-sample min–max scaled residual of utils/final_vaesimca.py:417-423 /
// 484-490 (its BCE-trained networks).  The scaling is evaluated in float32 in
// the reference's operation order; the sum of squares in f64.  One wave per row.
__global__ __launch_bounds__(256) void k_rowsq_minmax(const float* __restrict__ x, int64_t ldx,
                                                      const float* __restrict__ xh, int64_t ldxh, int64_t m, int p,
                                                      float eps, float* __restrict__ q) {
  const int64_t r = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (r >= m) return;
  const float* xr = x + r * ldx;
  const float* hr = xh + r * ldxh;
  float lo = INFINITY, hi = -INFINITY;
  for (int j = lane; j < p; j += 64) {
    const float v = xr[j];
    lo = fminf(lo, v);
    hi = fmaxf(hi, v);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    lo = fminf(lo, __shfl_xor(lo, o, 64));
    hi = fmaxf(hi, __shfl_xor(hi, o, 64));
  }
  const float den = (hi - lo) + eps;
  double s = 0.0;
  for (int j = lane; j < p; j += 64) {
    const float a = fminf(fmaxf((xr[j] - lo) / den, 0.f), 1.f);
    const float b = fminf(fmaxf((hr[j] - lo) / den, 0.f), 1.f);
    const float d = a - b;
    s += (double)(d * d);
  }
  s = wave_sum_f64(s);
  if (lane == 0) q[r] = (float)s;
}

__global__ void k_cast_f64_f32(const double* __restrict__ a, int64_t n, float* __restrict__ b) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) b[i] = (float)a[i];
}

// k_score_direct launch; a_diag: A is the k-vector diag(A).  k ≤ 64: one
// launch.  k > 64 (diagonal A only): component blocks of ≤ 64 in turn, each
// launch projecting the previous block's residual (the first block reads X and
// subtracts μ; the residual matrix R is written by every launch but the last,
// in place after the first), accumulating T² and writing its columns of T;
// the last block gives Q = ‖final residual‖², the decision and the moments.
// The loadings are orthonormal, so P_b·(y − P_aᵀt_a) = P_b·y up to rounding:
// the same T, T², Q as one pass, in the reference's float32 residual
// arithmetic (utils/SIMCA.py:67-68).
int score_direct(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                 const double* P, const double* mu, const double* A, int a_diag, int32_t k, float* T_out,
                 double* T2_out, float* Q_out, const ocm_decision* dec, double* accept_out, int64_t accept_stride,
                 double* stats_out, hipStream_t st) {
  if (m == 0) {
    if (stats_out) OCM_HIP(hipMemsetAsync(stats_out, 0, 4 * sizeof(double), st));
    return OCM_OK;
  }
  constexpr int KB = 64;  // components per launch
  const int nkb = (k + KB - 1) / KB;
  OCM_REQUIRE(nkb == 1 || a_diag, "ocm_score_f32: k > 64 needs a diagonal quadratic form (ocm_score_f32_diag)");
  const int64_t rows_per_blk = SROWS;
  const int64_t nblk = (m + rows_per_blk - 1) / rows_per_blk;
  OCM_REQUIRE(nblk < (1LL << 31), "ocm_score_f32: too many rows");
  const size_t part_bytes = stats_out ? (size_t)nblk * 4 * sizeof(double) : 0;
  const size_t cast_bytes = ((size_t)k * p + 2 * (size_t)p) * sizeof(float) + 1024;
  const bool need_t2 = nkb > 1 && !T2_out;  // the running T² between blocks
  const size_t extra = nkb > 1 ? (size_t)m * p * sizeof(float) + (need_t2 ? (size_t)m * sizeof(double) : 0) + 512 : 0;
  void* w = ocm::workspace(ctx, part_bytes + cast_bytes + extra + 1024, st);
  if (!w) return OCM_ERR_NOMEM;
  ocm::Carve cv{static_cast<char*>(w)};
  double* part = stats_out ? cv.take<double>((size_t)nblk * 4) : nullptr;
  // the f32 kernel takes f32 loadings / mean
  float* P32 = cv.take<float>((size_t)k * p);
  float* mu32 = cv.take<float>(p);
  float* zero32 = cv.take<float>(p);
  float* R = nkb > 1 ? cv.take<float>((size_t)m * p) : nullptr;
  double* T2run = nkb > 1 ? (T2_out ? T2_out : cv.take<double>((size_t)m)) : T2_out;
  hipLaunchKernelGGL(k_cast_f64_f32, dim3((unsigned)(((int64_t)k * p + 255) / 256)), dim3(256), 0, st, P,
                     (int64_t)k * p, P32);
  hipLaunchKernelGGL(k_cast_f64_f32, dim3((p + 255) / 256), dim3(256), 0, st, mu, (int64_t)p, mu32);
  OCM_CHECK_LAUNCH("k_cast_f64_f32");
  if (nkb > 1) OCM_HIP(hipMemsetAsync(zero32, 0, (size_t)p * sizeof(float), st));
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
  for (int bk = 0; bk < nkb; ++bk) {
    const int c0 = bk * KB, kb = std::min(KB, k - c0);
    const bool first = bk == 0, last = bk == nkb - 1;
    // input of this block: X (rows / ldx / μ) first, then the residual R (dense, μ = 0)
    const float* Xin = first ? X : R;
    const int64_t ldin = first ? ldx : (int64_t)p;
    const int64_t* rin = first ? rows : nullptr;
    const bool vin = first ? vec : (p % 4 == 0);
    const float* muin = first ? mu32 : zero32;
    float* Tb = T_out ? T_out + c0 : nullptr;
    const double* Ab = A + c0;  // diagonal entries of this block (a_diag) or the whole A (nkb == 1)
    DecArgs db = last ? d : DecArgs{};
    ocm::TimedRegion tr(ctx, OCM_KERNEL_SCORE, st);
#define OCM_SCORE_LAUNCH(KT_, V_)                                                                              \
  hipLaunchKernelGGL((k_score_direct<KT_, V_>), g, dim3(256), 0, st, Xin, ldin, rin, m, p, P32 + (size_t)c0 * p, \
                     muin, Ab, kb, a_diag, Tb, last ? T2_out : T2run, last ? Q_out : nullptr, db,             \
                     last ? accept_out : nullptr, accept_stride, last ? part : nullptr, k,                    \
                     first ? nullptr : T2run, last ? nullptr : R, (int64_t)p)
    if (kb <= 32) {
      if (vin) OCM_SCORE_LAUNCH(1, true); else OCM_SCORE_LAUNCH(1, false);
    } else {
      if (vin) OCM_SCORE_LAUNCH(2, true); else OCM_SCORE_LAUNCH(2, false);
    }
#undef OCM_SCORE_LAUNCH
    OCM_CHECK_LAUNCH("k_score");
  }
  if (stats_out) {
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(1024), 0, st, part, nblk, stats_out);
    OCM_CHECK_LAUNCH("k_stats_reduce");
  }
  return OCM_OK;
}

}  // namespace

extern "C" {

int ocm_score_f32(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                  const double* P, const double* mu, const double* A, int32_t k, float* T_out, double* T2_out,
                  float* Q_out, const ocm_decision* dec, double* accept_out, int64_t accept_stride,
                  double* stats_out, void* stream) {
  OCM_REQUIRE(ctx && X && P && mu && A, "ocm_score_f32: NULL argument");
  OCM_REQUIRE(m >= 0 && p > 0 && ldx >= p, "ocm_score_f32: bad shape");
  OCM_REQUIRE(k >= 1 && k <= 64, "ocm_score_f32: 1 <= k <= 64 (larger k: ocm_score_f32_diag)");
  OCM_REQUIRE(!dec || accept_out, "ocm_score_f32: decision requires accept_out");
  // general k×k quadratic form (k² FMAs per row are negligible)
  return score_direct(ctx, X, ldx, rows, m, p, P, mu, A, 0, k, T_out, T2_out, Q_out, dec, accept_out,
                      accept_stride, stats_out, (hipStream_t)stream);
}

}  // extern "C"

namespace {

int score_diag_impl(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                    const PrepArgs* pp, const double* P, const double* mu, const double* a_diag, int32_t k,
                    float* T_out, double* T2_out, float* Q_out, const ocm_decision* dec, double* accept_out,
                    int64_t accept_stride, double* stats_out, hipStream_t st) {
  int nj = p / 64;
  const bool vec = (ldx % 4 == 0) && ((reinterpret_cast<uintptr_t>(X) & 15) == 0);
  bool one_pass = vec && p % 64 == 0 && (nj == 4 || nj == 8 || nj == 16 || nj == 32) && k <= 20;
  const PrepArgs pa = pp ? *pp : PrepArgs{};
  if (pp && !pa.fused_form()) one_pass = false;
  if (!one_pass && pp) {  // a lazy view on the other shapes: materialise the rows, then score them
    if (m == 0) {
      if (stats_out) OCM_HIP(hipMemsetAsync(stats_out, 0, 4 * sizeof(double), st));
      return OCM_OK;
    }
    float* Y = nullptr;
    OCM_HIP(hipMallocAsync(reinterpret_cast<void**>(&Y), (size_t)m * p * sizeof(float), st));
    ++ctx->prep_materialised;
    int rc = ocm::prep_apply(ctx, X, ldx, rows, m, p, pa, Y, p, st);
    if (rc == OCM_OK)
      rc = score_diag_impl(ctx, Y, p, nullptr, m, p, nullptr, P, mu, a_diag, k, T_out, T2_out, Q_out, dec,
                           accept_out, accept_stride, stats_out, st);
    const hipError_t e = hipFreeAsync(Y, st);
    if (rc == OCM_OK && e != hipSuccess) return ocm::fail(OCM_ERR_HIP, std::string("hipFreeAsync: ") + hipGetErrorString(e));
    return rc;
  }
  if (!one_pass)  // other shapes: the two-sweep kernel
    return score_direct(ctx, X, ldx, rows, m, p, P, mu, a_diag, 1, k, T_out, T2_out, Q_out, dec, accept_out,
                        accept_stride, stats_out, st);
  if (m == 0) {
    if (stats_out) OCM_HIP(hipMemsetAsync(stats_out, 0, 4 * sizeof(double), st));
    return OCM_OK;
  }
  const int64_t ntiles = (m + s1p::R - 1) / s1p::R;
  const int grid = (int)std::min<int64_t>(ctx->num_cus, ntiles);
  double* part = nullptr;
  if (stats_out) {
    void* wsp = ocm::workspace(ctx, (size_t)grid * 4 * sizeof(double) + 256, st);
    if (!wsp) return OCM_ERR_NOMEM;
    part = static_cast<double*>(wsp);
  }
  DecArgs d{};
  if (dec) {
    d.enabled = 1;
    d.type = dec->type;
    d.t2_scale = dec->t2_scale;
    d.q_scale = dec->q_scale;
    d.dlim = dec->dlim;
  }
  {
    ocm::TimedRegion tr(ctx, OCM_KERNEL_SCORE, st);
#define OCM_S1P_H(NJ_, EX_, H_)                                                                                 \
  hipLaunchKernelGGL((k_score_1p<NJ_, EX_, H_>), dim3(grid), dim3(256), 0, st, X, ldx, rows, m, P, mu, a_diag, k, \
                     T_out, T2_out, Q_out, d, accept_out, accept_stride, part, ntiles, pa, pa.taps, pa.rowstat)
#ifdef OCM_S1P_W8  // make exp A/B: two waves per SIMD at p = 2048 (plain rows)
    if (nj == 32 && !pp && s1p_w8_enabled()) {
      if (k > 16)
        hipLaunchKernelGGL((k_score_1p<16, true, -1, 8>), dim3(grid), dim3(512), 0, st, X, ldx, rows, m, P, mu, a_diag,
                           k, T_out, T2_out, Q_out, d, accept_out, accept_stride, part, ntiles, pa, pa.taps,
                           pa.rowstat);
      else
        hipLaunchKernelGGL((k_score_1p<16, false, -1, 8>), dim3(grid), dim3(512), 0, st, X, ldx, rows, m, P, mu,
                           a_diag, k, T_out, T2_out, Q_out, d, accept_out, accept_stride, part, ntiles, pa, pa.taps,
                           pa.rowstat);
      nj = 0;  // launched
    }
#endif
#define OCM_S1P(NJ_, EX_)                                  \
  if (!pp)                                                 \
    OCM_S1P_H(NJ_, EX_, -1);                               \
  else if (pa.h == 0)                                      \
    OCM_S1P_H(NJ_, EX_, 0);                                \
  else if (pa.h == 2)                                      \
    OCM_S1P_H(NJ_, EX_, 2);                                \
  else                                                     \
    OCM_S1P_H(NJ_, EX_, 7);
#define OCM_S1P_K(NJ_) \
  if (k > 16) {        \
    OCM_S1P(NJ_, true) \
  } else {             \
    OCM_S1P(NJ_, false) \
  }
    if (nj == 0) {
    } else if (nj == 32) {
      OCM_S1P_K(32)
    } else if (nj == 16) {
      OCM_S1P_K(16)
    } else if (nj == 8) {
      OCM_S1P_K(8)
    } else {
      OCM_S1P_K(4)
    }
#undef OCM_S1P_K
#undef OCM_S1P
#undef OCM_S1P_H
  }
  OCM_CHECK_LAUNCH("k_score_1p");
  if (stats_out) {
    hipLaunchKernelGGL(k_stats_reduce, dim3(1), dim3(1024), 0, st, part, (int64_t)grid, stats_out);
    OCM_CHECK_LAUNCH("k_stats_reduce");
  }
  return OCM_OK;
}

}  // namespace

extern "C" {

int ocm_score_f32_diag(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                       const double* P, const double* mu, const double* a_diag, int32_t k, float* T_out,
                       double* T2_out, float* Q_out, const ocm_decision* dec, double* accept_out,
                       int64_t accept_stride, double* stats_out, void* stream) {
  OCM_REQUIRE(ctx && X && P && mu && a_diag, "ocm_score_f32_diag: NULL argument");
  OCM_REQUIRE(m >= 0 && p > 0 && ldx >= p, "ocm_score_f32_diag: bad shape");
  OCM_REQUIRE(k >= 1 && k <= p, "ocm_score_f32_diag: 1 <= k <= p");
  OCM_REQUIRE(!dec || accept_out, "ocm_score_f32_diag: decision requires accept_out");
  return score_diag_impl(ctx, X, ldx, rows, m, p, nullptr, P, mu, a_diag, k, T_out, T2_out, Q_out, dec, accept_out,
                         accept_stride, stats_out, (hipStream_t)stream);
}

int ocm_score_f32_diag_prep(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int32_t p,
                            const ocm_prep* prep, const double* P, const double* mu, const double* a_diag, int32_t k,
                            float* T_out, double* T2_out, float* Q_out, const ocm_decision* dec,
                            double* accept_out, int64_t accept_stride, double* stats_out, void* stream) {
  OCM_REQUIRE(ctx && X && P && mu && a_diag, "ocm_score_f32_diag_prep: NULL argument");
  OCM_REQUIRE(m >= 0 && p > 0 && ldx >= p, "ocm_score_f32_diag_prep: bad shape");
  OCM_REQUIRE(k >= 1 && k <= p, "ocm_score_f32_diag_prep: 1 <= k <= p");
  OCM_REQUIRE(!dec || accept_out, "ocm_score_f32_diag_prep: decision requires accept_out");
  if (int rc = ocm::check_prep(prep, p, "ocm_score_f32_diag_prep")) return rc;
  const PrepArgs pa = ocm::prep_args(prep);
  return score_diag_impl(ctx, X, ldx, rows, m, p, &pa, P, mu, a_diag, k, T_out, T2_out, Q_out, dec, accept_out,
                         accept_stride, stats_out, (hipStream_t)stream);
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

int ocm_rowsq_minmax_f32(ocm_ctx* ctx, const float* x, int64_t ldx, const float* xhat, int64_t ldxh, int64_t m,
                         int32_t p, float eps, float* q_out, void* stream) {
  OCM_REQUIRE(ctx && x && xhat && q_out, "ocm_rowsq_minmax_f32: NULL argument");
  OCM_REQUIRE(p > 0 && ldx >= p && ldxh >= p, "ocm_rowsq_minmax_f32: bad shape");
  if (m <= 0) return OCM_OK;
  hipLaunchKernelGGL(k_rowsq_minmax, dim3((unsigned)((m + 3) / 4)), dim3(256), 0, (hipStream_t)stream, x, ldx, xhat,
                     ldxh, m, p, eps, q_out);
  OCM_CHECK_LAUNCH("k_rowsq_minmax");
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
