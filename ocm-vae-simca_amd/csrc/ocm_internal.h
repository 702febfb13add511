// Internal helpers shared by the libocm translation units (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>
#include <utility>
#include <vector>

#include "ocm.h"

struct ocm_ctx {
  int device = 0;
  void* ws = nullptr;  // device workspace, grows on demand (ocm_ctx_reserve pre-sizes it)
  size_t ws_bytes = 0;
  void* ws_aux = nullptr;  // second grow-only arena for buffers that live across a call that takes `ws`
  size_t ws_aux_bytes = 0;
  void* host_pinned = nullptr;  // small pinned staging area for D2H scalars
  size_t host_bytes = 0;
  int num_cus = 256;
  uint32_t last_gram_marks = 0;  // outlier-guard marks of the last i8×3 Gram (ocm_gram_last_marks)
  int64_t prep_materialised = 0;  // lazy views written out by a fallback path (ocm_prep_materialised)
  // live kernel timing (ocm_ctx_set_timing): event pairs per timed kernel
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[OCM_TIMED_KERNELS];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  // side stream + events of the quantiser / Gram overlap (created on first use)
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> fork_ev;
  // the eigensolver's θ work beside its Jacobi (created on first use): a side
  // stream, fork / join events, and a sub-context whose workspaces the θ3
  // Gram takes (the main workspace holds the eigensolver's live buffers)
  hipStream_t eig_side[2] = {nullptr, nullptr};
  hipEvent_t eig_ev[7] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  ocm_ctx* eig_sub = nullptr;
  // the Rayleigh–Ritz test's in-flight hand-off (k_rr_resid32 → k_jacobi_1b):
  // a device counter raised to eig_epoch when S is stored; it only grows
  unsigned* eig_flag = nullptr;
  unsigned eig_epoch = 0;
  // Rayleigh–Ritz tests re-run because the fused test's wait for S timed out
  int64_t eig_test_reruns = 0;
};

namespace ocm {

// Record a start/stop event pair around a launch when timing is enabled.
struct TimedRegion {
  ocm_ctx* ctx;
  int id;
  hipStream_t st;
  std::pair<hipEvent_t, hipEvent_t> pr{nullptr, nullptr};
  TimedRegion(ocm_ctx* c, int i, hipStream_t s, bool on = true) : ctx(c), id(i), st(s) {
    if (!ctx->timing || !on) return;
    if (!ctx->ev_pool.empty()) {
      pr = ctx->ev_pool.back();
      ctx->ev_pool.pop_back();
    } else {
      (void)hipEventCreate(&pr.first);
      (void)hipEventCreate(&pr.second);
    }
    (void)hipEventRecord(pr.first, st);
  }
  ~TimedRegion() {
    if (!pr.first) return;
    (void)hipEventRecord(pr.second, st);
    ctx->ev[id].push_back(pr);
  }
};

void set_error(const std::string& msg);
int fail(int code, const std::string& msg);

// Workspace carve-out: returns a 256-byte aligned pointer into ctx->ws after
// growing it to at least `bytes` (all outstanding work on `stream` is drained
// before a re-allocation).
void* workspace(ocm_ctx* ctx, size_t bytes, hipStream_t stream);
void* workspace_aux(ocm_ctx* ctx, size_t bytes, hipStream_t stream);
void* host_staging(ocm_ctx* ctx, size_t bytes);

inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

struct Carve {
  char* base;
  size_t off = 0;
  template <typename T>
  T* take(size_t count) {
    off = align_up(off, 256);
    T* p = reinterpret_cast<T*>(base + off);
    off += count * sizeof(T);
    return p;
  }
};

// Reduced distance of a decision rule (utils/SIMCA.py:131-144):
// sim max(t, q), alt √(t²+q²), ci / dd t + q.
__device__ __forceinline__ double dred_of(int type, double t, double q) {
  switch (type) {
    case OCM_TYPE_SIM: return fmax(t, q);
    case OCM_TYPE_ALT: return sqrt(t * t + q * q);
    default: return t + q;  // ci, dd
  }
}

}  // namespace ocm

#define OCM_HIP(call)                                                                       \
  do {                                                                                      \
    hipError_t e_ = (call);                                                                 \
    if (e_ != hipSuccess)                                                                   \
      return ocm::fail(OCM_ERR_HIP, std::string(#call) + ": " + hipGetErrorString(e_));   \
  } while (0)

#define OCM_CHECK_LAUNCH(name)                                                              \
  do {                                                                                      \
    hipError_t e_ = hipGetLastError();                                                      \
    if (e_ != hipSuccess)                                                                   \
      return ocm::fail(OCM_ERR_HIP, std::string("launch ") + name + ": " + hipGetErrorString(e_)); \
  } while (0)

#define OCM_REQUIRE(cond, msg)                                  \
  do {                                                          \
    if (!(cond)) return ocm::fail(OCM_ERR_ARG, (msg));          \
  } while (0)

// ---- device helpers -------------------------------------------------------

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ double wave_sum_f64(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_sum_f32(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---- last-workgroup reductions without fences -----------------------------
// A grid's partial results meet in its last workgroup to finish.  MI355X's
// eight XCDs keep private L2s and a CU's L1 is never refreshed by other CUs'
// stores, so the hand-off is write-through (MI355X_MICROARCH.md, inter-
// workgroup visibility, valid forms, table row 1): every partial is stored
// sc1 (an agent-scope relaxed atomic store), each storing wave drains its
// stores (s_waitcnt vmcnt(0)) and then ONE lane per workgroup adds to an
// agent-scope counter; the workgroup whose add returns n − 1 is last and
// reads the partials with sc1 loads (which bypass its L1).  No
// __threadfence(): its L2 write-back + L1 invalidate cost ≈ 3.5 µs per
// workgroup (round 4: a 512-workgroup batch-norm reduction went 6 → 46 µs).
__device__ __forceinline__ void st_agent(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_agent(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_agent(const double* p) {
  return __hip_atomic_load(const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_agent(const float* p) {
  return __hip_atomic_load(const_cast<float*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// Σ_k p[k·stride] over k = lane, lane + 64, … < count in that order (one lane
// of a wave-strided sum), eight write-through loads in flight at a time (a
// runtime loop of atomic loads waits out each one: ≈ 1 µs apiece)
template <typename T, typename A>
__device__ __forceinline__ A lane_sum_agent(const T* p, int64_t stride, int count, int lane) {
  A acc = A(0);
  for (int k0 = lane; k0 < count; k0 += 64 * 8) {
    T v[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int k = k0 + 64 * r;
      const T x = ld_agent(p + (int64_t)(k < count ? k : lane) * stride);
      v[r] = k < count ? x : T(0);
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) acc += (A)v[r];
  }
  return acc;
}
// Called by every thread of the workgroup after its st_agent stores: true in
// the last of the n workgroups that share `*counter`, which it resets to 0 (so
// a counter zeroed once stays reusable across launches and graph replays).
__device__ __forceinline__ bool last_arrival(unsigned* counter, unsigned n) {
  __shared__ bool last_;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have left
  __syncthreads();                                   // ... and every other wave's
  if (threadIdx.x == 0) {
    const unsigned old = __hip_atomic_fetch_add(counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last_ = old == n - 1;
    if (last_) __hip_atomic_store(counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  __syncthreads();
  return last_;
}
// Two-level form for wide grids: n arrivals at one counter queue up at the
// memory-side atomic unit (≈ 50 ns apart: 256 workgroups of one batch-norm
// channel took ≈ 13 µs to count), so workgroup `idx` of the n counts in
// sub-counter idx / 16 and the last of each sixteen counts in the main
// counter: ≤ 16 + ⌈n/16⌉ adds in a row.  Counters of `slot` start at word
// slot · tickets_per_slot(n) · TICKET_STRIDE, one per 128-B line.
constexpr int TICKET_STRIDE = 32;
__host__ __device__ constexpr int tickets_per_slot(int n) { return 1 + (n + 15) / 16; }
__device__ __forceinline__ bool last_arrival2(unsigned* tickets, int slot, unsigned n, unsigned idx) {
  __shared__ bool last_;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's partial stores have left
  __syncthreads();                                   // ... and every other wave's
  if (threadIdx.x == 0) {
    const unsigned nsub = (n + 15) / 16, g = idx / 16;
    const unsigned gsize = n - 16 * g < 16u ? n - 16 * g : 16u;
    unsigned* base = tickets + (size_t)slot * tickets_per_slot((int)n) * TICKET_STRIDE;
    unsigned* sub = base + (1 + g) * TICKET_STRIDE;
    bool l = false;
    if (__hip_atomic_fetch_add(sub, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gsize - 1) {
      __hip_atomic_store(sub, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      if (__hip_atomic_fetch_add(base, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == nsub - 1) {
        __hip_atomic_store(base, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        l = true;
      }
    }
    last_ = l;
  }
  __syncthreads();
  return last_;
}

// ---- preprocessing in the load path (include/ocm.h ocm_prep) --------------
// Kernel-side copy of an ocm_prep (by value), plus the one scalar definition
// of the transform every fused kernel reproduces bit for bit.
struct PrepArgs {
  int w = 0;      // window (0: SNV only)
  int h = 0;      // w / 2
  int deriv = 0;  // 0, odd, even >= 2 select the interior form
  int snv = 0;
  const float* taps = nullptr;     // [w] interior ++ [h][w] left ++ [h][w] right
  const float* rowstat = nullptr;  // (m_r, s_r) per row of X
  // the forms the fused load paths implement (k_score_1p, the i8×3 quantiser):
  // SNV alone, or an odd-derivative filter (every reference driver: deriv 1)
  // of half-width 2 or 7, SNV optional; the rest is materialised first
  bool fused_form() const { return w == 0 ? snv != 0 : (h == 2 || h == 7) && (deriv & 1); }
};

namespace ocm {

// PrepArgs from a host ocm_prep (validated by the caller)
inline PrepArgs prep_args(const ocm_prep* p) {
  PrepArgs a;
  a.w = p->window;
  a.h = p->window / 2;
  a.deriv = p->window > 0 ? p->deriv : 0;
  a.snv = p->snv;
  a.taps = p->taps;
  a.rowstat = p->rowstat;
  return a;
}

int check_prep(const ocm_prep* prep, int p, const char* who);
// Σ_ij O_ij (XᵀX)_ij for the rows X of a symmetric p×p float32 O (p > 64): the
// i8×3 Gram without G, as ntr fp64 partials in tr_part (ntr ≤ 16·(p/128+1)²/2;
// sum them in order); zero shift, no outlier screen.  Uses the context
// workspace from offset 0 (callers must not hold workspace carve-outs across it).
int trace_gram_rows_i8(ocm_ctx* ctx, const float* X, int64_t ldx, int64_t n, int p, const float* O, double* tr_part,
                       int* ntr, hipStream_t st);
int prep_apply(ocm_ctx* ctx, const float* X, int64_t ldx, const int64_t* rows, int64_t m, int p, const PrepArgs& pa,
               float* out, int64_t ldo, hipStream_t st);

// a·b rounded to float32 and never fused into a consumer's add (HIP compiles
// with -ffp-contract=fast-honor-pragmas: a product written as a * b, or
// __fmul_rn, may become an FMA with the caller's y − shift; this one carries
// no contract flag).  Every kernel that forms a lazy view's values uses it, so
// they all round the same way.
__device__ __forceinline__ float mul_nc(float a, float b) {
#pragma clang fp contract(off)
  return a * b;
}

// y_j of row `xr` (raw X row): the formula of include/ocm.h, scalar loads.
// m, s: the row's (m_r, s_r) (ignored unless snv).
__device__ __forceinline__ float prep_elem(const float* __restrict__ xr, int p, int j, const PrepArgs& pa, float m,
                                           float s) {
  const bool sub = pa.snv && pa.deriv == 0;
  auto u = [&](int c) { return sub ? __fsub_rn(xr[c], m) : xr[c]; };
  const int H = pa.h;
  float a;
  if (pa.w == 0) {
    a = u(j);
  } else if (j < H || j >= p - H) {
    const bool left = j < H;
    const float* e = pa.taps + pa.w + (left ? j : H + j - (p - H)) * pa.w;
    const int s0 = left ? 0 : p - pa.w;
    const float ref = pa.deriv >= 1 ? u(j) : 0.f;
    a = 0.f;
    for (int t = 0; t < pa.w; ++t) a = fmaf(e[t], __fsub_rn(u(s0 + t), ref), a);
  } else {
    const float* c = pa.taps + H;  // c[t] = tap at offset t, t in [-H, H]
    if (pa.deriv & 1) {
      a = 0.f;
      for (int t = 1; t <= H; ++t) a = fmaf(c[t], __fsub_rn(u(j + t), u(j - t)), a);
    } else if (pa.deriv == 0) {
      a = mul_nc(c[0], u(j));
      for (int t = 1; t <= H; ++t) a = fmaf(c[t], __fadd_rn(u(j + t), u(j - t)), a);
    } else {
      const float uj = u(j);
      a = 0.f;
      for (int t = 1; t <= H; ++t) a = fmaf(c[t], __fadd_rn(__fsub_rn(u(j + t), uj), __fsub_rn(u(j - t), uj)), a);
    }
  }
  return pa.snv ? mul_nc(a, s) : a;
}

}  // namespace ocm
