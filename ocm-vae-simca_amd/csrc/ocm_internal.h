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
  void* host_pinned = nullptr;  // small pinned staging area for D2H scalars
  size_t host_bytes = 0;
  int num_cus = 256;
  uint32_t last_gram_marks = 0;  // outlier-guard marks of the last i8×3 Gram (ocm_gram_last_marks)
  // live kernel timing (ocm_ctx_set_timing): event pairs per timed kernel
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev[OCM_TIMED_KERNELS];
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pool;
  // side stream + events of the quantiser / Gram overlap (created on first use)
  hipStream_t side = nullptr;
  std::vector<hipEvent_t> fork_ev;
};

namespace ocm {

// Record a start/stop event pair around a launch when timing is enabled.
struct TimedRegion {
  ocm_ctx* ctx;
  int id;
  hipStream_t st;
  std::pair<hipEvent_t, hipEvent_t> pr{nullptr, nullptr};
  TimedRegion(ocm_ctx* c, int i, hipStream_t s) : ctx(c), id(i), st(s) {
    if (!ctx->timing) return;
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
