// Context, error reporting and workspace for libocm.
//
// One context per (device, stream): the workspace is reused by every call
// issued on that stream, so calls on one context are stream-ordered.
#include "ocm_internal.h"

namespace {
thread_local std::string g_last_error;
}

namespace ocm {

void set_error(const std::string& msg) { g_last_error = msg; }

int fail(int code, const std::string& msg) {
  g_last_error = msg;
  return code;
}

static void* grow(void*& buf, size_t& have, size_t bytes, hipStream_t stream) {
  bytes = align_up(bytes, 1 << 20);
  if (bytes <= have) return buf;
  if (buf) {
    // Work queued on this stream may still read the old buffer.
    (void)hipStreamSynchronize(stream);
    (void)hipFree(buf);
    buf = nullptr;
    have = 0;
  }
  void* p = nullptr;
  if (hipMalloc(&p, bytes) != hipSuccess) {
    set_error("workspace hipMalloc failed (" + std::to_string(bytes) + " bytes)");
    return nullptr;
  }
  buf = p;
  have = bytes;
  return p;
}

void* workspace(ocm_ctx* ctx, size_t bytes, hipStream_t stream) { return grow(ctx->ws, ctx->ws_bytes, bytes, stream); }

void* workspace_aux(ocm_ctx* ctx, size_t bytes, hipStream_t stream) {
  return grow(ctx->ws_aux, ctx->ws_aux_bytes, bytes, stream);
}

void* host_staging(ocm_ctx* ctx, size_t bytes) {
  if (bytes <= ctx->host_bytes) return ctx->host_pinned;
  if (ctx->host_pinned) (void)hipHostFree(ctx->host_pinned);
  ctx->host_pinned = nullptr;
  ctx->host_bytes = 0;
  bytes = align_up(bytes, 4096);
  if (hipHostMalloc(&ctx->host_pinned, bytes, hipHostMallocDefault) != hipSuccess) {
    set_error("hipHostMalloc failed");
    return nullptr;
  }
  ctx->host_bytes = bytes;
  return ctx->host_pinned;
}

}  // namespace ocm

extern "C" {

int ocm_abi_version(void) { return OCM_ABI_VERSION; }

const char* ocm_last_error(void) { return g_last_error.c_str(); }

int ocm_ctx_create(int device, ocm_ctx** out) {
  OCM_REQUIRE(out != nullptr, "ocm_ctx_create: out is NULL");
  int ndev = 0;
  OCM_HIP(hipGetDeviceCount(&ndev));
  OCM_REQUIRE(device >= 0 && device < ndev, "ocm_ctx_create: bad device index");
  OCM_HIP(hipSetDevice(device));
  hipDeviceProp_t prop;
  OCM_HIP(hipGetDeviceProperties(&prop, device));
  std::string arch(prop.gcnArchName);
  if (arch.rfind("gfx950", 0) != 0)
    return ocm::fail(OCM_ERR_UNSUPPORTED, "libocm is built for gfx950 (MI355X); device is " + arch);
  auto* c = new ocm_ctx();
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  *out = c;
  return OCM_OK;
}

int ocm_ctx_destroy(ocm_ctx* ctx) {
  if (!ctx) return OCM_OK;
  if (ctx->ws) (void)hipFree(ctx->ws);
  if (ctx->ws_aux) (void)hipFree(ctx->ws_aux);
  if (ctx->host_pinned) (void)hipHostFree(ctx->host_pinned);
  if (ctx->side) (void)hipStreamDestroy(ctx->side);
  for (auto e : ctx->fork_ev) (void)hipEventDestroy(e);
  for (auto s : ctx->eig_side)
    if (s) (void)hipStreamSynchronize(s);
  if (ctx->eig_sub) (void)ocm_ctx_destroy(ctx->eig_sub);
  for (auto s : ctx->eig_side)
    if (s) (void)hipStreamDestroy(s);
  for (auto e : ctx->eig_ev)
    if (e) (void)hipEventDestroy(e);
  if (ctx->eig_flag) (void)hipFree(ctx->eig_flag);
  for (auto& v : ctx->ev)
    for (auto& pr : v) ctx->ev_pool.push_back(pr);
  for (auto& pr : ctx->ev_pool) {
    (void)hipEventDestroy(pr.first);
    (void)hipEventDestroy(pr.second);
  }
  delete ctx;
  return OCM_OK;
}

int ocm_ctx_set_timing(ocm_ctx* ctx, int enable) {
  OCM_REQUIRE(ctx != nullptr, "ocm_ctx_set_timing: NULL ctx");
  ctx->timing = enable != 0;
  return OCM_OK;
}

int ocm_ctx_read_timing(ocm_ctx* ctx, int kernel_id, double* total_ms, int64_t* count) {
  OCM_REQUIRE(ctx && total_ms && count, "ocm_ctx_read_timing: NULL argument");
  OCM_REQUIRE(kernel_id >= 0 && kernel_id < OCM_TIMED_KERNELS, "ocm_ctx_read_timing: bad kernel id");
  double tot = 0.0;
  for (auto& pr : ctx->ev[kernel_id]) {
    OCM_HIP(hipEventSynchronize(pr.second));
    float ms = 0.f;
    OCM_HIP(hipEventElapsedTime(&ms, pr.first, pr.second));
    tot += ms;
    ctx->ev_pool.push_back(pr);
  }
  *count = (int64_t)ctx->ev[kernel_id].size();
  *total_ms = tot;
  ctx->ev[kernel_id].clear();
  return OCM_OK;
}

int ocm_ctx_reserve(ocm_ctx* ctx, size_t bytes) {
  OCM_REQUIRE(ctx != nullptr, "ocm_ctx_reserve: NULL ctx");
  if (!ocm::workspace(ctx, bytes, nullptr)) return OCM_ERR_NOMEM;
  return OCM_OK;
}

}  // extern "C"
