// Streaming-read microbenchmark for the scoring kernel's access pattern
// (1M × 2048 f32 = 8.19 GB).  Each variant only sums what it loads.
//   tile16: persistent workgroups of 8 waves; a wave reads its 1-KiB slice of
//           16 consecutive rows as 16 instructions of 16 rows × 64 B (lane
//           row = l & 15, 16 B at 16·(l >> 4)) — the k_score_1p pattern;
//   rowcont: the same bytes, each instruction one contiguous 1-KiB row piece.
// Prints GB/s per variant (hipEvent timing, median of 5).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int P = 2048, W = 8, R = 16, NJ = 16;

template <int MODE>
__global__ __launch_bounds__(512, 1) void k_read(const float* __restrict__ X, int64_t n, float* __restrict__ out) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int ln = lane & 15, lq = lane >> 4;
  const int64_t ntiles = n / R;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int64_t t = blockIdx.x; t < ntiles; t += gridDim.x) {
    f32x4 v[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) {
      const float* p;
      if (MODE == 0) p = X + (t * R + ln) * P + w * (P / W) + 16 * j + 4 * lq;
      else p = X + (t * R + j) * P + w * (P / W) + 4 * lane;  // row j of the tile, 1 KiB contiguous
      v[j] = *reinterpret_cast<const f32x4*>(p);
    }
#pragma unroll
    for (int j = 0; j < NJ; ++j) acc += v[j];
  }
  if (acc[0] + acc[1] + acc[2] + acc[3] == 12345.f) out[threadIdx.x] = acc[0];
}

int main() {
  const int64_t n = 1000000;
  float* X;
  float* out;
  if (hipMalloc(&X, n * P * sizeof(float)) != hipSuccess) return 1;
  (void)hipMalloc(&out, 4096);
  (void)hipMemset(X, 0, n * P * sizeof(float));
  int cus = 256;
  hipDeviceProp_t pr;
  if (hipGetDeviceProperties(&pr, 0) == hipSuccess) cus = pr.multiProcessorCount;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int mode = 0; mode < 2; ++mode) {
    for (int mult : {1, 2}) {
      std::vector<float> ms;
      for (int rep = 0; rep < 6; ++rep) {
        (void)hipEventRecord(a);
        if (mode == 0) hipLaunchKernelGGL(k_read<0>, dim3(cus * mult), dim3(512), 0, 0, X, n, out);
        else hipLaunchKernelGGL(k_read<1>, dim3(cus * mult), dim3(512), 0, 0, X, n, out);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float t = 0.f;
        (void)hipEventElapsedTime(&t, a, b);
        if (rep) ms.push_back(t);
      }
      std::sort(ms.begin(), ms.end());
      const double m = ms[ms.size() / 2];
      printf("{\"mode\": \"%s\", \"grid\": %d, \"ms\": %.4f, \"GBs\": %.1f}\n", mode ? "rowcont" : "tile16", cus * mult, m,
             n * P * 4.0 / m / 1e6);
    }
  }
  return 0;
}
