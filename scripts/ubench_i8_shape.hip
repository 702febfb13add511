// Micro-benchmark: int8 MFMA shape on RANDOM register operands (the clock the
// chip holds depends on operand toggling): 32x32x32 vs 16x16x64, same 64x64
// output tile per wave, 3 accumulator sets, 64 K-rows per iteration, one wave
// per SIMD, every CU busy.
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_i8_shape.hip -o /tmp/ubs && /tmp/ubs
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
constexpr int ITERS = 4096;

__global__ __launch_bounds__(256, 1) void k32(const i32x4* __restrict__ src, int* out) {
  i32x4 F[2][2][2][3];  // [stage][A|B][block][digit]
  const int t = threadIdx.x;
  for (int s = 0; s < 2; ++s)
    for (int o = 0; o < 2; ++o)
      for (int x = 0; x < 2; ++x)
        for (int d = 0; d < 3; ++d) F[s][o][x][d] = src[((((s * 2 + o) * 2 + x) * 3 + d) * 256 + t)];
  i32x16 acc1[2][2] = {}, acc2[2][2] = {}, acc3[2][2] = {};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int c = 0; c < 2; ++c) {
          const i32x4* A = F[s][0][a];
          const i32x4* B = F[s][1][c];
          acc1[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[0], B[0], acc1[a][c], 0, 0, 0);
          acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[0], B[1], acc2[a][c], 0, 0, 0);
          acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[1], B[0], acc2[a][c], 0, 0, 0);
          acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[0], B[2], acc3[a][c], 0, 0, 0);
          acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[2], B[0], acc3[a][c], 0, 0, 0);
          acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(A[1], B[1], acc3[a][c], 0, 0, 0);
        }
  }
  int s = 0;
  for (int a = 0; a < 2; ++a)
    for (int c = 0; c < 2; ++c)
      for (int r = 0; r < 16; ++r) s += acc1[a][c][r] + acc2[a][c][r] + acc3[a][c][r];
  out[blockIdx.x * 256 + t] = s;
}

__global__ __launch_bounds__(256, 1) void k16(const i32x4* __restrict__ src, int* out) {
  i32x4 F[2][4][3];  // [A|B][block of 16][digit], 64 K-rows
  const int t = threadIdx.x;
  for (int o = 0; o < 2; ++o)
    for (int x = 0; x < 4; ++x)
      for (int d = 0; d < 3; ++d) F[o][x][d] = src[(((o * 4 + x) * 3 + d) * 256 + t)];
  i32x4 acc1[4][4] = {}, acc2[4][4] = {}, acc3[4][4] = {};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const i32x4* A = F[0][a];
        const i32x4* B = F[1][c];
        acc1[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[0], acc1[a][c], 0, 0, 0);
        acc2[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[1], acc2[a][c], 0, 0, 0);
        acc2[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B[0], acc2[a][c], 0, 0, 0);
        acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[0], B[2], acc3[a][c], 0, 0, 0);
        acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[2], B[0], acc3[a][c], 0, 0, 0);
        acc3[a][c] = __builtin_amdgcn_mfma_i32_16x16x64_i8(A[1], B[1], acc3[a][c], 0, 0, 0);
      }
  }
  int s = 0;
  for (int a = 0; a < 4; ++a)
    for (int c = 0; c < 4; ++c)
      for (int r = 0; r < 4; ++r) s += acc1[a][c][r] + acc2[a][c][r] + acc3[a][c][r];
  out[blockIdx.x * 256 + t] = s;
}

int main() {
  const int n = 64 * 256;
  std::vector<int> h(n * 4);
  unsigned x = 12345;
  for (auto& v : h) {
    x = x * 1664525u + 1013904223u;
    v = (int)x;
  }
  i32x4* src;
  int* out;
  hipMalloc(&src, n * sizeof(i32x4));
  hipMemcpy(src, h.data(), n * sizeof(i32x4), hipMemcpyHostToDevice);
  hipMalloc(&out, 4096 * 256 * sizeof(int));
  const int grid = 256 * 4;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const double ops = (double)grid * 4 * ITERS * 96 * (32.0 * 32 * 32);  // 48 MFMA 32x32x32 × 2 = 96 × 32768 ... per wave-iter
  for (int rep = 0; rep < 6; ++rep) {
    for (int v = 0; v < 2; ++v) {
      hipEventRecord(e0);
      if (v == 0)
        hipLaunchKernelGGL(k32, dim3(grid), dim3(256), 0, 0, src, out);
      else
        hipLaunchKernelGGL(k16, dim3(grid), dim3(256), 0, 0, src, out);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      // per wave-iteration: 48 MFMA 32x32x32 (2·32768 ops each) = 96 MFMA 16x16x64 (2·16384 ops each)
      const double o = (double)grid * 4 * ITERS * 48 * (2.0 * 32 * 32 * 32);
      printf("%s random operands: %.3f ms  %.1f TOPS (%.1f%% of 5000)\n", v ? "16x16x64" : "32x32x32", ms,
             o / ms / 1e9, o / ms / 1e9 / 50.0);
    }
  }
  (void)ops;
  return 0;
}
