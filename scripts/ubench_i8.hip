// Micro-benchmark: sustained rate of the k_gram8 MFMA pattern (int8
// 32x32x32, 3 accumulator sets × 4 blocks, operands in registers), one wave
// per SIMD, every CU busy.  hipcc --offload-arch=gfx950 -O3 scripts/ubench_i8.hip -o /tmp/ubi8 && /tmp/ubi8
#include <hip/hip_runtime.h>

#include <cstdio>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
constexpr int ITERS = 2048;

__global__ __launch_bounds__(256, 1) void k_i8(int* out, int seed) {
  i32x4 fa[2][3], fb[2][3];
  for (int a = 0; a < 2; ++a)
    for (int d = 0; d < 3; ++d) {
      fa[a][d] = i32x4{seed + a + d + (int)threadIdx.x, 1, 2, 3};
      fb[a][d] = i32x4{seed - a - d, 3, (int)threadIdx.x, 1};
    }
  i32x16 acc1[2][2] = {}, acc2[2][2] = {}, acc3[2][2] = {};
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        acc1[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a][0], fb[c][0], acc1[a][c], 0, 0, 0);
        acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a][0], fb[c][1], acc2[a][c], 0, 0, 0);
        acc2[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a][1], fb[c][0], acc2[a][c], 0, 0, 0);
        acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a][0], fb[c][2], acc3[a][c], 0, 0, 0);
        acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a][2], fb[c][0], acc3[a][c], 0, 0, 0);
        acc3[a][c] = __builtin_amdgcn_mfma_i32_32x32x32_i8(fa[a][1], fb[c][1], acc3[a][c], 0, 0, 0);
      }
  }
  int s = 0;
  for (int a = 0; a < 2; ++a)
    for (int c = 0; c < 2; ++c)
      for (int r = 0; r < 16; ++r) s += acc1[a][c][r] + acc2[a][c][r] + acc3[a][c][r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
  int* out;
  hipMalloc(&out, 4096 * 256 * sizeof(int));
  const int grid = 256 * 8;
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int rep = 0; rep < 3; ++rep) {
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_i8, dim3(grid), dim3(256), 0, 0, out, rep);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    const double ops = (double)grid * 4 * ITERS * 24 * (32.0 * 32 * 32 * 2);
    printf("i8 pattern: %.3f ms  %.1f TOPS  (%.1f%% of 5000)\n", ms, ops / ms / 1e9, ops / ms / 1e9 / 50.0);
  }
  return 0;
}
