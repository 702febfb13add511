// Micro-benchmark: issue rate of the MFMA / VALU forms the SIMCA kernels can
// use on gfx950 (one wave per SIMD, 4 independent accumulators, operands in
// registers).  Build+run on the GPU box:
//   hipcc --offload-arch=gfx950 -O3 scripts/ubench_mfma.hip -o /tmp/ub && /tmp/ub
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

constexpr int ITERS = 4096;

__global__ __launch_bounds__(256) void k_f32_32x32x2(float* out, float a, float b) {
  f32x16 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  float x = a + threadIdx.x, y = b - threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    c0 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, y, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, x, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f32_32x32x2f32(x, x, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f32_32x32x2f32(y, y, c3, 0, 0, 0);
  }
  float s = 0;
  for (int r = 0; r < 16; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_f64_16x16x4(double* out, double a, double b) {
  f64x4 c0 = {}, c1 = {}, c2 = {}, c3 = {};
  double x = a + threadIdx.x, y = b - threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
    c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, y, c0, 0, 0, 0);
    c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, x, c1, 0, 0, 0);
    c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(x, x, c2, 0, 0, 0);
    c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(y, y, c3, 0, 0, 0);
  }
  double s = 0;
  for (int r = 0; r < 4; ++r) s += c0[r] + c1[r] + c2[r] + c3[r];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

__global__ __launch_bounds__(256) void k_f64_valu(double* out, double a, double b) {
  double c[8];
  for (int j = 0; j < 8; ++j) c[j] = a + j + threadIdx.x;
  for (int i = 0; i < ITERS; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) c[j] = fma(c[j], b, a);
  }
  double s = 0;
  for (int j = 0; j < 8; ++j) s += c[j];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <typename F>
double time_it(F f, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < reps; ++r) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const int blocks = 256 * 4;  // 4 blocks of 4 waves per CU -> 4 waves/SIMD
  float* of;
  double* od;
  hipMalloc(&of, blocks * 256 * sizeof(float));
  hipMalloc(&od, blocks * 256 * sizeof(double));
  for (int wps : {1, 2, 4}) {
    const int nb = 256 * wps;
    double ms = time_it([&] { hipLaunchKernelGGL(k_f32_32x32x2, dim3(nb), dim3(256), 0, 0, of, 1.f, 2.f); }, 5);
    double fl = (double)nb * 4 * ITERS * 4 * (32.0 * 32 * 2 * 2);
    printf("f32 32x32x2 waves/SIMD=%d  %.1f TFLOP/s\n", wps, fl / ms / 1e9);
    ms = time_it([&] { hipLaunchKernelGGL(k_f64_16x16x4, dim3(nb), dim3(256), 0, 0, od, 1.0, 2.0); }, 5);
    fl = (double)nb * 4 * ITERS * 4 * (16.0 * 16 * 4 * 2);
    printf("f64 16x16x4 waves/SIMD=%d  %.1f TFLOP/s\n", wps, fl / ms / 1e9);
    ms = time_it([&] { hipLaunchKernelGGL(k_f64_valu, dim3(nb), dim3(256), 0, 0, od, 1.0, 0.999); }, 5);
    fl = (double)nb * 256 * ITERS * 8 * 2;
    printf("f64 VALU fma waves/SIMD=%d  %.1f TFLOP/s\n", wps, fl / ms / 1e9);
  }
  return 0;
}
