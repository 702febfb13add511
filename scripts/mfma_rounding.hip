// Microtest: how does an MFMA round when it adds its products into the
// accumulator?  acc starts at 1.0; each MFMA adds exactly one product equal to
// 0.75 ulp(1.0) = 0.75·2^-23.  Round-to-nearest-even grows acc by 1 ulp per
// MFMA, truncation leaves it at 1.0.  Also: two products of 0.375 ulp each
// (sum exact inside the MFMA?), and the FP32-input MFMA for comparison.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(float* out, int reps, int mode) {
  const int lane = threadIdx.x;
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = 1.0f;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) { a[j] = (__bf16)0.0f; b[j] = (__bf16)0.0f; }
  const float tiny = 0.75f * 1.1920928955078125e-07f;  // 0.75 * 2^-23 (exact in bf16: 1.5 * 2^-24)
  if (mode == 0) {          // one product per MFMA into row 0 / col 0 (lane 0 holds A[0][0..7], B[0..7][0])
    if (lane == 0) { a[0] = (__bf16)tiny; b[0] = (__bf16)1.0f; }
  } else if (mode == 1) {   // two products of 0.375 ulp each (k = 0, 1)
    if (lane == 0) { a[0] = (__bf16)(tiny * 0.5f); b[0] = (__bf16)1.0f; a[1] = (__bf16)(tiny * 0.5f); b[1] = (__bf16)1.0f; }
  }
  if (mode <= 1) {
    for (int i = 0; i < reps; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  } else {                  // FP32-input MFMA, one product of 0.75 ulp
    float af = lane == 0 ? tiny : 0.f, bf = lane == 0 ? 1.0f : 0.f;
    for (int i = 0; i < reps; ++i) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(af, bf, acc, 0, 0, 0);
  }
  if (lane == 0) out[0] = acc[0];  // row 0, col 0
}

int main() {
  float* d;
  hipMalloc(&d, 4);
  const int reps = 1000;
  const char* names[3] = {"bf16 1 product 0.75ulp", "bf16 2 products 0.375ulp", "f32 1 product 0.75ulp"};
  for (int mode = 0; mode < 3; ++mode) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, reps, mode);
    float h;
    hipMemcpy(&h, d, 4, hipMemcpyDeviceToHost);
    printf("%-26s after %d MFMAs: acc - 1 = %.3f ulp (RNE: %d, truncation: 0)\n", names[mode], reps,
           (h - 1.0f) / 1.1920928955078125e-07f, mode == 1 ? 0 : reps);
  }
  return 0;
}
