// Microtest 2: internal precision of the 16-product sum of
// v_mfma_f32_32x32x16_bf16 (lane 0 / lane 32 carry the k-octets of row 0 and
// column 0).  Each case: acc0 plus products p[0..15]; prints the result next
// to the correctly rounded (RNE) exact sum.
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct Case {
  const char* name;
  float acc0;
  float a[16], b[16];
};

__global__ void k(const Case* c, float* out) {
  const int lane = threadIdx.x;
  bf16x8 a, b;
  for (int j = 0; j < 8; ++j) {
    const int kk = (lane >> 5) * 8 + j;
    const bool row0 = (lane & 31) == 0;
    a[j] = (__bf16)(row0 ? c->a[kk] : 0.f);
    b[j] = (__bf16)(row0 ? c->b[kk] : 0.f);
  }
  f32x16 acc;
  for (int r = 0; r < 16; ++r) acc[r] = c->acc0;
  acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
  if (lane == 0) out[0] = acc[0];
}

int main() {
  Case cs[5] = {};
  const float u = ldexpf(1.f, -24);
  cs[0].name = "sticky: 0 + 1 + 2^-24 + 2^-40";
  cs[0].a[0] = 1.f; cs[0].b[0] = 1.f; cs[0].a[1] = ldexpf(1.f, -12); cs[0].b[1] = ldexpf(1.f, -12);
  cs[0].a[2] = ldexpf(1.f, -20); cs[0].b[2] = ldexpf(1.f, -20);
  cs[1].name = "sticky: 1 + 2^-24 + 2^-40"; cs[1].acc0 = 1.f;
  cs[1].a[0] = ldexpf(1.f, -12); cs[1].b[0] = ldexpf(1.f, -12); cs[1].a[1] = ldexpf(1.f, -20); cs[1].b[1] = ldexpf(1.f, -20);
  cs[2].name = "cancel: 0 + 1 - 1 + 2^-30";
  cs[2].a[0] = 1.f; cs[2].b[0] = 1.f; cs[2].a[1] = -1.f; cs[2].b[1] = 1.f; cs[2].a[2] = ldexpf(1.f, -15); cs[2].b[2] = ldexpf(1.f, -15);
  cs[3].name = "16 sub-ulp: 1 + 16*2^-25"; cs[3].acc0 = 1.f;
  for (int i = 0; i < 16; ++i) { cs[3].a[i] = ldexpf(1.f, -13); cs[3].b[i] = ldexpf(1.f, -12); }
  cs[4].name = "mixed: 1 + 2^-8 - 2^-8 + 3*2^-26"; cs[4].acc0 = 1.f;
  cs[4].a[0] = ldexpf(1.f, -4); cs[4].b[0] = ldexpf(1.f, -4); cs[4].a[1] = -ldexpf(1.f, -4); cs[4].b[1] = ldexpf(1.f, -4);
  for (int i = 2; i < 5; ++i) { cs[4].a[i] = ldexpf(1.f, -13); cs[4].b[i] = ldexpf(1.f, -13); }
  Case* d;
  float* o;
  (void)hipMalloc(&d, sizeof(Case));
  (void)hipMalloc(&o, 4);
  for (int i = 0; i < 5; ++i) {
    (void)hipMemcpy(d, &cs[i], sizeof(Case), hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o);
    float h;
    (void)hipMemcpy(&h, o, 4, hipMemcpyDeviceToHost);
    double ex = cs[i].acc0;
    for (int j = 0; j < 16; ++j) ex += (double)cs[i].a[j] * cs[i].b[j];
    printf("%-36s got %.10e  exact %.10e  RNE(exact) %.10e  (got-RNE)/ulp(1) %.2f\n", cs[i].name, h, ex,
           (double)(float)ex, (h - (float)ex) / (2 * u));
  }
  return 0;
}
