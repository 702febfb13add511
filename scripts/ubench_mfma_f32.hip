// v_mfma_f32_16x16x4_f32 throughput, one wave per SIMD: accumulators in
// AGPRs vs VGPRs, 2 or 4 interleaved chains.  Prints cycles per MFMA per SIMD
// (s_memtime around the loop, wave 0 of each workgroup).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 2000;

template <int MODE>  // 0: AGPR acc 4 chains, 1: VGPR acc 4 chains, 2: VGPR acc 2 chains, 3: AGPR 2 chains,
                    // 4: VGPR 4 chains + 4 accvgpr_read + 4 DPP adds in the gaps (sweep-1 shape),
                    // 5: as 4, srcB = the DPP results of the previous iteration
__global__ __launch_bounds__(256, 1) void k(float a, float b, float* out, unsigned long long* cyc) {
  f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  f32x4 xa = {a, b, a, b};
  float n0 = a, n1 = b, n2 = a, n3 = b;
  asm volatile("v_accvgpr_write_b32 %0, %4\n\tv_accvgpr_write_b32 %1, %4\n\tv_accvgpr_write_b32 %2, %4\n\t"
               "v_accvgpr_write_b32 %3, %4" : "=a"(xa[0]), "=a"(xa[1]), "=a"(xa[2]), "=a"(xa[3]) : "v"(b));
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (MODE == 0) {
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %4, %5, %0\n\tv_mfma_f32_16x16x4_f32 %1, %4, %5, %1\n\t"
                   "v_mfma_f32_16x16x4_f32 %2, %4, %5, %2\n\tv_mfma_f32_16x16x4_f32 %3, %4, %5, %3"
                   : "+a"(c0), "+a"(c1), "+a"(c2), "+a"(c3) : "v"(a), "v"(b));
    } else if constexpr (MODE == 1) {
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %4, %5, %0\n\tv_mfma_f32_16x16x4_f32 %1, %4, %5, %1\n\t"
                   "v_mfma_f32_16x16x4_f32 %2, %4, %5, %2\n\tv_mfma_f32_16x16x4_f32 %3, %4, %5, %3"
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3) : "v"(a), "v"(b));
    } else if constexpr (MODE == 2) {
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %2, %3, %0\n\tv_mfma_f32_16x16x4_f32 %1, %2, %3, %1\n\t"
                   "v_mfma_f32_16x16x4_f32 %0, %2, %3, %0\n\tv_mfma_f32_16x16x4_f32 %1, %2, %3, %1"
                   : "+v"(c0), "+v"(c1) : "v"(a), "v"(b));
    } else if constexpr (MODE == 3) {
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %2, %3, %0\n\tv_mfma_f32_16x16x4_f32 %1, %2, %3, %1\n\t"
                   "v_mfma_f32_16x16x4_f32 %0, %2, %3, %0\n\tv_mfma_f32_16x16x4_f32 %1, %2, %3, %1"
                   : "+a"(c0), "+a"(c1) : "v"(a), "v"(b));
    } else if constexpr (MODE == 5) {  // reads only
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %8, %4, %0\n\t"
                   "v_mfma_f32_16x16x4_f32 %1, %8, %5, %1\n\t"
                   "v_accvgpr_read_b32 %4, %10\n\tv_accvgpr_read_b32 %5, %11\n\t"
                   "v_accvgpr_read_b32 %6, %12\n\tv_accvgpr_read_b32 %7, %13\n\t"
                   "v_mfma_f32_16x16x4_f32 %2, %8, %6, %2\n\t"
                   "v_mfma_f32_16x16x4_f32 %3, %8, %7, %3"
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3)
                   : "v"(a), "v"(b), "a"(xa[0]), "a"(xa[1]), "a"(xa[2]), "a"(xa[3]));
    } else if constexpr (MODE == 6) {  // DPP adds only
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %8, %4, %0\n\t"
                   "v_mfma_f32_16x16x4_f32 %1, %8, %5, %1\n\t"
                   "v_mfma_f32_16x16x4_f32 %2, %8, %6, %2\n\t"
                   "v_add_f32_dpp %4, %9, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_add_f32_dpp %5, %9, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_add_f32_dpp %6, %9, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_add_f32_dpp %7, %9, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_mfma_f32_16x16x4_f32 %3, %8, %7, %3"
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3)
                   : "v"(a), "v"(b));
    } else if constexpr (MODE == 7) {  // plain adds
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %8, %4, %0\n\t"
                   "v_mfma_f32_16x16x4_f32 %1, %8, %5, %1\n\t"
                   "v_mfma_f32_16x16x4_f32 %2, %8, %6, %2\n\t"
                   "v_add_f32_e32 %4, %9, %4\n\tv_add_f32_e32 %5, %9, %5\n\t"
                   "v_add_f32_e32 %6, %9, %6\n\tv_add_f32_e32 %7, %9, %7\n\t"
                   "v_mfma_f32_16x16x4_f32 %3, %8, %7, %3"
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3)
                   : "v"(a), "v"(b));
    } else if constexpr (MODE == 8) {  // srcB from AGPRs, no VALU
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %4, %5, %0\n\t"
                   "v_mfma_f32_16x16x4_f32 %1, %4, %6, %1\n\t"
                   "v_mfma_f32_16x16x4_f32 %2, %4, %7, %2\n\t"
                   "v_mfma_f32_16x16x4_f32 %3, %4, %8, %3"
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3)
                   : "v"(a), "a"(xa[0]), "a"(xa[1]), "a"(xa[2]), "a"(xa[3]));
    } else if constexpr (MODE == 9) {  // 16 DPP FMAs spread over the 4 gaps
#define F4(L) "v_fmac_f32_dpp %4, %9, %8 row_newbcast:" #L " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
              "v_fmac_f32_dpp %5, %9, %8 row_newbcast:" #L " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
              "v_fmac_f32_dpp %6, %9, %8 row_newbcast:" #L " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t" \
              "v_fmac_f32_dpp %7, %9, %8 row_newbcast:" #L " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
      asm volatile("v_mfma_f32_16x16x4_f32 %0, %8, %9, %0\n\t" F4(1)
                   "v_mfma_f32_16x16x4_f32 %1, %8, %9, %1\n\t" F4(2)
                   "v_mfma_f32_16x16x4_f32 %2, %8, %9, %2\n\t" F4(3)
                   "v_mfma_f32_16x16x4_f32 %3, %8, %9, %3\n\t" F4(4)
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3)
                   : "v"(a), "v"(b));
#undef F4
    } else {
      asm volatile("s_nop 1\n\t"
                   "v_mfma_f32_16x16x4_f32 %0, %8, %4, %0\n\t"
                   "v_mfma_f32_16x16x4_f32 %1, %8, %5, %1\n\t"
                   "v_accvgpr_read_b32 %4, %10\n\tv_accvgpr_read_b32 %5, %11\n\t"
                   "v_accvgpr_read_b32 %6, %12\n\tv_accvgpr_read_b32 %7, %13\n\t"
                   "v_mfma_f32_16x16x4_f32 %2, %8, %6, %2\n\t"
                   "s_nop 1\n\t"
                   "v_add_f32_dpp %4, %9, %4 row_newbcast:1 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_add_f32_dpp %5, %9, %5 row_newbcast:2 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_add_f32_dpp %6, %9, %6 row_newbcast:3 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_add_f32_dpp %7, %9, %7 row_newbcast:4 row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
                   "v_mfma_f32_16x16x4_f32 %3, %8, %7, %3"
                   : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3), "+v"(n0), "+v"(n1), "+v"(n2), "+v"(n3)
                   : "v"(a), "v"(b), "a"(xa[0]), "a"(xa[1]), "a"(xa[2]), "a"(xa[3]));
    }
  }
  asm volatile("s_nop 15" ::: "memory");
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  const f32x4 s = c0 + c1 + c2 + c3 + (n0 + n1 + n2 + n3);
  if (s[0] == 1.2345f) out[threadIdx.x] = s[1];
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 4096);
  (void)hipMalloc(&cyc, 4096 * 8);
  const char* names[] = {"agpr_4chains", "vgpr_4chains", "vgpr_2chains", "agpr_2chains", "sweep1_shape",
                         "reads_only", "dpp_adds_only", "plain_adds", "srcB_agpr", "dpp_fmac16"};
  for (int mode = 0; mode < 10; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (mode) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 3: hipLaunchKernelGGL(k<3>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 4: hipLaunchKernelGGL(k<4>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 5: hipLaunchKernelGGL(k<5>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 6: hipLaunchKernelGGL(k<6>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 7: hipLaunchKernelGGL(k<7>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 8: hipLaunchKernelGGL(k<8>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        default: hipLaunchKernelGGL(k<9>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
      }
      (void)hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(256);
    (void)hipMemcpy(h.data(), cyc, 256 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    printf("{\"mode\": \"%s\", \"cycles_per_mfma\": %.2f}\n", names[mode], s / 256 / (ITERS * 4.0));
  }
  return 0;
}
