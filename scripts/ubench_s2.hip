// Cycle cost of the k_score_1p sweep-2 pair sequence (one wave per SIMD, no
// memory): variants remove parts of it to find what the matrix pipe waits on.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
typedef float f32x4 __attribute__((ext_vector_type(4)));
constexpr int ITERS = 1000;
#define M16(R, A, T) "v_mfma_f32_16x16x4_f32 %[" #R "], %[" #A "], %[" #T "], %[" #R "]\n\t"
#define M4(R, A, T) "v_mfma_f32_4x4x1_16b_f32 %[" #R "], %[" #A "], %[" #T "], %[" #R "]\n\t"
#define RD(S, P) "v_accvgpr_read_b32 %[" #S "], %[" #P "]\n\t"
#define FM(Q, S) "v_fmac_f32_e32 %[" #Q "], %[" #S "], %[" #S "]\n\t"
template <int MODE>
__global__ __launch_bounds__(256, 1) void k(float a, float b, float* out, unsigned long long* cyc) {
  f32x4 x0 = {a, b, a, b}, x1 = x0, y0 = x0, y1 = x0;
  float u0 = a, u1 = b, u2 = a, u3 = b, u4 = a, t0 = b, t1 = a, t2 = b, t3 = a, t4 = b, m0 = a, on = 1.f;
  float q0 = 0.f, q1 = 0.f, q2 = 0.f, q3 = 0.f, s0, s1, s2, s3;
  typedef float f32x2 __attribute__((ext_vector_type(2)));
  f32x2 lds2;
  float l0, l1, l2, l3, l4, l5, l6, l7;
  int laddr = (threadIdx.x & 63) * 4;
  f32x4 g0, g1;
  const float* gp = out + (threadIdx.x & 63) * 4;
  asm volatile("v_accvgpr_write_b32 %0, %1" : "=a"(x0[0]) : "v"(a));
  const unsigned long long c0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < ITERS; ++i) {
    if constexpr (MODE == 0) {  // full: 10 x 16x16 + 2 x 4x4 + 16 VALU (reads of the other pair)
      auto pair = [&](f32x4& x0, f32x4& x1, const f32x4& y0, const f32x4& y1) {
      asm volatile("s_nop 1\n\t" M16(x0, u0, t0) M16(x1, u0, t0) M16(x0, u1, t1) RD(s0, p00) FM(q0, s0) RD(s1, p10)
                   M16(x1, u1, t1) FM(q1, s1) RD(s0, p01) FM(q0, s0) M16(x0, u2, t2) RD(s1, p11) FM(q1, s1) RD(s0, p02)
                   M16(x1, u2, t2) FM(q0, s0) RD(s1, p12) FM(q1, s1) M16(x0, u3, t3) RD(s0, p03) FM(q0, s0) RD(s1, p13)
                   M16(x1, u3, t3) FM(q1, s1) M16(x0, u4, t4) M16(x1, u4, t4) "s_nop 11\n\t" M4(x0, m0, on)
                   M4(x1, m0, on)
                   : [x0] "+a"(x0), [x1] "+a"(x1), [q0] "+v"(q0), [q1] "+v"(q1), [s0] "=&v"(s0), [s1] "=&v"(s1)
                   : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0), [t1] "v"(t1),
                     [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4), [m0] "v"(m0), [on] "v"(on), [p00] "a"(y0[0]),
                     [p01] "a"(y0[1]), [p02] "a"(y0[2]), [p03] "a"(y0[3]), [p10] "a"(y1[0]), [p11] "a"(y1[1]),
                     [p12] "a"(y1[2]), [p13] "a"(y1[3]));
      };
      pair(x0, x1, y0, y1);
      pair(y0, y1, x0, x1);
    } else if constexpr (MODE == 1) {  // no VALU
      asm volatile("s_nop 1\n\t" M16(x0, u0, t0) M16(x1, u0, t0) M16(x0, u1, t1) M16(x1, u1, t1) M16(x0, u2, t2)
                   M16(x1, u2, t2) M16(x0, u3, t3) M16(x1, u3, t3) M16(x0, u4, t4) M16(x1, u4, t4) "s_nop 11\n\t"
                   M4(x0, m0, on) M4(x1, m0, on)
                   : [x0] "+a"(x0), [x1] "+a"(x1)
                   : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0), [t1] "v"(t1),
                     [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4), [m0] "v"(m0), [on] "v"(on));
    } else if constexpr (MODE == 2) {  // no VALU, no 4x4
      asm volatile("s_nop 1\n\t" M16(x0, u0, t0) M16(x1, u0, t0) M16(x0, u1, t1) M16(x1, u1, t1) M16(x0, u2, t2)
                   M16(x1, u2, t2) M16(x0, u3, t3) M16(x1, u3, t3) M16(x0, u4, t4) M16(x1, u4, t4)
                   : [x0] "+a"(x0), [x1] "+a"(x1)
                   : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0), [t1] "v"(t1),
                     [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4));
    } else if constexpr (MODE == 3) {  // 4 chains (two pairs interleaved), no VALU
      asm volatile(M16(x0, u0, t0) M16(x1, u0, t0) M16(y0, u0, t0) M16(y1, u0, t0) M16(x0, u1, t1) M16(x1, u1, t1)
                   M16(y0, u1, t1) M16(y1, u1, t1) M16(x0, u2, t2) M16(x1, u2, t2) M16(y0, u2, t2) M16(y1, u2, t2)
                   M16(x0, u3, t3) M16(x1, u3, t3) M16(y0, u3, t3) M16(y1, u3, t3) M16(x0, u4, t4) M16(x1, u4, t4)
                   M16(y0, u4, t4) M16(y1, u4, t4)
                   : [x0] "+a"(x0), [x1] "+a"(x1), [y0] "+a"(y0), [y1] "+a"(y1)
                   : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0), [t1] "v"(t1),
                     [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4));
    } else if constexpr (MODE == 4) {  // 2 chains, VGPR accumulators
      f32x4 v0 = x0, v1 = x1;
      asm volatile(M16(x0, u0, t0) M16(x1, u0, t0) M16(x0, u1, t1) M16(x1, u1, t1) M16(x0, u2, t2)
                   M16(x1, u2, t2) M16(x0, u3, t3) M16(x1, u3, t3) M16(x0, u4, t4) M16(x1, u4, t4)
                   : [x0] "+v"(v0), [x1] "+v"(v1)
                   : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0), [t1] "v"(t1),
                     [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4));
      x0 = v0; x1 = v1;
    } else if constexpr (MODE >= 6 && MODE <= 8) {  // the kernel's current pair: mu first, grouped VALU
      auto pair = [&](f32x4& x0, f32x4& x1, const f32x4& y0, const f32x4& y1, int it) {
        if constexpr (MODE >= 7) {  // nine LDS reads for the next pair, then wait for the previous nine
          asm volatile("ds_read2_b32 %0, %1 offset0:0 offset1:16\n\t"
                       "ds_read_b32 %2, %1 offset:256\n\tds_read_b32 %3, %1 offset:512\n\t"
                       "ds_read_b32 %4, %1 offset:768\n\tds_read_b32 %5, %1 offset:1024\n\t"
                       "ds_read_b32 %6, %1 offset:1280\n\tds_read_b32 %7, %1 offset:1536\n\t"
                       "ds_read_b32 %8, %1 offset:1792\n\tds_read_b32 %9, %1 offset:2048\n\t"
                       "s_waitcnt lgkmcnt(0)"
                       : "=v"(lds2), "+v"(laddr), "=v"(l0), "=v"(l1), "=v"(l2), "=v"(l3), "=v"(l4), "=v"(l5), "=v"(l6), "=v"(l7));
        }
        asm volatile("s_nop 1\n\t" M4(x0, m0, on) M4(x1, m0, on) "s_nop 4\n\t" M16(x0, u0, t0) M16(x1, u0, t0)
                     RD(s0, p00) RD(s1, p10) RD(s2, p01) RD(s3, p11) M16(x0, u1, t1) FM(q0, s0) FM(q1, s1) FM(q2, s2)
                     FM(q3, s3) M16(x1, u1, t1) RD(s0, p02) RD(s1, p12) RD(s2, p03) RD(s3, p13) M16(x0, u2, t2)
                     FM(q0, s0) FM(q1, s1) FM(q2, s2) FM(q3, s3) M16(x1, u2, t2) M16(x0, u3, t3) M16(x1, u3, t3)
                     M16(x0, u4, t4) M16(x1, u4, t4)
                     : [x0] "+a"(x0), [x1] "+a"(x1), [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3),
                       [s0] "=&v"(s0), [s1] "=&v"(s1), [s2] "=&v"(s2), [s3] "=&v"(s3)
                     : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0), [t1] "v"(t1),
                       [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4), [m0] "v"(m0), [on] "v"(on), [p00] "a"(y0[0]),
                       [p01] "a"(y0[1]), [p02] "a"(y0[2]), [p03] "a"(y0[3]), [p10] "a"(y1[0]), [p11] "a"(y1[1]),
                       [p12] "a"(y1[2]), [p13] "a"(y1[3]));
        if constexpr (MODE == 8) {  // two refill loads (L2-resident lines), waited a pair later
          asm volatile("s_waitcnt vmcnt(2)\n\tglobal_load_dwordx4 %0, %2, off\n\tglobal_load_dwordx4 %1, %2, off offset:64"
                       : "=a"(g0), "=a"(g1) : "v"(gp) : "memory");
        }
        (void)it;
      };
      pair(x0, x1, y0, y1, i);
      pair(y0, y1, x0, x1, i);
    } else if constexpr (MODE == 9 || MODE == 10 || MODE == 11) {  // VALU kind / spacing probes
      auto pair = [&](f32x4& x0, f32x4& x1, const f32x4& y0, const f32x4& y1) {
        if constexpr (MODE == 9)  // 16 fmac only, 4 per gap
          asm volatile("s_nop 1\n\t" M4(x0, m0, on) M4(x1, m0, on) "s_nop 4\n\t" M16(x0, u0, t0) M16(x1, u0, t0)
                       FM(q0, u0) FM(q1, u1) FM(q2, u2) FM(q3, u3) M16(x0, u1, t1) FM(q0, u0) FM(q1, u1) FM(q2, u2) FM(q3, u3)
                       M16(x1, u1, t1) FM(q0, u0) FM(q1, u1) FM(q2, u2) FM(q3, u3) M16(x0, u2, t2)
                       FM(q0, u0) FM(q1, u1) FM(q2, u2) FM(q3, u3) M16(x1, u2, t2) M16(x0, u3, t3) M16(x1, u3, t3)
                       M16(x0, u4, t4) M16(x1, u4, t4)
                       : [x0] "+a"(x0), [x1] "+a"(x1), [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3)
                       : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0),
                         [t1] "v"(t1), [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4), [m0] "v"(m0), [on] "v"(on));
        else if constexpr (MODE == 10)  // 16 accvgpr reads only, 4 per gap
          asm volatile("s_nop 1\n\t" M4(x0, m0, on) M4(x1, m0, on) "s_nop 4\n\t" M16(x0, u0, t0) M16(x1, u0, t0)
                       RD(s0, p00) RD(s1, p10) RD(s2, p01) RD(s3, p11) M16(x0, u1, t1) RD(s0, p02) RD(s1, p12) RD(s2, p03)
                       RD(s3, p13) M16(x1, u1, t1) RD(s0, p00) RD(s1, p10) RD(s2, p01) RD(s3, p11) M16(x0, u2, t2)
                       RD(s0, p02) RD(s1, p12) RD(s2, p03) RD(s3, p13) M16(x1, u2, t2) M16(x0, u3, t3) M16(x1, u3, t3)
                       M16(x0, u4, t4) M16(x1, u4, t4)
                       : [x0] "+a"(x0), [x1] "+a"(x1), [s0] "=&v"(s0), [s1] "=&v"(s1), [s2] "=&v"(s2), [s3] "=&v"(s3)
                       : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0),
                         [t1] "v"(t1), [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4), [m0] "v"(m0), [on] "v"(on),
                         [p00] "a"(y0[0]), [p01] "a"(y0[1]), [p02] "a"(y0[2]), [p03] "a"(y0[3]), [p10] "a"(y1[0]),
                         [p11] "a"(y1[1]), [p12] "a"(y1[2]), [p13] "a"(y1[3]));
        else  // reads + fmac, 2 per gap over 8 gaps
          asm volatile("s_nop 1\n\t" M4(x0, m0, on) M4(x1, m0, on) "s_nop 4\n\t" M16(x0, u0, t0) M16(x1, u0, t0)
                       RD(s0, p00) RD(s1, p10) M16(x0, u1, t1) RD(s2, p01) RD(s3, p11) M16(x1, u1, t1) FM(q0, s0)
                       FM(q1, s1) M16(x0, u2, t2) FM(q2, s2) FM(q3, s3) M16(x1, u2, t2) RD(s0, p02) RD(s1, p12)
                       M16(x0, u3, t3) RD(s2, p03) RD(s3, p13) M16(x1, u3, t3) FM(q0, s0) FM(q1, s1) M16(x0, u4, t4)
                       FM(q2, s2) FM(q3, s3) M16(x1, u4, t4)
                       : [x0] "+a"(x0), [x1] "+a"(x1), [q0] "+v"(q0), [q1] "+v"(q1), [q2] "+v"(q2), [q3] "+v"(q3),
                         [s0] "=&v"(s0), [s1] "=&v"(s1), [s2] "=&v"(s2), [s3] "=&v"(s3)
                       : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0),
                         [t1] "v"(t1), [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4), [m0] "v"(m0), [on] "v"(on),
                         [p00] "a"(y0[0]), [p01] "a"(y0[1]), [p02] "a"(y0[2]), [p03] "a"(y0[3]), [p10] "a"(y1[0]),
                         [p11] "a"(y1[1]), [p12] "a"(y1[2]), [p13] "a"(y1[3]));
      };
      pair(x0, x1, y0, y1);
      pair(y0, y1, x0, x1);
    } else if constexpr (MODE == 12) {  // mu-first pair without VALU (the floor of the current shape)
      auto pair = [&](f32x4& x0, f32x4& x1) {
        asm volatile("s_nop 1\n\t" M4(x0, m0, on) M4(x1, m0, on) "s_nop 4\n\t" M16(x0, u0, t0) M16(x1, u0, t0)
                     M16(x0, u1, t1) M16(x1, u1, t1) M16(x0, u2, t2) M16(x1, u2, t2) M16(x0, u3, t3) M16(x1, u3, t3)
                     M16(x0, u4, t4) M16(x1, u4, t4)
                     : [x0] "+a"(x0), [x1] "+a"(x1)
                     : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0),
                       [t1] "v"(t1), [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4), [m0] "v"(m0), [on] "v"(on));
      };
      pair(x0, x1);
      pair(y0, y1);
    } else {  // 1 chain of 10 (fully dependent)
      asm volatile(M16(x0, u0, t0) M16(x0, u0, t0) M16(x0, u1, t1) M16(x0, u1, t1) M16(x0, u2, t2)
                   M16(x0, u2, t2) M16(x0, u3, t3) M16(x0, u3, t3) M16(x0, u4, t4) M16(x0, u4, t4)
                   : [x0] "+a"(x0)
                   : [u0] "v"(u0), [u1] "v"(u1), [u2] "v"(u2), [u3] "v"(u3), [u4] "v"(u4), [t0] "v"(t0), [t1] "v"(t1),
                     [t2] "v"(t2), [t3] "v"(t3), [t4] "v"(t4));
    }
  }
  asm volatile("s_nop 15" ::: "memory");
  const unsigned long long c1 = __builtin_amdgcn_s_memtime();
  const f32x4 s = x0 + x1 + y0 + y1 + (q0 + q1 + q2 + q3 + l0 + l1 + l2 + l3 + l4 + l5 + l6 + l7 + lds2[0]) + g0 + g1;
  if (s[0] == 1.2345f) out[threadIdx.x] = s[1];
  if (threadIdx.x == 0) cyc[blockIdx.x] = c1 - c0;
}

int main() {
  float* out;
  unsigned long long* cyc;
  (void)hipMalloc(&out, 1 << 20);
  (void)hipMemset(out, 0, 1 << 20);
  (void)hipMalloc(&cyc, 4096 * 8);
  const char* names[] = {"full_pair", "no_valu", "no_valu_no_4x4", "4chains_20", "vgpr_acc_10", "1chain_10", "cur_pair", "cur_pair_lds", "cur_pair_lds_vmem", "fmac_only_4pg", "reads_only_4pg", "rd_fm_2pg", "mu_first_novalu"};
  for (int mode = 0; mode < 13; ++mode) {
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
        case 9: hipLaunchKernelGGL(k<9>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 10: hipLaunchKernelGGL(k<10>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        case 11: hipLaunchKernelGGL(k<11>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
        default: hipLaunchKernelGGL(k<12>, dim3(256), dim3(256), 0, 0, 1.0f, 1e-3f, out, cyc); break;
      }
      (void)hipDeviceSynchronize();
    }
    std::vector<unsigned long long> h(256);
    (void)hipMemcpy(h.data(), cyc, 256 * 8, hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    printf("{\"mode\": \"%s\", \"cycles_per_pair\": %.1f}\n", names[mode], s / 256 / ITERS / (mode == 0 || mode == 3 || mode >= 6 ? 2 : 1));
  }
  return 0;
}
