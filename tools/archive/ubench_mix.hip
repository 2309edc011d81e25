// Which VALU instructions hide behind the 4-block f64 MFMA on gfx950? (diagnostic, not
// product). One wave per SIMD runs 64 v_mfma_f64_4x4x4_4b (four independent
// accumulators) with 64 instructions of one kind interleaved (independent of the MFMAs
// and of each other); cycles per MFMA from s_memtime. The backward's step interleaves
// f64 VALU (factorisation), b32 selects and LDS permutes with its MFMAs.
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
#define MF "v_mfma_f64_4x4x4_4b_f64 %[a0], %[x], %[y], %[a0]\n\t"                      \
           "v_mfma_f64_4x4x4_4b_f64 %[a1], %[x], %[y], %[a1]\n\t"                      \
           "v_mfma_f64_4x4x4_4b_f64 %[a2], %[x], %[y], %[a2]\n\t"                      \
           "v_mfma_f64_4x4x4_4b_f64 %[a3], %[x], %[y], %[a3]\n\t"
#define AOUT [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3)
#define XIN [x] "v"(x), [y] "v"(y)

template <int KIND>
__global__ __launch_bounds__(256) void k(double* out, long long* cyc) {
  double a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, x = 1.0 + threadIdx.x * 1e-3, y = 0.5;
  double f0 = 1, f1 = 2, f2 = 3, f3 = 4;
  unsigned u0 = threadIdx.x, u1 = u0 + 1, u2 = u0 + 2, u3 = u0 + 3;
  const int ad = ((threadIdx.x & ~3) | 1) * 4;
  long long t0 = __builtin_readcyclecounter();
  for (int it = 0; it < 16; ++it) {
    if constexpr (KIND == 0) {  // MFMAs alone
      asm volatile(REP8(MF) : AOUT : XIN);
    } else if constexpr (KIND == 1) {  // + v_cndmask_b32 (vcc-free form)
      asm volatile(REP8(MF "v_cndmask_b32_e32 %[u0], %[u0], %[u1], vcc\n\t"
                           "v_cndmask_b32_e32 %[u1], %[u1], %[u2], vcc\n\t"
                           "v_cndmask_b32_e32 %[u2], %[u2], %[u3], vcc\n\t"
                           "v_cndmask_b32_e32 %[u3], %[u3], %[u0], vcc\n\t")
                   : AOUT, [u0] "+v"(u0), [u1] "+v"(u1), [u2] "+v"(u2), [u3] "+v"(u3) : XIN : "vcc");
    } else if constexpr (KIND == 2) {  // + v_add_u32
      asm volatile(REP8(MF "v_add_u32 %[u0], %[u0], %[u1]\n\t"
                           "v_add_u32 %[u1], %[u1], %[u2]\n\t"
                           "v_add_u32 %[u2], %[u2], %[u3]\n\t"
                           "v_add_u32 %[u3], %[u3], %[u0]\n\t")
                   : AOUT, [u0] "+v"(u0), [u1] "+v"(u1), [u2] "+v"(u2), [u3] "+v"(u3) : XIN);
    } else if constexpr (KIND == 3) {  // + v_fma_f64
      asm volatile(REP8(MF "v_fma_f64 %[f0], %[f0], %[x], %[y]\n\t"
                           "v_fma_f64 %[f1], %[f1], %[x], %[y]\n\t"
                           "v_fma_f64 %[f2], %[f2], %[x], %[y]\n\t"
                           "v_fma_f64 %[f3], %[f3], %[x], %[y]\n\t")
                   : AOUT, [f0] "+v"(f0), [f1] "+v"(f1), [f2] "+v"(f2), [f3] "+v"(f3) : XIN);
    } else if constexpr (KIND == 4) {  // + v_fma_f32
      asm volatile(REP8(MF "v_fma_f32 %[u0], %[u0], %[u1], %[u2]\n\t"
                           "v_fma_f32 %[u1], %[u1], %[u2], %[u3]\n\t"
                           "v_fma_f32 %[u2], %[u2], %[u3], %[u0]\n\t"
                           "v_fma_f32 %[u3], %[u3], %[u0], %[u1]\n\t")
                   : AOUT, [u0] "+v"(u0), [u1] "+v"(u1), [u2] "+v"(u2), [u3] "+v"(u3) : XIN);
    } else if constexpr (KIND == 7) {  // + ds_bpermute_b32 (results consumed after the group)
      asm volatile(REP8(MF "ds_bpermute_b32 %[u0], %[ad], %[u1]\n\t"
                           "ds_bpermute_b32 %[u1], %[ad], %[u2]\n\t"
                           "ds_bpermute_b32 %[u2], %[ad], %[u3]\n\t"
                           "ds_bpermute_b32 %[u3], %[ad], %[u0]\n\t") "s_waitcnt lgkmcnt(0)\n\t"
                   : AOUT, [u0] "+v"(u0), [u1] "+v"(u1), [u2] "+v"(u2), [u3] "+v"(u3) : XIN, [ad] "v"(ad));
    } else if constexpr (KIND == 8) {  // + v_mov_b32 DPP quad broadcast
      asm volatile(REP8(MF "v_mov_b32_dpp %[u0], %[u1] quad_perm:[1,1,1,1] row_mask:0xf bank_mask:0xf\n\t"
                           "v_mov_b32_dpp %[u1], %[u2] quad_perm:[2,2,2,2] row_mask:0xf bank_mask:0xf\n\t"
                           "v_mov_b32_dpp %[u2], %[u3] quad_perm:[3,3,3,3] row_mask:0xf bank_mask:0xf\n\t"
                           "v_mov_b32_dpp %[u3], %[u0] quad_perm:[0,0,0,0] row_mask:0xf bank_mask:0xf\n\t")
                   : AOUT, [u0] "+v"(u0), [u1] "+v"(u1), [u2] "+v"(u2), [u3] "+v"(u3) : XIN);
    } else if constexpr (KIND == 5) {  // the 64 b32 selects alone
      asm volatile(REP8("v_cndmask_b32_e32 %0, %0, %1, vcc\n\t"
                        "v_cndmask_b32_e32 %1, %1, %2, vcc\n\t"
                        "v_cndmask_b32_e32 %2, %2, %3, vcc\n\t"
                        "v_cndmask_b32_e32 %3, %3, %0, vcc\n\t")
                   : "+v"(u0), "+v"(u1), "+v"(u2), "+v"(u3) : : "vcc");
    } else if constexpr (KIND == 6) {  // the 64 f64 FMAs alone
      asm volatile(REP8("v_fma_f64 %0, %0, %4, %5\n\t"
                        "v_fma_f64 %1, %1, %4, %5\n\t"
                        "v_fma_f64 %2, %2, %4, %5\n\t"
                        "v_fma_f64 %3, %3, %4, %5\n\t")
                   : "+v"(f0), "+v"(f1), "+v"(f2), "+v"(f3) : "v"(x), "v"(y));
    }
  }
  long long t1 = __builtin_readcyclecounter();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + f0 + f1 + f2 + f3 + u0 + u1 + u2 + u3;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

int main() {
  const int G = 256;  // one workgroup of 4 waves per CU: one wave per SIMD
  double* out;
  long long* cyc;
  hipMalloc(&out, G * 256 * 8);
  hipMalloc(&cyc, G * 8);
  const char* names[] = {"64 MFMA", "64 MFMA + 64 v_cndmask_b32", "64 MFMA + 64 v_add_u32", "64 MFMA + 64 v_fma_f64",
                         "64 MFMA + 64 v_fma_f32", "64 v_cndmask_b32 alone", "64 v_fma_f64 alone",
                         "64 MFMA + 64 ds_bpermute_b32", "64 MFMA + 64 v_mov_b32_dpp"};
  void (*kern[])(double*, long long*) = {k<0>, k<1>, k<2>, k<3>, k<4>, k<5>, k<6>, k<7>, k<8>};
  for (int rep = 0; rep < 2; ++rep)
    for (int v = 0; v < 9; ++v) {
      kern[v]<<<G, 256>>>(out, cyc);
      long long h[G];
      hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
      double s = 0;
      for (int i = 0; i < G; ++i) s += h[i];
      // s_memtime-based counter: report per group of 64 (per `it`) in counter ticks
      printf("%-32s %8.1f ticks per 64-op group\n", names[v], s / G / 16);
    }
  return 0;
}
