// Microbenchmark: f64 FMA throughput on gfx950 for the operand-delivery forms a
// VALU Riccati step would use, at 1/2/4 waves per SIMD:
//   plain   v_fma_f64 (16 independent accumulators)
//   dpp     v_fmac_f64_dpp row_newbcast:k (DPP64 broadcast of lane k of each row)
//   swap    v_permlane16_swap_b32 pairs + v_add_f64 (a cross-row reduction step)
// Used to decide the backward-pass mapping. Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

#define DPP16(A, S, C)                                                                            \
  asm volatile(                                                                                   \
      "v_fmac_f64_dpp %0, %16, %17 row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %1, %16, %17 row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %2, %16, %17 row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %3, %16, %17 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %4, %16, %17 row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %5, %16, %17 row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %6, %16, %17 row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %7, %16, %17 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %8, %16, %17 row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %9, %16, %17 row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"                  \
      "v_fmac_f64_dpp %10, %16, %17 row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"                \
      "v_fmac_f64_dpp %11, %16, %17 row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"                \
      "v_fmac_f64_dpp %12, %16, %17 row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"                \
      "v_fmac_f64_dpp %13, %16, %17 row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"                \
      "v_fmac_f64_dpp %14, %16, %17 row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"                \
      "v_fmac_f64_dpp %15, %16, %17 row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"                \
      : "+v"(A[0]), "+v"(A[1]), "+v"(A[2]), "+v"(A[3]), "+v"(A[4]), "+v"(A[5]), "+v"(A[6]),     \
        "+v"(A[7]), "+v"(A[8]), "+v"(A[9]), "+v"(A[10]), "+v"(A[11]), "+v"(A[12]), "+v"(A[13]),  \
        "+v"(A[14]), "+v"(A[15])                                                                \
      : "v"(S), "v"(C))

// MODE 0 plain fma, 1 dpp fma, 2 permlane16 swap + add
template <int MODE>
__global__ __launch_bounds__(64) void kern(double* out, int iters) {
  const int lane = threadIdx.x;
  double a = 1.0 + lane * 1e-9, b = 1.0 - lane * 1e-9;
  double acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = i * 1e-3;
  for (int it = 0; it < iters; ++it) {
    if constexpr (MODE == 0) {
#pragma unroll
      for (int i = 0; i < 16; ++i) acc[i] = __builtin_fma(a, b, acc[i]);
      asm volatile("" : "+v"(a));
    } else if constexpr (MODE == 1) {
      DPP16(acc, a, b);
    } else {
#pragma unroll
      for (int i = 0; i < 16; i += 2) {
        union { double d; unsigned u[2]; } x, y;
        x.d = acc[i];
        y.d = acc[i + 1];
        auto lo = __builtin_amdgcn_permlane16_swap(x.u[0], y.u[0], false, false);
        auto hi = __builtin_amdgcn_permlane16_swap(x.u[1], y.u[1], false, false);
        x.u[0] = lo[0]; y.u[0] = lo[1];
        x.u[1] = hi[0]; y.u[1] = hi[1];
        acc[i] = x.d + y.d;
        acc[i + 1] = x.d - y.d;
      }
    }
  }
  double r = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) r += acc[i];
  out[blockIdx.x * 64 + lane] = r;
}

template <int MODE>
int run(const char* name, int waves_per_simd, int iters) {
  const int blocks = 1024 * waves_per_simd;
  double* out;
  CHECK(hipMalloc(&out, blocks * 64 * sizeof(double)));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  for (int w = 0; w < 3; ++w) kern<MODE><<<blocks, 64>>>(out, iters);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  kern<MODE><<<blocks, 64>>>(out, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  // wave-instructions of the measured kind per wave
  const double ops = (MODE == 2) ? iters * 8.0 * 3.0 : iters * 16.0;  // swap: 2 permlanes + 1 add per pair
  const double wave_ops_per_s = blocks * ops / (ms * 1e-3);
  const double per_simd_ns = 1e9 / (wave_ops_per_s / 1024.0);
  printf("%-34s waves/SIMD=%d  ms=%8.3f  wave-ops/SIMD/us=%7.1f  ns/op/SIMD=%6.3f  f64 TFLOP/s=%6.2f\n",
         name, waves_per_simd, ms, wave_ops_per_s / 1024.0 / 1e6, per_simd_ns,
         MODE == 2 ? 0.0 : wave_ops_per_s * 128.0 / 1e12);
  CHECK(hipFree(out));
  return 0;
}

int main() {
  hipDeviceProp_t p; CHECK(hipGetDeviceProperties(&p, 0));
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  const int it = 20000;
  for (int w : {1, 2, 4, 8}) run<0>("plain v_fma_f64, 16 acc", w, it);
  for (int w : {1, 2, 4, 8}) run<1>("dpp v_fmac_f64 row_newbcast, 16 acc", w, it);
  for (int w : {1, 2, 4}) run<2>("permlane16_swap x2 + add/sub", w, it);
  return 0;
}
