// Microbenchmark (round 5): dependent chains of v_fmac_f64_dpp row_newbcast at one wave
// per SIMD — 16 FMAs per dot product spread over 1, 2 or 4 accumulators, plus the zeroing
// moves and the final adds the dot needs — to see whether the ring forward's 4-accumulator
// dots (ilqr_fwd_ring.h) could use fewer. Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
#define F(A, K) "v_fmac_f64_dpp %[" #A "], %[s], %[c] row_newbcast:" #K " row_mask:0xf bank_mask:0xf\n\t"

template <int NACC>
__device__ __forceinline__ double dot16(double s, double c) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if constexpr (NACC == 1) {
    asm volatile("s_nop 4\n\t" F(a0, 0) F(a0, 1) F(a0, 2) F(a0, 3) F(a0, 4) F(a0, 5) F(a0, 6) F(a0, 7) F(a0, 8)
                     F(a0, 9) F(a0, 10) F(a0, 11) F(a0, 12) F(a0, 13) F(a0, 14) F(a0, 15)
                 : [a0] "+v"(a0) : [s] "v"(s), [c] "v"(c));
    return a0;
  } else if constexpr (NACC == 2) {
    asm volatile("s_nop 4\n\t" F(a0, 0) F(a1, 1) F(a0, 2) F(a1, 3) F(a0, 4) F(a1, 5) F(a0, 6) F(a1, 7) F(a0, 8)
                     F(a1, 9) F(a0, 10) F(a1, 11) F(a0, 12) F(a1, 13) F(a0, 14) F(a1, 15)
                 : [a0] "+v"(a0), [a1] "+v"(a1) : [s] "v"(s), [c] "v"(c));
    return a0 + a1;
  } else {
    asm volatile("s_nop 4\n\t" F(a0, 0) F(a1, 1) F(a2, 2) F(a3, 3) F(a0, 4) F(a1, 5) F(a2, 6) F(a3, 7) F(a0, 8)
                     F(a1, 9) F(a2, 10) F(a3, 11) F(a0, 12) F(a1, 13) F(a2, 14) F(a3, 15)
                 : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3) : [s] "v"(s), [c] "v"(c));
    return (a0 + a1) + (a2 + a3);
  }
}

// two independent dots per iteration (the ring step has the A x̄ and K δx dots in flight
// together), each result feeding the next iteration's source (the step's dependence)
template <int NACC>
__global__ __launch_bounds__(64) void kern(double* out, int iters) {
  double x = 1.0 + threadIdx.x * 1e-9, y = 1.0 - threadIdx.x * 1e-9;
  const double c = 0.5;
  for (int it = 0; it < iters; ++it) {
    const double p = dot16<NACC>(x, c);
    const double q = dot16<NACC>(y, c);
    x = p * 0.0625 + 0.5;
    y = q * 0.0625 + 0.5;
  }
  out[blockIdx.x * 64 + threadIdx.x] = x + y;
}

template <int NACC>
int run(int cus) {
  double* d;
  CHECK(hipMalloc(&d, sizeof(double) * 64 * cus * 4));
  const int iters = 20000;
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  kern<NACC><<<cus * 4, 64>>>(d, 100);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  kern<NACC><<<cus * 4, 64>>>(d, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double ns_per_dot = ms * 1e6 / iters / 2;
  printf("%d accumulator(s): %.2f ns per 16-FMA dot (%.2f ns per FMA incl. zeroing + adds), 1 wave/SIMD\n", NACC,
         ns_per_dot, ns_per_dot / 16);
  CHECK(hipFree(d));
  return 0;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  for (int rep = 0; rep < 2; ++rep) {
    if (run<4>(cus) || run<2>(cus) || run<1>(cus)) return 1;
  }
  return 0;
}
