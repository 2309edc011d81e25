// Microbenchmark: f64 MFMA (v_mfma_f64_16x16x4_f64) vs f64 VALU FMA rates on gfx950,
// and whether the two pipes overlap when different waves of one SIMD issue them.
// Used to choose the backward-pass mapping. Not part of the product.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d4 __attribute__((ext_vector_type(4)));

#define CHECK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

// mode 0: MFMA, NACC independent accumulators; mode 1: VALU fma f64, 8 independent chains;
// mode 2: waves with (wave id & 1)==0 do MFMA, odd waves do VALU (co-issue test)
template <int MODE, int NACC>
__global__ __launch_bounds__(256) void kern(double* out, long long* cyc, int iters) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  double a = 1.0 + lane * 1e-3, b = 1.0 - lane * 1e-3;
  long long t0 = __builtin_amdgcn_s_memtime();
  double res = 0;
  bool do_mfma = (MODE == 0) || (MODE == 2 && (wid & 1) == 0);
  if (MODE == 5) {  // one wave: 8-acc 4x4x4_4b MFMAs, each followed by NACC-1 fmas on 8 independent chains
    double acc[8], c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) { acc[i] = 0.0; c[i] = 0.5 + lane + i; }
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < NACC - 1; ++r) c[(i + r) & 7] = __builtin_fma(c[(i + r) & 7], a, b);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) res += acc[i] + c[i];
  } else if (MODE == 4) {  // one wave: 8-acc 4x4x4_4b MFMAs with NACC dependent VALU fmas after each
    double acc[8], c = 0.5 + lane;
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
#pragma unroll
        for (int r = 0; r < NACC - 1; ++r) c = __builtin_fma(c, a, b);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) res += acc[i];
    res += c;
  } else if (MODE == 3) {  // v_mfma_f64_4x4x4_4b: four independent 4×4×4 blocks per instruction
    double acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NACC; ++i) res += acc[i];
  } else if (do_mfma) {
    d4 acc[NACC];
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < NACC; ++i) res += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  } else {
    double c[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) c[i] = i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < NACC; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) c[i] = __builtin_fma(c[i], a, b);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) res += c[i];
  }
  long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = res;
  if (lane == 0) cyc[blockIdx.x * 4 + wid] = t1 - t0;
}

template <int MODE, int NACC>
int run(const char* name, int blocks, int iters) {
  double* out; long long* cyc;
  CHECK(hipMalloc(&out, blocks * 256 * sizeof(double)));
  CHECK(hipMalloc(&cyc, blocks * 4 * sizeof(long long)));
  hipEvent_t e0, e1; CHECK(hipEventCreate(&e0)); CHECK(hipEventCreate(&e1));
  kern<MODE, NACC><<<blocks, 256>>>(out, cyc, iters);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  kern<MODE, NACC><<<blocks, 256>>>(out, cyc, iters);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms; CHECK(hipEventElapsedTime(&ms, e0, e1));
  std::vector<long long> c(blocks * 4);
  CHECK(hipMemcpy(c.data(), cyc, c.size() * 8, hipMemcpyDeviceToHost));
  double avg = 0; for (auto v : c) avg += v; avg /= c.size();
  double waves_per_simd = blocks * 4.0 / 1024.0;
  long long nops = (long long)iters * NACC * (MODE == 1 ? 8 : 1);
  // flops: MFMA 16x16x4 = 2048 flop per wave-instr; VALU fma wave64 = 128 flop
  double flop_per = (MODE == 1) ? 128.0 : (MODE == 3 ? 512.0 : 2048.0);
  double tflops;
  if (MODE == 2) tflops = (blocks * 2.0 * nops * 2048.0 + blocks * 2.0 * (double)iters * NACC * 8 * 128.0) / (ms * 1e-3) / 1e12;
  else tflops = blocks * 4.0 * nops * flop_per / (ms * 1e-3) / 1e12;
  printf("%-28s blocks=%5d waves/SIMD=%.1f  ms=%8.3f  cyc/wave=%10.0f  cyc/op/wave=%7.2f  TFLOP/s=%7.2f\n",
         name, blocks, waves_per_simd, ms, avg, avg / nops, tflops);
  CHECK(hipFree(out)); CHECK(hipFree(cyc));
  return 0;
}

int main() {
  hipDeviceProp_t p; hipGetDeviceProperties(&p, 0);
  printf("device %s CUs=%d clock=%d kHz\n", p.gcnArchName, p.multiProcessorCount, p.clockRate);
  const int it = 4000;
  run<0, 1>("mfma_f64 1 acc (latency)", 256, it);
  run<0, 4>("mfma_f64 4 acc", 256, it / 4);
  run<0, 4>("mfma_f64 4 acc", 1024, it / 4);
  run<0, 1>("mfma_f64 1 acc", 1024, it);
  run<0, 1>("mfma_f64 1 acc", 2048, it);
  run<1, 1>("valu fma_f64 8 chains", 256, it);
  run<1, 1>("valu fma_f64 8 chains", 1024, it);
  run<1, 1>("valu fma_f64 8 chains", 2048, it);
  run<2, 4>("mixed mfma(4acc)|valu(4x8)", 512, it / 4);
  run<2, 4>("mixed mfma(4acc)|valu(4x8)", 1024, it / 4);
  run<3, 1>("mfma_f64 4x4x4_4b 1 acc", 256, it);
  run<3, 4>("mfma_f64 4x4x4_4b 4 acc", 256, it / 4);
  run<3, 4>("mfma_f64 4x4x4_4b 4 acc", 1024, it / 4);
  run<3, 8>("mfma_f64 4x4x4_4b 8 acc", 1024, it / 8);
  run<0, 4>("mfma_f64 16x16x4 4 acc (again)", 1024, it / 4);
  run<3, 8>("mfma_f64 4x4x4_4b 8 acc", 256, it / 8);
  run<3, 16>("mfma_f64 4x4x4_4b 16 acc", 256, it / 16);
  run<3, 8>("mfma_f64 4x4x4_4b 8 acc", 512, it / 8);
  run<3, 16>("mfma_f64 4x4x4_4b 16 acc", 512, it / 16);
  run<4, 1>("4x4x4 8 acc, 0 valu/mfma", 256, it / 8);
  run<4, 2>("4x4x4 8 acc + 1 dep valu/mfma", 256, it / 8);
  run<4, 3>("4x4x4 8 acc + 2 dep valu/mfma", 256, it / 8);
  run<4, 5>("4x4x4 8 acc + 4 dep valu/mfma", 256, it / 8);
  run<5, 2>("4x4x4 8 acc + 1 indep valu/mfma", 256, it / 8);
  run<5, 3>("4x4x4 8 acc + 2 indep valu/mfma", 256, it / 8);
  run<5, 5>("4x4x4 8 acc + 4 indep valu/mfma", 256, it / 8);
  return 0;
}
