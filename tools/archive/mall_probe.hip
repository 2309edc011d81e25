// Does a buffer the previous kernel wrote come back from the Infinity Cache (MALL)?
// (diagnostic, not product). For each size: kernel W writes the buffer, kernel R
// streams it back (reduction); R's bandwidth against size. A read served by the
// 256 MB memory-side cache would run above the HBM rate for sizes below it.
// Also: R after a second, unrelated write of the same size (the buffer evicted).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void wr(double4* p, size_t n, double v) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    p[i] = make_double4(v, v + 1, v + 2, v + 3);
}
__global__ void rd(const double4* p, size_t n, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const double4 q = p[i];
    s += q.x + q.y + q.z + q.w;
  }
  if (s == 12345.678) out[0] = s;  // keep the loads
}

int main() {
  const size_t MB = 1 << 20;
  const size_t sizes[] = {32 * MB, 64 * MB, 128 * MB, 170 * MB, 224 * MB, 320 * MB, 512 * MB, 2048 * MB};
  double4 *a, *b;
  double* out;
  hipMalloc(&a, 2048 * MB);
  hipMalloc(&b, 2048 * MB);
  hipMalloc(&out, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int grid = 256 * 8, block = 256;
  for (size_t S : sizes) {
    const size_t n = S / sizeof(double4);
    float best_hot = 1e9, best_cold = 1e9, best_w = 1e9;
    for (int rep = 0; rep < 6; ++rep) {
      float ms;
      hipEventRecord(e0);
      wr<<<grid, block>>>(a, n, rep);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      best_w = ms < best_w ? ms : best_w;
      hipEventRecord(e0);
      rd<<<grid, block>>>(a, n, out);  // right after its write
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      best_hot = ms < best_hot ? ms : best_hot;
      wr<<<grid, block>>>(b, 1024 * MB / sizeof(double4), rep);  // 1 GB of other traffic
      hipEventRecord(e0);
      rd<<<grid, block>>>(a, n, out);  // evicted
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      hipEventElapsedTime(&ms, e0, e1);
      best_cold = ms < best_cold ? ms : best_cold;
    }
    printf("%5zu MB: write %6.2f TB/s   read after write %6.2f TB/s   read after 1 GB elsewhere %6.2f TB/s\n",
           S / MB, S / best_w / 1e9, S / best_hot / 1e9, S / best_cold / 1e9);
  }
  return 0;
}
