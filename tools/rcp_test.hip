// Accuracy of v_rcp_f64 and Newton refinements on gfx950 (diagnostic, not product).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cmath>
#include <vector>
#include <random>
__global__ void k(const double* x, double* r0, double* r1, double* r2, int n) {
  int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  double v = x[i];
  double r = __builtin_amdgcn_rcp(v);
  r0[i] = r;
  double e = fma(-v, r, 1.0); double a = fma(r, e, r);
  r1[i] = a;
  e = fma(-v, a, 1.0); r2[i] = fma(a, e, a);
}
int main() {
  const int n = 1 << 20;
  std::vector<double> x(n); std::mt19937_64 g(3); std::uniform_real_distribution<double> U(-20, 20);
  for (auto& v : x) { v = std::ldexp(1.0 + std::fabs(U(g)) / 20.0, (int)U(g)); if (g() & 1) v = -v; }
  double *xd, *a, *b, *c; hipMalloc(&xd, n * 8); hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&c, n * 8);
  hipMemcpy(xd, x.data(), n * 8, hipMemcpyHostToDevice);
  k<<<n / 256, 256>>>(xd, a, b, c, n);
  std::vector<double> r[3] = {std::vector<double>(n), std::vector<double>(n), std::vector<double>(n)};
  hipMemcpy(r[0].data(), a, n * 8, hipMemcpyDeviceToHost); hipMemcpy(r[1].data(), b, n * 8, hipMemcpyDeviceToHost);
  hipMemcpy(r[2].data(), c, n * 8, hipMemcpyDeviceToHost);
  for (int s = 0; s < 3; ++s) {
    double worst = 0;
    for (int i = 0; i < n; ++i) { double ex = 1.0 / x[i]; double ulp = std::fabs(std::nextafter(ex, INFINITY) - ex);
      worst = std::fmax(worst, std::fabs(r[s][i] - ex) / ulp); }
    printf("newton steps %d: max err %.3g ulp\n", s, worst);
  }
  return 0;
}
