// Elementary functions for the dynamics functors (gfx950). Private header.
#pragma once
#include <hip/hip_runtime.h>
#include <math.h>

namespace ilqr {
namespace {

// ---------------------------------------------------------------------------
// sin and cos together: Cody-Waite reduction by π/2 (three-part constant, exact
// for |x| < 1e5) and the fdlibm kernel polynomials on [−π/4, π/4]. ≤ 1 ulp from
// glibc over |x| ≤ 200 (checked on 2·10⁷ points); ≈ 35 instructions where the
// device library's sincos (with its Payne-Hanek path) is ≈ 190 — the dynamics
// evaluate it four times per RK4 step. Larger |x| falls back to the library.
// ---------------------------------------------------------------------------
__device__ __attribute__((noinline)) void big_sincos(double x, double* s, double* c) {
  sincos(x, s, c);
}
// the reduction and polynomials alone: valid for |x| ≤ 1e5 (a caller that cannot
// branch per evaluation checks the range itself and redoes the rare large argument)
__device__ __forceinline__ void sincos_reduced(double x, double& s, double& c) {
  const double k = rint(x * 6.36619772367581382433e-01);  // x · 2/π
  double r = fma(-k, 1.5707963267948966e+00, x);
  r = fma(-k, 6.123233995736766e-17, r);
  r = fma(-k, -1.4973849048591698e-33, r);
  const double z = r * r;
  double ps = fma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08);
  ps = fma(z, ps, 2.75573137070700676789e-06);
  ps = fma(z, ps, -1.98412698298579493134e-04);
  ps = fma(z, ps, 8.33333333332248946124e-03);
  ps = fma(z, ps, -1.66666666666666324348e-01);
  const double sr = fma(r * z, ps, r);
  double pc = fma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09);
  pc = fma(z, pc, -2.75573143513906633035e-07);
  pc = fma(z, pc, 2.48015872894767294178e-05);
  pc = fma(z, pc, -1.38888888888741095749e-03);
  pc = fma(z, pc, 4.16666666666666019037e-02);
  const double hz = 0.5 * z;
  const double w = 1.0 - hz;
  const double cr = w + (((1.0 - w) - hz) + z * z * pc);
  const int q = (int)k & 3;
  const double a = (q & 1) ? cr : sr;
  const double b = (q & 1) ? sr : cr;
  s = (q & 2) ? -a : a;
  c = ((q + 1) & 2) ? -b : b;
}
__device__ __forceinline__ void fast_sincos(double x, double& s, double& c) {
  if (__builtin_expect(fabs(x) > 1e5, 0)) {
    big_sincos(x, &s, &c);
    return;
  }
  sincos_reduced(x, s, c);
}

// fp32 counterpart: Cody-Waite reduction by π/2 (three-part float constant, Cephes
// split, exact enough for |x| < 8192) and the Cephes sinf/cosf minimax polynomials
// on [−π/4, π/4]; ≈1 ulp. The device library's sincosf carries a Payne-Hanek path
// whose registers made the chain dynamics spill.
__device__ __attribute__((noinline)) void big_sincosf(float x, float* s, float* c) {
  sincosf(x, s, c);
}
__device__ __forceinline__ void sincosf_reduced(float x, float& s, float& c);
__device__ __forceinline__ void fast_sincosf(float x, float& s, float& c) {
  if (__builtin_expect(fabsf(x) > 8192.0f, 0)) {
    big_sincosf(x, &s, &c);
    return;
  }
  sincosf_reduced(x, s, c);
}
// the reduction and polynomials alone: valid for |x| ≤ 8192
__device__ __forceinline__ void sincosf_reduced(float x, float& s, float& c) {
  const float k = rintf(x * 0.63661977236758134f);  // x · 2/π
  float r = fmaf(-k, 1.5703125f, x);
  r = fmaf(-k, 4.837512969970703125e-4f, r);
  r = fmaf(-k, 7.54978995489188216e-8f, r);
  const float z = r * r;
  float ps = fmaf(z, -1.9515295891e-4f, 8.3321608736e-3f);
  ps = fmaf(z, ps, -1.6666654611e-1f);
  const float sr = fmaf(r * z, ps, r);
  float pc = fmaf(z, 2.443315711809948e-5f, -1.388731625493765e-3f);
  pc = fmaf(z, pc, 4.166664568298827e-2f);
  const float cr = fmaf(z * z, pc, fmaf(-0.5f, z, 1.0f));
  const int q = (int)k & 3;
  const float a = (q & 1) ? cr : sr;
  const float b = (q & 1) ? sr : cr;
  s = (q & 2) ? -a : a;
  c = ((q + 1) & 2) ? -b : b;
}

// sin/cos(θ + h) from s0 = sin θ, c0 = cos θ by the angle-addition formulas and Taylor
// series in h, for |h| ≤ 1/8 (the caller flags larger h): fp64 through h⁹ / h¹⁰,
// fp32 through h⁵ / h⁴ (truncation below 0.2 ulp of the type in both)
__device__ __forceinline__ void sincos_shift_t(double s0, double c0, double h, double& s, double& c) {
  const double z = h * h;
  double ps = fma(z, 1.0 / 362880.0, -1.0 / 5040.0);
  ps = fma(z, ps, 1.0 / 120.0);
  ps = fma(z, ps, -1.0 / 6.0);
  const double sh = fma(h * z, ps, h);
  double pc = fma(z, -1.0 / 3628800.0, 1.0 / 40320.0);
  pc = fma(z, pc, -1.0 / 720.0);
  pc = fma(z, pc, 1.0 / 24.0);
  pc = fma(z, pc, -0.5);
  const double ch = fma(z, pc, 1.0);
  s = fma(s0, ch, c0 * sh);
  c = fma(c0, ch, -(s0 * sh));
}
__device__ __forceinline__ void sincos_shift_t(float s0, float c0, float h, float& s, float& c) {
  const float z = h * h;
  const float sh = fmaf(h * z, fmaf(z, 1.0f / 120.0f, -1.0f / 6.0f), h);
  const float ch = fmaf(z, fmaf(z, 1.0f / 24.0f, -0.5f), 1.0f);
  s = fmaf(s0, ch, c0 * sh);
  c = fmaf(c0, ch, -(s0 * sh));
}
__device__ __forceinline__ void sincos_red_t(double x, double& s, double& c) { sincos_reduced(x, s, c); }
__device__ __forceinline__ void sincos_red_t(float x, float& s, float& c) { sincosf_reduced(x, s, c); }
template <class V> struct ReducedRange;                       // |x| the reductions cover
template <> struct ReducedRange<double> { static constexpr double v = 1e5; };
template <> struct ReducedRange<float> { static constexpr float v = 8192.0f; };

}  // namespace
}  // namespace ilqr
