// MI355X (gfx950) kernels for the 2-link arm problem family (ILQR_PROBLEM_TWO_LINK):
// the reference's only runnable nonlinear example, test/2_link_example/
// 2_link_helper_functions.jl:1-108 (configs 1-2 of BASELINE.json), nx = 4, nu = 2
// (the reference's shape), and the nu = 1 variant BASELINE.json's configs 1-2 name:
// f₁(x, u) = f(x, [u₁, 0]) — build-defined (the reference multiplies inv(M), 2×2, by
// u, :63-65, so a length-1 u would throw), not reference-pinned. Every kernel is
// templated on NU ∈ {1, 2}.
//
// What replaces what:
//  * dynamicsf (RK4 of continuous_dynamics, :49-79) is a device functor templated on
//    the scalar type: `double` for the forward rollout, Dual<6> (forward-mode AD with
//    the 4 state + 2 input directions carried together) for linearize_dynamics
//    (src/backward_pass.jl:25-40, two ForwardDiff.jacobian calls). The CoriolisMatrix
//    quirk (:36-47: `for k in length(θ)` visits k = 2 only; the nested
//    jacobian(InertiaMatrix) is restated by its closed-form derivative ∂M/∂θ₂ — the
//    value ForwardDiff produces) is reproduced term by term.
//  * immediate_cost / final_cost (:82-108) are quadratic in (θ, u): their
//    ForwardDiff gradient/Hessian (src/backward_pass.jl:81-153) are the exact
//    constants lxx = diag(2,2,0,0), luu = 2I, lux = 0, lx = 2(θ-θ*), lu = 2u.
//
// Mapping:
//  * tl_linearize: one lane per (trajectory, time step) — the only part of the
//    backward pass that is parallel in time, and the FLOP-heavy one (≈3 kFLOP/step).
//    Writes J = [A | B] (+ θ, u) to a [b][t][28] workspace: each lane of the
//    sequential pass then reads its step's 224 contiguous bytes with 16-byte loads.
//  * tl_backward: four trajectories per wave on the 4-block f64 MFMA (the LQ
//    family's ilqr_bw4.hip layout), the same exact step_back rewrite as the LQ
//    kernels ([S s] = [Qxx | lx+Aᵀs] − Kᵀ((H+2μI)[K|d]); S's upper triangle
//    mirrored, so it is symmetric by construction).
//  * tl_forward: RK4 rollout + α-halving line search (src/forward_pass.jl:55-93), a
//    group of L = 4 lanes per trajectory evaluating four line-search candidates side by
//    side (one lane per trajectory past B = 65536), on an RK4 rearranged for a short
//    dependent chain (rk4_roll); inputs of step t+1 prefetched during step t.
// The sequential passes are latency-bound (one RK4 or one Riccati step per step per
// lane); with B = 1024 the chip is far from full — see DESIGN.md for the measured
// numbers and what would change that.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ilqr_internal.h"
#include "ilqr_device.h"
#include "ilqr_math.h"
#include "ilqr_fwd_group.h"
#include "../../include/ilqr.h"

namespace ilqr {
namespace {

constexpr int TL_NX = 4;
// per-step linearisation record [A | B] (4 × (4 + NU), row-major), θ₁, θ₂, u (NU),
// padded to a whole number of 16-byte pairs: the backward's whole input for a step
template <int NU> constexpr int tl_nj() { return TL_NX * (TL_NX + NU); }
template <int NU> constexpr int tl_njr() { return tl_nj<NU>() + 4; }  // 28 (NU = 2), 24 (NU = 1)
constexpr int TL_NJR_MAX = 28;
constexpr int TL_BW4_PF = 4;                     // backward prefetch depth (steps)

// ---------------------------------------------------------------------------
// Forward-mode dual numbers: value + N partials (ForwardDiff.Dual restated).
// ---------------------------------------------------------------------------
template <int N>
struct Dual {
  double v;
  double d[N];
  Dual() = default;
  __device__ __forceinline__ Dual(double c) : v(c) {  // a constant: zero partials
#pragma unroll
    for (int i = 0; i < N; ++i) d[i] = 0.0;
  }
};

template <int N>
__device__ __forceinline__ Dual<N> operator+(const Dual<N>& a, const Dual<N>& b) {
  Dual<N> r;
  r.v = a.v + b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a.d[i] + b.d[i];
  return r;
}
template <int N>
__device__ __forceinline__ Dual<N> operator-(const Dual<N>& a, const Dual<N>& b) {
  Dual<N> r;
  r.v = a.v - b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a.d[i] - b.d[i];
  return r;
}
template <int N>
__device__ __forceinline__ Dual<N> operator-(const Dual<N>& a) {
  Dual<N> r;
  r.v = -a.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = -a.d[i];
  return r;
}
template <int N>
__device__ __forceinline__ Dual<N> operator*(const Dual<N>& a, const Dual<N>& b) {
  Dual<N> r;  // (ab)' = a'b + ab'
  r.v = a.v * b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a.d[i] * b.v + a.v * b.d[i];
  return r;
}
template <int N>
__device__ __forceinline__ Dual<N> operator*(double a, const Dual<N>& b) {
  Dual<N> r;
  r.v = a * b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = a * b.d[i];
  return r;
}
template <int N>
__device__ __forceinline__ Dual<N> operator/(const Dual<N>& a, const Dual<N>& b) {
  Dual<N> r;  // (a/b)' = (a'b − ab') / b²
  r.v = a.v / b.v;
  const double b2 = b.v * b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = (a.d[i] * b.v - a.v * b.d[i]) / b2;
  return r;
}
template <int N>
__device__ __forceinline__ Dual<N> operator/(double a, const Dual<N>& b) {
  Dual<N> r;  // (a/b)' = −a b' / b²
  r.v = a / b.v;
  const double b2 = b.v * b.v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = -(a * b.d[i]) / b2;
  return r;
}
template <int N>
__device__ __forceinline__ Dual<N> operator+(double a, const Dual<N>& b) {
  Dual<N> r = b;
  r.v = a + b.v;
  return r;
}
template <int N>
__device__ __forceinline__ void sin_cos(const Dual<N>& a, Dual<N>& s, Dual<N>& c) {
  double sv, cv;
  fast_sincos(a.v, sv, cv);
  s.v = sv;
  c.v = cv;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    s.d[i] = cv * a.d[i];
    c.d[i] = -sv * a.d[i];
  }
}
__device__ __forceinline__ void sin_cos(double a, double& s, double& c) { fast_sincos(a, s, c); }

template <int N>
__device__ __forceinline__ Dual<N> seed(double v, int dir) {
  Dual<N> r;
  r.v = v;
#pragma unroll
  for (int i = 0; i < N; ++i) r.d[i] = i == dir ? 1.0 : 0.0;
  return r;
}

// 1/det on the rollout's dependent chain: v_rcp_f64 + two Newton steps (5 dependent
// ops against the IEEE division's ~10: scale, rcp, 4 FMAs, fmas, fixup); det ∈
// [δ(α−δ)−β², δ(α−δ)] is far from 0 and from the denormal range. Duals divide.
__device__ __forceinline__ double tl_recip(double x) {
  double r = __builtin_amdgcn_rcp(x);
  r = fma(r, fma(-x, r, 1.0), r);
  return fma(r, fma(-x, r, 1.0), r);
}
template <int N>
__device__ __forceinline__ Dual<N> tl_recip(const Dual<N>& x) { return 1.0 / x; }

// ---------------------------------------------------------------------------
// dynamicsf of test/2_link_example/2_link_helper_functions.jl:49-79, generic in S.
// ---------------------------------------------------------------------------
// u has NU entries; NU = 1 is f(x, [u₁, 0]) (the second torque a constant zero)
template <class S, int NU>
__device__ __forceinline__ void continuous_dynamics(const TwoLinkParams& P, const S (&x)[4],
                                                    const S (&u)[NU], S (&xd)[4]) {
  // InertiaMatrix (:29-33): M = [α+2βc₂  δ+βc₂; δ+βc₂  δ]
  S s2, c2;
  sin_cos(x[1], s2, c2);
  const S m00 = P.alpha + (2.0 * P.beta) * c2;
  const S m01 = P.delta + P.beta * c2;  // = m10
  // ∂M/∂θ₂ (the nested jacobian at :37): d/dθ₂ cos θ₂ = −sin θ₂; ∂M/∂θ₁ = 0, ∂M₂₂ = 0
  const S ns2 = -s2;
  const S dm00 = (2.0 * P.beta) * ns2;
  const S dm01 = P.beta * ns2;
  // CoriolisMatrix (:42-44) with k = 2 only: C[i,j] = ½(∇M[2,i,j] + ∇M[j,i,2] − ∇M[i,2,j])·θ̇₂
  // → C₁₁ = ½∂M₁₁θ̇₂, C₁₂ = ½((∂M₂₁ + ∂M₂₁) − ∂M₁₂)θ̇₂ = ½∂M₁₂θ̇₂, C₂₁ = ½∂M₁₂θ̇₂, C₂₂ = 0
  const S c00 = (0.5 * dm00) * x[3];
  const S c01 = (0.5 * dm01) * x[3];
  // inv(M) (:63) and M\C (:61) for the 2×2 M (δ = M₂₂ is a constant)
  const S det = P.delta * m00 - m01 * m01;
  const S idet = tl_recip(det);  // one reciprocal per evaluation (the rest are products)
  const S i00 = P.delta * idet;
  const S i01 = -(m01 * idet);
  const S i11 = m00 * idet;
  // MC = M⁻¹C, C = [c00 c01; c01 0]
  const S mc00 = i00 * c00 + i01 * c01;
  const S mc01 = i00 * c01;
  const S mc10 = i01 * c00 + i11 * c01;
  const S mc11 = i01 * c01;
  // state_dot = [θ̇; −(M\C)θ̇ + M⁻¹u] (:56-66)
  xd[0] = x[2];
  xd[1] = x[3];
  const S u1 = NU > 1 ? u[NU - 1] : S(0.0);
  xd[2] = -(mc00 * x[2] + mc01 * x[3]) + (i00 * u[0] + i01 * u1);
  xd[3] = -(mc10 * x[2] + mc11 * x[3]) + (i01 * u[0] + i11 * u1);
}

// RK4 (:71-78): k_i = Δt·f(·); x' = x + (1/6)(k1 + 2k2 + 2k3 + k4)
template <class S, int NU>
__device__ __forceinline__ void rk4(const TwoLinkParams& P, const S (&x)[4], const S (&u)[NU],
                                    S (&out)[4]) {
  S k1[4], k2[4], k3[4], k4[4], y[4];
  continuous_dynamics(P, x, u, k1);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    k1[i] = P.dt * k1[i];
    y[i] = x[i] + 0.5 * k1[i];
  }
  continuous_dynamics(P, y, u, k2);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    k2[i] = P.dt * k2[i];
    y[i] = x[i] + 0.5 * k2[i];
  }
  continuous_dynamics(P, y, u, k3);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    k3[i] = P.dt * k3[i];
    y[i] = x[i] + k3[i];
  }
  continuous_dynamics(P, y, u, k4);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    k4[i] = P.dt * k4[i];
    out[i] = x[i] + (1.0 / 6.0) * (((k1[i] + 2.0 * k2[i]) + 2.0 * k3[i]) + k4[i]);
  }
}


// The same RK4 step for the linearisation's duals (round 3), the forward's rearrangement
// of the dynamics minus its angle shifts: θ̈ = M⁻¹(u − Cθ̇) as one 2×2 solve applied to a
// vector — C = −g[1 ½; ½ 0], g = β sin θ₂ θ̇₂ (the k = 2-only Coriolis matrix of :36-47) —
// instead of M\C and M⁻¹u (≈15 dual operations per evaluation against ≈30), and θ₁'s
// stage values (f never reads them) not formed. Each stage takes sin/cos of its own θ₂
// (for duals the direct sin/cos is cheaper than the shift's polynomial).
template <class S, int NU>
__device__ __forceinline__ void tl_accel_s(const TwoLinkParams& P, const S& s2, const S& c2, const S& w1,
                                           const S& w2, const S (&u)[NU], S& a1, S& a2) {
  const S g = (P.beta * s2) * w2;
  const S r0 = g * (0.5 * w2 + w1) + u[0];  // u₁ − (Cθ̇)₁
  const S hg = 0.5 * g;
  S r1 = hg * w1;                             // u₂ − (Cθ̇)₂
  if constexpr (NU > 1) r1 = r1 + u[NU - 1];
  const S m00 = P.alpha + (2.0 * P.beta) * c2;
  const S m01 = P.delta + P.beta * c2;
  const S idet = tl_recip(P.delta * m00 - m01 * m01);
  a1 = (P.delta * r0 - m01 * r1) * idet;
  a2 = (m00 * r1 - m01 * r0) * idet;
}
template <class S, int NU>
__device__ __forceinline__ void rk4_lin(const TwoLinkParams& P, const S (&x)[4], const S (&u)[NU], S (&out)[4]) {
  S s, c, a1, a2;
  sin_cos(x[1], s, c);
  tl_accel_s<S, NU>(P, s, c, x[2], x[3], u, a1, a2);
  const S k10 = P.dt * x[2], k11 = P.dt * x[3], k12 = P.dt * a1, k13 = P.dt * a2;
  S y1 = x[1] + 0.5 * k11, y2 = x[2] + 0.5 * k12, y3 = x[3] + 0.5 * k13;
  sin_cos(y1, s, c);
  tl_accel_s<S, NU>(P, s, c, y2, y3, u, a1, a2);
  const S k20 = P.dt * y2, k21 = P.dt * y3, k22 = P.dt * a1, k23 = P.dt * a2;
  y1 = x[1] + 0.5 * k21;
  y2 = x[2] + 0.5 * k22;
  y3 = x[3] + 0.5 * k23;
  sin_cos(y1, s, c);
  tl_accel_s<S, NU>(P, s, c, y2, y3, u, a1, a2);
  const S k30 = P.dt * y2, k31 = P.dt * y3, k32 = P.dt * a1, k33 = P.dt * a2;
  y1 = x[1] + k31;
  y2 = x[2] + k32;
  y3 = x[3] + k33;
  sin_cos(y1, s, c);
  tl_accel_s<S, NU>(P, s, c, y2, y3, u, a1, a2);
  const S k40 = P.dt * y2, k41 = P.dt * y3, k42 = P.dt * a1, k43 = P.dt * a2;
  out[0] = x[0] + (1.0 / 6.0) * (((k10 + 2.0 * k20) + 2.0 * k30) + k40);
  out[1] = x[1] + (1.0 / 6.0) * (((k11 + 2.0 * k21) + 2.0 * k31) + k41);
  out[2] = x[2] + (1.0 / 6.0) * (((k12 + 2.0 * k22) + 2.0 * k32) + k42);
  out[3] = x[3] + (1.0 / 6.0) * (((k13 + 2.0 * k23) + 2.0 * k33) + k43);
}

// ---------------------------------------------------------------------------
// Linearisation: J_t = [A_t | B_t] = ∂f/∂(x,u) at (x_t, u_t), one lane per (b, t).
// ---------------------------------------------------------------------------
template <int NU>
__global__ __launch_bounds__(256) void tl_linearize_kernel(TwoLinkParams P, int B, int T,
                                                           const double* __restrict__ x,
                                                           const double* __restrict__ u,
                                                           const int32_t* __restrict__ status,
                                                           double* __restrict__ J) {
  constexpr int ND = TL_NX + NU;  // directions: the 4 states and NU inputs
  constexpr int NJ = tl_nj<NU>(), NJR = tl_njr<NU>();
  const int b = blockIdx.x * 256 + threadIdx.x;
  const int t = blockIdx.y;
  if (b >= B || (status && status[b] != ILQR_TRAJ_OK)) return;
  const double* xb = x + ((size_t)b * (T + 1) + t) * TL_NX;
  const double* ub = u + ((size_t)b * T + t) * NU;
  Dual<ND> xs[4], us[NU], out[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) xs[i] = seed<ND>(xb[i], i);
#pragma unroll
  for (int i = 0; i < NU; ++i) us[i] = seed<ND>(ub[i], 4 + i);
  rk4_lin<Dual<ND>, NU>(P, xs, us, out);
  double jv[NJR];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int k = 0; k < ND; ++k) jv[i * ND + k] = out[i].d[k];
  jv[NJ] = xb[0];
  jv[NJ + 1] = xb[1];
#pragma unroll
  for (int i = 0; i < 2; ++i) jv[NJ + 2 + i] = i < NU ? ub[i] : 0.0;
  double2* Jt = reinterpret_cast<double2*>(J + ((size_t)b * T + t) * NJR);
#pragma unroll
  for (int e = 0; e < NJR; e += 2) Jt[e / 2] = make_double2(jv[e], jv[e + 1]);
}

// linearize_dynamics (backward_pass.jl:25-40) in the caller's layout (ilqr_linearize):
// the same Dual<4+NU> RK4 as tl_linearize_kernel, so the same bits as the backward's
// own [A|B]; A (B, T, 4, 4), B (B, T, 4, NU), one lane per (b, t)
template <int NU>
__global__ __launch_bounds__(256) void tl_jacobian_kernel(TwoLinkParams P, int B, int T,
                                                          const double* __restrict__ x,
                                                          const double* __restrict__ u,
                                                          double* __restrict__ A, double* __restrict__ Bm) {
  constexpr int ND = TL_NX + NU;
  const int b = blockIdx.x * 256 + threadIdx.x;
  if (b >= B) return;
  // steps on grid y, strided past 65,535 (HIP's limit for gridDim.y)
  for (int t = blockIdx.y; t < T; t += gridDim.y) {
    const double* xb = x + ((size_t)b * (T + 1) + t) * TL_NX;
    const double* ub = u + ((size_t)b * T + t) * NU;
    Dual<ND> xs[4], us[NU], out[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) xs[i] = seed<ND>(xb[i], i);
#pragma unroll
    for (int i = 0; i < NU; ++i) us[i] = seed<ND>(ub[i], 4 + i);
    rk4_lin<Dual<ND>, NU>(P, xs, us, out);
    double* At = A + ((size_t)b * T + t) * 16;
    double* Bt = Bm + ((size_t)b * T + t) * 4 * NU;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
#pragma unroll
      for (int k = 0; k < 4; ++k) At[i * 4 + k] = out[i].d[k];
#pragma unroll
      for (int k = 0; k < NU; ++k) Bt[i * NU + k] = out[i].d[4 + k];
    }
  }
}

// ---------------------------------------------------------------------------
// Riccati recursion on the 4-block f64 MFMA (v_mfma_f64_4x4x4f64), FOUR trajectories
// per wave — the layout of the LQ family's ilqr_bw4.hip: lane
// 16ρ + 4β + κ holds element [ρ][κ] of slot β's 4×4 block, mfa(a, b, c) = c + aᵀb,
// vectors are replicated blocks (v[ρ] in every κ). nx = 4 is one block; B (4×2) is
// zero-padded to a block, so rows/columns 2, 3 of the u-side blocks are 0 (G, g, K,
// d) and the padded block of (H + μI)⁻¹ is set to 0. Per step: 11 MFMAs (S·A, S·B,
// AᵀSA + lxx, BᵀSA, BᵀSB + luu, the gradient's Aᵀs and Bᵀs, (H + μI)⁻¹ times G and g,
// the update of S and s) against ≈260 f64 VALU ops per trajectory for a lane-per-
// trajectory recursion (v6).
__device__ __forceinline__ double mfa(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ double mfa_n(double a, double b, double c) {  // −aᵀb + c
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 1);
}

// Slots whose bit in `active` is clear, or past B, compute on clamped data and store
// nothing. Returns the NaN slots (bit β). As in ilqr_bw4.hip, a NaN in any K_t or d_t
// reaches K_0 or d_0, so only the last step's gains are tested.
template <int NU>
__device__ unsigned tl_backward4_wave(const TwoLinkParams& P, int b0, int B, unsigned active, int T,
                                      const double* __restrict__ x, const double* __restrict__ J,
                                      double* __restrict__ dg, double* __restrict__ Kg, double mu,
                                      double* lds) {
  b0 = __builtin_amdgcn_readfirstlane(b0);
  const int l = threadIdx.x & 63;
  const int rho = l >> 4, beta = (l >> 2) & 3, kap = l & 3;
  const int b = b0 + beta;
  const bool live = b < B && ((active >> beta) & 1u);
  const int bc = b < B ? b : B - 1;
  const int nslot = B - b0 < 4 ? B - b0 : 4;
  constexpr int ND = TL_NX + NU, NJ = tl_nj<NU>(), NJR = tl_njr<NU>();
  const bool ru = rho < NU;  // a real u row
  const double tg = rho == 0 ? P.tgt0 : P.tgt1;

  // final_cost_quadratization (:134-153): ∇²ℓ_f = lxx = diag(2,2,0,0), ∇ℓ_f = [2(θ−θ*), 0, 0]
  const double lxx = (rho == kap && rho < 2) ? 2.0 : 0.0;  // also luu (pad rows 0)
  double S = lxx;
  const double xT = x[((size_t)bc * (T + 1) + T) * TL_NX + (rho < 2 ? rho : 0)];
  double s = rho < 2 ? -2.0 * (tg - xT) : 0.0;

  // per-step record J[b][t] = [A|B] (4×(4+NU) row-major), θ₁, θ₂, u via one buffer
  // resource over the wave's slots; the step is the scalar offset (loads past a
  // record's live entries read 0: the B block is zero-padded to 4×4)
  const auto rJ = buffer_rsrc(const_cast<double*>(J) + (size_t)b0 * T * NJR,
                              (uint32_t)(nslot * T * NJR * 8));
  const uint32_t base = (uint32_t)(beta * T * NJR * 8);
  const uint32_t oA = base + (uint32_t)((rho * ND + kap) * 8);
  const uint32_t oB = kap < NU ? base + (uint32_t)((rho * ND + 4 + kap) * 8) : 0x80000000u;
  const uint32_t oT = rho < 2 ? base + (uint32_t)((NJ + rho) * 8) : 0x80000000u;
  const uint32_t oU = ru ? base + (uint32_t)((NJ + 2 + rho) * 8) : 0x80000000u;
  auto ld = [&](uint32_t off, int t) {
    return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rJ, off, (uint32_t)(t * NJR * 8), 0));
  };
  const auto rK = buffer_rsrc(Kg + (size_t)b0 * T * NU * TL_NX, (uint32_t)(nslot * T * NU * TL_NX * 8));
  const auto rD = buffer_rsrc(dg + (size_t)b0 * T * NU, (uint32_t)(nslot * T * NU * 8));
  const uint32_t kv = (live && ru) ? (uint32_t)((beta * T * NU * TL_NX + rho * TL_NX + kap) * 8) : 0x80000000u;
  const uint32_t dv = (live && ru && kap == 0) ? (uint32_t)((beta * T * NU + rho) * 8) : 0x80000000u;
  const double Id = rho == kap ? 1.0 : 0.0;            // the identity block
  double* Hl = lds + beta * 16;

  // inputs TL_BW4_PF steps ahead in a register ring (a step is ≈0.5 µs, HBM latency
  // 1-2 µs); the loop is unrolled by the ring depth so the slots are registers
  constexpr int PF = TL_BW4_PF;
  double rA[PF], rB[PF], rT[PF], rU[PF];
#pragma unroll
  for (int k = 0; k < PF; ++k) {
    const int tk = T - 1 - k > 0 ? T - 1 - k : 0;
    rA[k] = ld(oA, tk); rB[k] = ld(oB, tk); rT[k] = ld(oT, tk); rU[k] = ld(oU, tk);
  }
  __builtin_amdgcn_s_waitcnt(0);
  double Kl = 0.0, dl = 0.0;
  auto step = [&](int t, int k) {
    const double A = rA[k], Bm = rB[k], th = rT[k], uu = rU[k];
    const int tn = t - PF > 0 ? t - PF : 0;
    rA[k] = ld(oA, tn); rB[k] = ld(oB, tn); rT[k] = ld(oT, tn); rU[k] = ld(oU, tn);
    // immediate_cost_quadratization (:81-109): lx = [2(θ−θ*), 0, 0], lu = 2u
    const double lx = rho < 2 ? -2.0 * (tg - th) : 0.0;
    const double lu = ru ? 2.0 * uu : 0.0;
    const double Y0 = mfa(S, A, 0.0);                             // S·A
    const double Z = mfa(A, Y0, lxx);                             // lxx + AᵀSA
    const double G = mfa(Bm, Y0, 0.0);                            // BᵀSA (lux = 0)
    const double gx = mfa(A, s, lx), gu = mfa(Bm, s, lu);         // lx + Aᵀs, lu + Bᵀs
    // feedback_parameters (:207-218): (H + μI)⁻¹ of the NU×NU block by its adjugate, in
    // every lane (H = 2I + BᵀSB with B = O(Δt): condition ≈ 1, so the explicit inverse
    // costs nothing in accuracy and one MFMA stage less than two triangular sweeps)
    double K, d;
    if constexpr (NU == 2) {
      const double Y1 = mfa(S, Bm, 0.0);                          // S·B
      const double H = mfa(Bm, Y1, lxx);                          // luu + BᵀSB
      Hl[rho * 4 + kap] = H;
      wave_lds_fence();
      const double h00 = Hl[0], h10 = Hl[4], h11 = Hl[5];
      wave_lds_fence();
      const double a00 = h00 + mu, a11 = h11 + mu;
      const double idet = rcp<2>(fma(a00, a11, -h10 * h10));
      const bool in2 = rho < 2 && kap < 2;
      const double Hi = !in2 ? 0.0 : (rho != kap ? -h10 : (rho == 0 ? a11 : a00)) * idet;
      K = mfa_n(Hi, G, 0.0);                                      // −(H+μI)⁻¹ G
      d = mfa_n(Hi, gu, 0.0);                                     // −(H+μI)⁻¹ g
    } else {
      // H is 1×1: with B's column replicated over κ (a quad broadcast) the two MFMAs
      // that form it leave bᵀSb in every lane of the slot — no LDS hand-off — and the
      // gains are VALU products: the bits of the block form (its other terms are 0)
      const double Br = dpp_quad_bcast0(Bm);
      const double Y1 = mfa(S, Br, 0.0);                          // S·b, replicated
      const double H = mfa(Br, Y1, 2.0);                          // luu + bᵀSb everywhere
      const double hi = rcp<2>(H + mu);
      K = -(hi * G);                                              // −(H+μ)⁻¹ G (row 0)
      d = -(hi * gu);                                             // −(H+μ)⁻¹ g
      (void)Hl;
    }
    store_or_drop(K, rK, kv != 0x80000000u, kv + (uint32_t)(t * NU * TL_NX * 8));
    store_or_drop(d, rD, dv != 0x80000000u, dv + (uint32_t)(t * NU * 8));
    // step_back (:262-273), exact rewrite: W = (H+2μI)[K|d] = μ[K|d] − [G|g]
    const double W = fma(mu, K, -G), Wd = fma(mu, d, -gu);
    const double Sf = mfa_n(K, W, Z);                             // Qxx − KᵀW_K
    // S as the reference's symmetric matrix: the upper triangle, mirrored
    // (the transpose on the MFMA, mfa(Sf, I, 0) = Sfᵀ exactly: a ≈50-cycle result where
    // a ds_bpermute round trip sat on the recursion's chain)
    const double Sm = mfa(Sf, Id, 0.0);
    S = rho <= kap ? Sf : Sm;
    s = mfa_n(K, Wd, gx);                                         // lx + Aᵀs − KᵀW_d
    Kl = K; dl = d;
  };
  int t = T - 1;
  for (; t >= PF - 1; t -= PF) {
#pragma unroll
    for (int k = 0; k < PF; ++k) step(t - k, k);
  }
#pragma unroll
  for (int k = 0; k < PF - 1; ++k)
    if (t - k >= 0) step(t - k, k);
  const unsigned long long nb = __ballot(__builtin_isnan(Kl) || __builtin_isnan(dl));
  unsigned r = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) r |= (nb & ((0xFull << (4 * q)) * 0x0001000100010001ull)) ? (1u << q) : 0u;
  return r;
}

// ---------------------------------------------------------------------------
// The rollout's RK4 in double (forward pass and rollout; the linearisation keeps
// rk4<Dual> above). The same dynamics as continuous_dynamics + rk4, rearranged for
// fewer instructions and a shorter dependent chain per step — one lane runs a step in
// ≈230 f64 ops against ≈390 for rk4<double>:
//  * θ̈ = M⁻¹(u − Cθ̇) with C = −g[1 ½; ½ 0], g = β sin θ₂ θ̇₂ (the k = 2-only Coriolis
//    matrix of the reference, :36-47), and det M = δ(α − δ) − β² cos²θ₂ (M's entries
//    are affine in cos θ₂): one 2×2 solve applied to a vector instead of M\C and M⁻¹u;
//  * θ₁ never enters f, so the stages' θ₁ is never formed;
//  * stages 2-4 take sin/cos(θ₂ + h) (h = ½k₁[2], ½k₂[2], k₃[2]) from stage 1's sin/cos θ₂
//    by the angle-addition formulas and Taylor series in h (|h| ≤ 1/8: truncation below
//    0.2 ulp); a rollout that meets a larger h is redone on rk4<double>.
// Mathematically the reference's dynamicsf (2_link_helper_functions.jl:49-79); the
// rounding differs from rk4<double>'s by a few ulp per step (tests/test_gpu_twolink.py).
// ---------------------------------------------------------------------------

struct TLRoll {
  double alpha, beta, delta, beta2, det0, bsq, dt;
};
__device__ __forceinline__ TLRoll tl_roll_consts(const TwoLinkParams& P) {
  return {P.alpha, P.beta, P.delta, 2.0 * P.beta, P.delta * (P.alpha - P.delta), P.beta * P.beta, P.dt};
}

// θ̈ at (θ₂ with sin s2 / cos c2, θ̇ = (w1, w2), u)
template <int NU>
__device__ __forceinline__ void tl_accel(const TLRoll& R, double s2, double c2, double w1, double w2,
                                         const double (&u)[NU], double& a1, double& a2) {
  const double g = (R.beta * s2) * w2;
  const double r0 = fma(g, fma(0.5, w2, w1), u[0]);  // u₁ − (Cθ̇)₁
  const double hg = 0.5 * g;
  const double r1 = NU > 1 ? fma(hg, w1, u[NU - 1]) : hg * w1;  // u₂ − (Cθ̇)₂
  const double m00 = fma(R.beta2, c2, R.alpha);
  const double m01 = fma(R.beta, c2, R.delta);
  const double idet = tl_recip(fma(-(R.bsq * c2), c2, R.det0));
  a1 = fma(R.delta, r0, -(m01 * r1)) * idet;
  a2 = fma(m00, r1, -(m01 * r0)) * idet;
}

// sin/cos(θ + h) from s0 = sin θ, c0 = cos θ, for |h| ≤ 1/8 (the caller flags larger h)
__device__ __forceinline__ void sincos_shift(double s0, double c0, double h, double& s, double& c) {
  const double z = h * h;
  double ps = fma(z, 1.0 / 362880.0, -1.0 / 5040.0);
  ps = fma(z, ps, 1.0 / 120.0);
  ps = fma(z, ps, -1.0 / 6.0);
  const double sh = fma(h * z, ps, h);  // sin h, through h⁹
  double pc = fma(z, -1.0 / 3628800.0, 1.0 / 40320.0);
  pc = fma(z, pc, -1.0 / 720.0);
  pc = fma(z, pc, 1.0 / 24.0);
  pc = fma(z, pc, -0.5);
  const double ch = fma(z, pc, 1.0);  // cos h, through h¹⁰
  s = fma(s0, ch, c0 * sh);
  c = fma(c0, ch, -(s0 * sh));
}

// dt·θ̈ at (θ₂ with sin s2 / cos c2, θ̇ = (w1, w2), u): tl_accel with dt folded into the
// reciprocal of det M (one product fewer per stage than dt·a, dt·b)
template <int NU>
__device__ __forceinline__ void tl_kdot(const TLRoll& R, double s2, double c2, double w1, double w2,
                                        const double (&u)[NU], double& ka, double& kb) {
  const double g = (R.beta * s2) * w2;
  const double r0 = fma(g, fma(0.5, w2, w1), u[0]);  // u₁ − (Cθ̇)₁
  const double hg = 0.5 * g;
  const double r1 = NU > 1 ? fma(hg, w1, u[NU - 1]) : hg * w1;  // u₂ − (Cθ̇)₂
  const double m00 = fma(R.beta2, c2, R.alpha);
  const double m01 = fma(R.beta, c2, R.delta);
  const double idt = R.dt * tl_recip(fma(-(R.bsq * c2), c2, R.det0));
  ka = fma(R.delta, r0, -(m01 * r1)) * idt;
  kb = fma(m00, r1, -(m01 * r0)) * idt;
}

// sin/cos of the state's θ₂, carried from step to step: the step's stage 1 reads it and
// leaves sin/cos(θ₂') of the new state by the same angle shift the stages use,
// h = θ₂' − θ₂ — the range reduction runs once per rollout instead of once per step
struct TLCarry {
  double s, c;
};

// One RK4 step without a branch (one basic block, so the scheduler can overlap the
// stages' independent chains and the next step's reduction). `bad` is set when an
// argument left the ranges the branch-free forms cover (|θ₂| > 1e5, a shift |h| > 1/8);
// the caller then redoes the rollout on rk4<double>. θ₁'s update sums the stage
// velocities and scales once: θ₁ feeds nothing else.
template <int NU>
__device__ __forceinline__ void rk4_roll(const TLRoll& R, const double (&x)[4], const double (&u)[NU],
                                         double (&out)[4], bool& bad, TLCarry& cy) {
  const double s1 = cy.s, c1 = cy.c;
  double s, c, k12, k13, k22, k23, k32, k33, k42, k43;
  tl_kdot<NU>(R, s1, c1, x[2], x[3], u, k12, k13);
  const double k11 = R.dt * x[3];
  double y2 = x[2] + 0.5 * k12, y3 = x[3] + 0.5 * k13;
  sincos_shift(s1, c1, 0.5 * k11, s, c);
  tl_kdot<NU>(R, s, c, y2, y3, u, k22, k23);
  const double v2 = y2, k21 = R.dt * y3;
  y2 = x[2] + 0.5 * k22;
  y3 = x[3] + 0.5 * k23;
  sincos_shift(s1, c1, 0.5 * k21, s, c);
  tl_kdot<NU>(R, s, c, y2, y3, u, k32, k33);
  const double v3 = y2, k31 = R.dt * y3;
  y2 = x[2] + k32;
  y3 = x[3] + k33;
  sincos_shift(s1, c1, k31, s, c);
  tl_kdot<NU>(R, s, c, y2, y3, u, k42, k43);
  const double k41 = R.dt * y3;
  constexpr double sixth = 1.0 / 6.0;
  out[0] = x[0] + (R.dt * sixth) * (((x[2] + 2.0 * v2) + 2.0 * v3) + y2);
  out[1] = x[1] + sixth * (((k11 + 2.0 * k21) + 2.0 * k31) + k41);
  out[2] = x[2] + sixth * (((k12 + 2.0 * k22) + 2.0 * k32) + k42);
  out[3] = x[3] + sixth * (((k13 + 2.0 * k23) + 2.0 * k33) + k43);
  const double h = out[1] - x[1];
  sincos_shift(s1, c1, h, cy.s, cy.c);
  // |h| ≤ 1/8 for h = ½k₁₁, ½k₂₁, k₃₁ ⇐ max(|k₁₁|, |k₂₁|, 2|k₃₁|) ≤ 1/4, and the carry's
  // shift (NaN: not flagged, the rollout is NaN on either path)
  const double hm = fmax(fmax(fabs(k11), fabs(k21)), fmax(2.0 * fabs(k31), 2.0 * fabs(h)));
  bad |= (hm > 0.25) | (fabs(x[1]) > 1e5);
}

// ---------------------------------------------------------------------------
// The arm as a model of the shared forward group (ilqr_fwd_group.h: four line-search
// candidates per trajectory, branch-free stores, the fast/robust RK4 pair)
// ---------------------------------------------------------------------------
template <int NU_>
struct TwoLinkModel {
  using V = double;
  static constexpr int NU = NU_;
  static constexpr bool HAS_FAST = true;
  static constexpr bool HAS_CARRY = true;
  using Carry = TLCarry;
  TwoLinkParams P;
  TLRoll R;
  __device__ __forceinline__ Carry carry_init(const double (&x)[4]) const {
    Carry k;
    sincos_reduced(x[1], k.s, k.c);
    return k;
  }
  __device__ __forceinline__ void rk4_fast(const double (&x)[4], const double (&u)[NU], double (&o)[4],
                                           bool& bad, Carry& k) const {
    rk4_roll<NU>(R, x, u, o, bad, k);
  }
  __device__ __forceinline__ void rk4_robust(const double (&x)[4], const double (&u)[NU], double (&o)[4]) const {
    rk4<double, NU>(P, x, u, o);
  }
  // ℓ(x̄ₖ − x_trajₖ, ūₖ) (forward_pass.jl:187-190; 2_link_helper_functions.jl:82-97)
  __device__ __forceinline__ double stage_cost(const double (&xb)[4], const double (&xt)[4], double xtw,
                                               const double (&ub)[NU]) const {
    const double e0 = P.tgt0 - fma(-xtw, xt[0], xb[0]);
    const double e1 = P.tgt1 - fma(-xtw, xt[1], xb[1]);
    double uu;
    if constexpr (NU == 2) uu = ub[0] * ub[0] + ub[NU - 1] * ub[NU - 1];
    else uu = ub[0] * ub[0];
    return (e0 * e0 + e1 * e1) + uu;
  }
  // final_cost(x̄_N) on the raw state (:192; 2_link_helper_functions.jl:100-108)
  __device__ __forceinline__ double final_cost(const double (&xb)[4]) const {
    const double f0 = P.tgt0 - xb[0], f1 = P.tgt1 - xb[1];
    return f0 * f0 + f1 * f1;
  }
};

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------

// four trajectories per wave, four waves per workgroup
constexpr int TL_BW4_WAVES = 4;
template <int NU>
__global__ __launch_bounds__(64 * TL_BW4_WAVES) void tl_backward_kernel(TwoLinkParams P, int B, int T,
                                                                      const double* __restrict__ x,
                                                                      const double* __restrict__ J,
                                                                      double* __restrict__ d,
                                                                      double* __restrict__ K,
                                                                      int32_t* __restrict__ status,
                                                                      double mu) {
  __shared__ double lds[TL_BW4_WAVES * 64];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * TL_BW4_WAVES + w) * 4;
  if (b0 >= B) return;
  const unsigned nan = tl_backward4_wave<NU>(P, b0, B, 0xFu, T, x, J, d, K, mu, lds + w * 64);
  const int l = threadIdx.x & 63;
  if (status && l < 4 && b0 + l < B) status[b0 + l] = ((nan >> l) & 1u) ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

// L = 4 line-search candidates per trajectory up to B = 65536, one lane per trajectory
// past it. At B = 1024 the candidate lanes sit on otherwise idle SIMDs (trial 1: 28.0
// vs 27.6 µs; trials 1-4: 61.9 vs 143.5 µs, nu = 1, T = 50); at B = 65536, where one
// lane per trajectory already fills every SIMD, the candidates' extra waves still hide
// latency (236 vs 275 µs; profiles/r02/tl_fw_probe.log). W waves per workgroup: 1 for
// the candidate grids (four 1-lane waves on one CU at B = 1024 ran 27.6 → 54.7 µs), 4
// past B = 65536 (1-wave workgroups past 256 waves were packed two to a SIMD).
inline int tl_fw_lanes(int B, bool wide = false) { return fg_lanes(B, wide); }

template <int NU, int L, int W>
__global__ __launch_bounds__(64 * W) void tl_forward_kernel(
    TwoLinkParams P, int B, int T, const double* __restrict__ x, const double* __restrict__ u,
    const double* __restrict__ xtraj, const double* __restrict__ d, const double* __restrict__ K,
    const double* __restrict__ prev_cost, double* __restrict__ xnew, double* __restrict__ unew,
    double* __restrict__ new_cost, int32_t* __restrict__ trials, int32_t* __restrict__ status,
    LSParams ls) {
  const int b = (blockIdx.x * 64 * W + threadIdx.x) / L;  // a group of L lanes per trajectory
  if (b >= B) return;
  const double pc = prev_cost ? prev_cost[b] : INFINITY;
  const TwoLinkModel<NU> m{P, tl_roll_consts(P)};
  const FgOut<double> r = fwd_group<TwoLinkModel<NU>, L>(m, b, B, T, x, u, xtraj, d, K, pc, xnew, unew, ls);
  if (!r.owner) return;
  if (!r.accepted) {  // exhausted (the reference would loop forever): return the inputs
    for (int i = 0; i < (T + 1) * TL_NX; ++i) xnew[(size_t)b * (T + 1) * TL_NX + i] = x[(size_t)b * (T + 1) * TL_NX + i];
    for (int i = 0; i < T * NU; ++i) unew[(size_t)b * T * NU + i] = u[(size_t)b * T * NU + i];
  }
  new_cost[b] = r.cost;
  if (trials) trials[b] = r.trials;
  if (status) status[b] = r.accepted ? ILQR_TRAJ_OK
                                     : (r.cost != r.cost ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED);
}

// One fit iteration (forward_pass.jl:161-176): backward part (after tl_linearize),
// slots whose status is not OK computed on and never stored.
template <int NU>
__global__ __launch_bounds__(64 * TL_BW4_WAVES) void tl_iter_backward_kernel(TwoLinkParams P, int B, int T,
                                                                           IterArgs a, const double* J,
                                                                           double mu) {
  __shared__ double lds[TL_BW4_WAVES * 64];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * TL_BW4_WAVES + w) * 4;
  if (b0 >= B) return;
  unsigned active = 0;
  for (int q = 0; q < 4; ++q)
    if (b0 + q < B && a.status[b0 + q] == ILQR_TRAJ_OK) active |= 1u << q;
  if (active == 0) return;
  const unsigned nan = tl_backward4_wave<NU>(P, b0, B, active, T, a.x, J, a.d, a.K, mu, lds + w * 64) & active;
  const int l = threadIdx.x & 63;
  if (l < 4 && ((nan >> l) & 1u)) {
    a.status[b0 + l] = ILQR_TRAJ_NAN;  // reference: AssertionError at backward_pass.jl:353
    if (a.res_parity) a.res_parity[b0 + l] = a.parity;
  }
}

// Forward part + the convergence test (:163-175).
template <int NU, int L, int W>
__global__ __launch_bounds__(64 * W) void tl_iter_forward_kernel(TwoLinkParams P, int B, int T,
                                                                 IterArgs a, LSParams ls) {
  const int b = (blockIdx.x * 64 * W + threadIdx.x) / L;
  if (b >= B || a.status[b] != ILQR_TRAJ_OK) return;
  const double pc = a.prev_cost ? a.prev_cost[b] : INFINITY;
  const TwoLinkModel<NU> m{P, tl_roll_consts(P)};
  const FgOut<double> r = fwd_group<TwoLinkModel<NU>, L>(m, b, B, T, a.x, a.u, a.xtraj, a.d, a.K, pc, a.xnew,
                                                          a.unew, ls, a.res_parity == nullptr);
  if (!r.owner) return;
  if (a.trials) a.trials[b] = r.trials;
  if (a.du2) a.du2[b] = r.du2;
  if (a.iters) a.iters[b] = a.iter;
  if (!r.accepted) {
    a.status[b] = (r.cost != r.cost) ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED;
    if (a.res_parity) a.res_parity[b] = a.parity;
  } else {
    a.new_cost[b] = r.cost;  // prev_cost = new_cost (:168)
    if (r.du2 <= ls.tol) {   // (:171) break BEFORE the update → result is the input iterate
      a.status[b] = ILQR_TRAJ_CONVERGED;
      if (a.res_parity) a.res_parity[b] = a.parity;
    }
  }
}

}  // namespace

// ---------------------------------------------------------------------------
// Host side
// ---------------------------------------------------------------------------
TwoLinkParams two_link_params() {
#pragma clang fp contract(off)
  // test/2_link_example/2_link_helper_functions.jl:4-26, same expression order
  const double l1 = sqrt(2.) / 2., l2 = sqrt(2.) / 2.;
  const double r1 = 0.5 * l1, r2 = 0.5 * l2;
  const double m1 = 1.0, m2 = 1.0;
  const double Iz1 = 1.0 / 12.0 * m1 * (l1 * l1), Iz2 = 1.0 / 12.0 * m2 * (l2 * l2);
  TwoLinkParams P;
  P.alpha = Iz1 + Iz2 + m1 * (r1 * r1) + m2 * (l1 * l1 + r2 * r2);
  P.beta = m2 * l1 * r2;
  P.delta = Iz2 + m2 * (r2 * r2);
  P.dt = 0.01;
  const double tx = 0.6, ty = -0.5;  // target_tool_loc (:16)
  const double q2 = acos((tx * tx + ty * ty - l1 * l1 - l2 * l2) / (2 * l1 * l2));
  const double q1 = atan2(ty, tx) - atan2(l2 * sin(q2), l1 + l2 * cos(q2));
  P.tgt0 = q1;
  P.tgt1 = q2;
  return P;
}

bool tl_supported(int nx, int nu) { return nx == TL_NX && (nu == 1 || nu == 2); }

size_t tl_workspace_doubles(int B, int T) { return (size_t)T * TL_NJR_MAX * B; }

namespace {
template <int NU>
hipError_t tl_backward_nu(const TwoLinkParams& P, int B, int T, const double* x, const double* u,
                          double* J, double* d, double* K, int32_t* status, double mu, hipStream_t s) {
  tl_linearize_kernel<NU><<<dim3((B + 255) / 256, T), 256, 0, s>>>(P, B, T, x, u, nullptr, J);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int per_wg = 4 * TL_BW4_WAVES;
  tl_backward_kernel<NU><<<(B + per_wg - 1) / per_wg, 64 * TL_BW4_WAVES, 0, s>>>(P, B, T, x, J, d, K, status, mu);
  return hipGetLastError();
}

// the forward's buffer resources span one wave's trajectories: 64 · (T+1) · 32 bytes
// below 2³¹ (the out-of-range offset that drops a store)
inline bool tl_fw_fits(int T) { return fg_fits<double>(T); }

template <int NU>
hipError_t tl_forward_nu(const TwoLinkParams& P, int B, int T, const double* x, const double* u,
                         const double* xtraj, const double* d, const double* K,
                         const double* prev_cost, double* xnew, double* unew, double* new_cost,
                         int32_t* trials, int32_t* status, const LSParams& ls, hipStream_t s) {
  if (!tl_fw_fits(T)) return hipErrorInvalidValue;
  const int L = tl_fw_lanes(B);
  if (L == 32)
    tl_forward_kernel<NU, 32, 1><<<(32 * B + 63) / 64, 64, 0, s>>>(
        P, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls);
  else if (L == 4)
    tl_forward_kernel<NU, 4, 1><<<(4 * B + 63) / 64, 64, 0, s>>>(
        P, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls);
  else
    tl_forward_kernel<NU, 1, 4><<<(B + 255) / 256, 256, 0, s>>>(
        P, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls);
  return hipGetLastError();
}

template <int NU>
hipError_t tl_iteration_nu(const TwoLinkParams& P, int B, int T, const IterArgs& a, double* J,
                           const LSParams& ls, hipStream_t s) {
  if (!tl_fw_fits(T)) return hipErrorInvalidValue;
  tl_linearize_kernel<NU><<<dim3((B + 255) / 256, T), 256, 0, s>>>(P, B, T, a.x, a.u, a.status, J);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int per_wg = 4 * TL_BW4_WAVES;
  tl_iter_backward_kernel<NU><<<(B + per_wg - 1) / per_wg, 64 * TL_BW4_WAVES, 0, s>>>(P, B, T, a, J, ls.mu);
  if ((e = hipGetLastError()) != hipSuccess) return e;
  const int L = tl_fw_lanes(B, a.iter >= 2);  // a fit past its first iteration
  if (L == 32)
    tl_iter_forward_kernel<NU, 32, 1><<<(32 * B + 63) / 64, 64, 0, s>>>(P, B, T, a, ls);
  else if (L == 4)
    tl_iter_forward_kernel<NU, 4, 1><<<(4 * B + 63) / 64, 64, 0, s>>>(P, B, T, a, ls);
  else
    tl_iter_forward_kernel<NU, 1, 4><<<(B + 255) / 256, 256, 0, s>>>(P, B, T, a, ls);
  return hipGetLastError();
}
}  // namespace

hipError_t launch_tl_backward(const TwoLinkParams& P, int nu, int B, int T, const double* x,
                              const double* u, double* J, double* d, double* K, int32_t* status,
                              double mu, hipStream_t s) {
  return nu == 1 ? tl_backward_nu<1>(P, B, T, x, u, J, d, K, status, mu, s)
                 : tl_backward_nu<2>(P, B, T, x, u, J, d, K, status, mu, s);
}

hipError_t launch_tl_forward(const TwoLinkParams& P, int nu, int B, int T, const double* x,
                             const double* u, const double* xtraj, const double* d,
                             const double* K, const double* prev_cost, double* xnew,
                             double* unew, double* new_cost, int32_t* trials, int32_t* status,
                             const LSParams& ls, hipStream_t s) {
  return nu == 1 ? tl_forward_nu<1>(P, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls, s)
                 : tl_forward_nu<2>(P, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls, s);
}

hipError_t launch_tl_jacobian(const TwoLinkParams& P, int nu, int B, int T, const double* x,
                              const double* u, double* A, double* Bm, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const dim3 g((B + 255) / 256, T < 65535 ? T : 65535);
  if (nu == 1)
    tl_jacobian_kernel<1><<<g, 256, 0, s>>>(P, B, T, x, u, A, Bm);
  else
    tl_jacobian_kernel<2><<<g, 256, 0, s>>>(P, B, T, x, u, A, Bm);
  return hipGetLastError();
}

hipError_t launch_tl_iteration(const TwoLinkParams& P, int nu, int B, int T, const IterArgs& a,
                               double* J, const LSParams& ls, hipStream_t s) {
  return nu == 1 ? tl_iteration_nu<1>(P, B, T, a, J, ls, s) : tl_iteration_nu<2>(P, B, T, a, J, ls, s);
}

}  // namespace ilqr
