// MI355X (gfx950) kernels for the batched iLQR hot path, LQ problem family.
//
// Reference path (aabouman/iLQR.jl): backward_pass (src/backward_pass.jl:324-357,
// with linearize_dynamics :25-40, immediate_cost_quadratization :81-109,
// final_cost_quadratization :134-153, optimal_controller_param :177-186,
// feedback_parameters :207-218, step_back :262-273) and forward_pass + line
// search (src/forward_pass.jl:55-93, total_cost :182-196), one iteration of
// fit (src/forward_pass.jl:161-176).
//
// Mapping:
//  * backward: ONE WAVE PER TRAJECTORY. The value-function state is kept in the
//    accumulator layout of v_mfma_f64_16x16x4_f64 as the symmetric 16×16 tile
//        Sp = [[S, s], [sᵀ, 0]]      (rows/cols ≥ nx+1 zero)
//    lane l = (c = l&15, q = l>>4) holds Sp[q+4r][c] in register r. Because Sp is
//    symmetric, that same register is the MFMA A-operand fragment of Sp, so the
//    recursion never leaves registers:
//        Y  = Sp·F          F = [A | B]  (nx × (nx+nu), zero-padded)   ceil(nx/4) MFMAs
//        Z  = L + Fᵀ·Y      L = blockdiag(Q+Qᵀ, R+Rᵀ)                  ceil(nx/4) MFMAs
//    Z holds Qxx (= lxx + AᵀSA), G = BᵀSA (+lux = 0) and H = luu + BᵀSB; row nx of
//    Y is sᵀF, giving g = lu + Bᵀs and lx + Aᵀs. The nu×nu solve (H + μI)⁻¹
//    (LDLᵀ, redundantly in every lane) yields K_aug = [K | d]. The reference's
//    step_back (:268-270) with G = -H_reg K, g = -H_reg d simplifies exactly to
//        [S s] = [Qxx  lx+Aᵀs] - K_augᵀ (H + 2μI) K_aug
//    which is ONE more MFMA (k = nu ≤ 4) with A = -K_augᵀ, B = (H+2μI)K_aug
//    = -[G|g] + μ K_aug, accumulating into [Qxx | lx+Aᵀs].
//  * forward: 16 lanes per trajectory (4 trajectories per wave, one DPP row each);
//    lane j < nx owns x̄_j, lanes nx.. own ū; mat-vecs broadcast the distributed
//    vector with v_fmac_f64_dpp row_newbcast, inputs prefetched 4 steps ahead.
//  * one fit iteration = backward launch (4 waves/SIMD) + forward launch; the ABI
//    pipelines them over two batch chunks on two streams (ilqr_abi.cpp).
#include <hip/hip_runtime.h>
#include <math.h>

#include "ilqr_internal.h"
#include "ilqr_device.h"
#include "ilqr_fwd_ring.h"
#include "../../include/ilqr.h"

namespace ilqr {
namespace {

// ---------------------------------------------------------------------------
// Backward pass of one trajectory by one wave (backward_pass.jl:324-357).
// Writes d (T,NU) and K (T,NU,NX) of trajectory b. Returns true if any gain is NaN
// (the reference's @assert !any(isnan, δu/K), :353-354).
// ---------------------------------------------------------------------------
// (Measured variants — Y/Z on the VALU, a Schur-complement or cofactor gain solve, two
// Newton steps per reciprocal, other symmetrisation periods, the round-1 gradient and
// gain stores — and tools/ablate_bw.hip's ablation bits live in
// tools/ablation/restore_alternates.patch)
template <int NX, int NU>
__device__ bool lq_backward_wave(const LQParams& P, int b, int T, const double* __restrict__ x,
                                 const double* __restrict__ u, double* __restrict__ d_out,
                                 double* __restrict__ K_out, double mu, double* lds) {
  static_assert(NX + NU <= 16 && NX < 16 && NU <= 4, "MFMA tile mapping needs nx+nu <= 16, nu <= 4");
  constexpr int KS = (NX + 3) / 4;  // k-steps of 4 over the state dimension
  constexpr int SROW = NX;          // row/column of Sp holding s
  b = __builtin_amdgcn_readfirstlane(b);  // one trajectory per wave: keep its pointers scalar
  const int l = threadIdx.x & 63;
  const int c = l & 15;
  const int q = l >> 4;
  const bool cx = c < NX;                  // state column
  const bool cu = c >= NX && c < NX + NU;  // input column
  const int ci = cx ? c : 0;
  const int cj = cu ? c - NX : 0;

  const double* Ab = P.A + (size_t)b * NX * NX;
  const double* Bb = P.B + (size_t)b * NX * NU;
  const double* Qb = P.Q + (size_t)b * NX * NX;
  const double* Rb = P.R + (size_t)b * NU * NU;
  const double* Qfb = P.Qf + (size_t)b * NX * NX;

  // F fragments (A- and B-operand of the same MFMA family): fB[kk] = F[4kk+q][c], F = [A | B]
  double fB[KS];
#pragma unroll
  for (int kk = 0; kk < KS; ++kk) {
    const int i = 4 * kk + q;
    const bool ri = i < NX;
    const int ii = ri ? i : 0;
    const double a = ldz(ri && cx, Ab + ii * NX + ci, Ab);
    const double bb = ldz(ri && cu, Bb + ii * NU + cj, Bb);
    fB[kk] = a + bb;
  }
  // Cost Hessian L = blockdiag(Q+Qᵀ, R+Rᵀ) in accumulator layout: Lc[r] = L[q+4r][c]
  // (immediate_cost_quadratization :101-106 of ℓ = xᵀQx + uᵀRu: 𝐐 = Q+Qᵀ, 𝐑 = R+Rᵀ, 𝐏 = 0)
  d4 Lc;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int i = q + 4 * r;
    const bool rx = i < NX, ru = i >= NX && i < NX + NU;
    const int ix = rx ? i : 0, iu = ru ? i - NX : 0;
    const double lq = ldz(rx && cx, Qb + ix * NX + ci, Qb) + ldz(rx && cx, Qb + ci * NX + ix, Qb);
    const double lr = ldz(ru && cu, Rb + iu * NU + cj, Rb) + ldz(ru && cu, Rb + cj * NU + iu, Rb);
    Lc[r] = lq + lr;
  }

  double* Gl = lds;       // Gl[j*16 + c] = Z[NX+j][c]   (j < NU): [G | H] rows
  double* gl = lds + 64;  // gl[c] = (L z + Fᵀ s)[c]:   [lx + Aᵀs | lu + Bᵀs]
  constexpr int ZERO = 80;  // a slot holding 0.0: lanes with nothing to read read it
  lds[ZERO] = 0.0;
  // per-lane LDS addresses of the hand-off reads (branch-free: one ds_read each)
  int col_at[NU];
#pragma unroll
  for (int j = 0; j < NU; ++j) col_at[j] = cx ? j * 16 + c : (c == SROW ? 64 + NX + j : ZERO);
  const int qq = q < NU ? q : 0;
  const int colq_at = cx ? qq * 16 + c : (c == SROW ? 64 + NX + qq : ZERO);
  int qv_at[KS];
#pragma unroll
  for (int r = 0; r < KS; ++r) qv_at[r] = (c == SROW && q + 4 * r < NX) ? 64 + q + 4 * r : ZERO;
  // Terminal value function (final_cost_quadratization :134-153, ℓ_f = xᵀQf x):
  // S = Qf+Qfᵀ, s = (Qf+Qfᵀ) x_N.
  const double* xN = x + ((size_t)b * (T + 1) + T) * NX;
  d4 Sp;
  {
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      const bool rx = i < NX;
      const int ix = rx ? i : 0;
      const double v = ldz(rx && cx, Qfb + ix * NX + ci, Qfb) + ldz(rx && cx, Qfb + ci * NX + ix, Qfb);
      Sp[r] = v;
      part = fma(v, ldz(rx, xN + ix, xN), part);
    }
    const double sc = colsum4(part);  // s[c] for c < NX
    if (q == 0) gl[c] = sc;
    wave_lds_fence();
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      const double sv = gl[i < NX ? i : 0];
      if (c == SROW && i < NX) Sp[r] = sv;
    }
    wave_lds_fence();
  }

  bool nan = false;
  // gradient operands z = [x_t; u_t] at rows q+4r, prefetched one step ahead
  auto load_z = [&](int t) {
    const double* xt = x + ((size_t)b * (T + 1) + t) * NX;
    const double* ut = u + ((size_t)b * T + t) * NU;
    d4 z;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      const bool rx = i < NX, ru = i >= NX && i < NX + NU;
      const double* p = rx ? xt + i : (ru ? ut + (i - NX) : xt);
      const double v = *p;
      z[r] = (rx || ru) ? v : 0.0;
    }
    return z;
  };
  d4 zc = load_z(T - 1);
  double* Kb = K_out + (size_t)b * T * NU * NX;
  double* db = d_out + (size_t)b * T * NU;
  // gains go out through raw buffer stores (inactive lanes dropped, no exec branch)
  const auto rK = buffer_rsrc(Kb, (uint32_t)(T * NU * NX * 8));
  const auto rD = buffer_rsrc(db, (uint32_t)(T * NU * 8));
  constexpr int JUNK = 96 + 16 * 17;  // LDS row the lanes without a g value write to

  for (int t = T - 1; t >= 0; --t) {
    const d4 zn = load_z(t > 0 ? t - 1 : 0);

    // Y = Sp · F (optimal_controller_param's S'A, S'B and the row sᵀF)
    // Z = L + Fᵀ Y = [[lxx + AᵀSA, AᵀSB], [BᵀSA, luu + BᵀSB]]  (:182-183, first terms of :270)
    d4 Y = {0.0, 0.0, 0.0, 0.0};
    d4 Z = Lc;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) Y = mfma(Sp[kk], fB[kk], Y);
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) Z = mfma(fB[kk], Y[kk], Z);

    // gq[c] = (L z)[c] + (Fᵀ s)[c]: lx + Aᵀs (c < NX), g = lu + Bᵀs (c ≥ NX)  (:181, :269).
    // (L z)[c] does not depend on the recursion: its 4-lane reduction overlaps the
    // MFMAs; (Fᵀ s)[c] = Y[SROW][c] sits in lane q = SROW%4 only, which alone
    // publishes g (the other lanes write a junk LDS row), so no reduction waits on Y.
    double part = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) part = fma(Lc[r], zc[r], part);
    const double gq = colsum4(part) + Y[SROW / 4];  // exact in lane q = SROW%4

    // hand the NU rows [G | H] and g to every lane
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = q + 4 * r;
      if (i >= NX && i < NX + NU) Gl[(i - NX) * 16 + c] = Z[r];
    }
    lds[(q == SROW % 4) ? 64 + c : JUNK + l] = gq;
    double h[NU][NU];
    d4 col = {0.0, 0.0, 0.0, 0.0};
    double qv[KS];
    wave_lds_fence();
#pragma unroll
    for (int i = 0; i < NU; ++i)
#pragma unroll
      for (int k = 0; k <= i; ++k) h[i][k] = Gl[i * 16 + NX + k];
#pragma unroll
    for (int j = 0; j < NU; ++j) col[j] = lds[col_at[j]];     // [G | g][j][c], 0 for c > NX
    const double colq = lds[colq_at];                         // [G | g][q][c]
#pragma unroll
    for (int r = 0; r < KS; ++r) qv[r] = lds[qv_at[r]];       // (lx + Aᵀs)[q+4r] in column NX
    wave_lds_fence();

    // feedback_parameters (:207-218): K_aug[:,c] = -(H + μI)⁻¹ [G | g][:,c]
    LDLT<NU, 1> f;
    f.factor(h, mu);
    const double sol = f.solve(col)[qq];  // ((H + μI)⁻¹ [G | g])[q][c]
    const double kq = (q < NU) ? -sol : 0.0;              // K_aug[q][c]
    const double wk = (q < NU) ? fma(mu, kq, -colq) : 0.0;   // ((H + 2μI) K_aug)[q][c]
    nan |= __builtin_isnan(kq);

    store_or_drop(kq, rK, q < NU && cx, (uint32_t)(((t * NU + qq) * NX + ci) * 8));
    store_or_drop(kq, rD, q < NU && c == SROW, (uint32_t)((t * NU + qq) * 8));

    // step_back (:269-270): Sp ← [Qxx | lx + Aᵀs] − K_augᵀ (H + 2μI) K_aug
    d4 Cin;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double v = 0.0;
      if (r < KS) v = cx ? Z[r] : qv[r];
      Cin[r] = (q + 4 * r < NX) ? v : 0.0;
    }
    Sp = mfma(-kq, wk, Cin);
    zc = zn;

    // S ← (S + Sᵀ)/2 on the state block (the identity in exact arithmetic). The
    // accumulator tile feeds the next Y MFMA as its own transpose, so rounding
    // asymmetry E evolves as E ← −AᵀEA and grows like ρ(A)^2t on unstable A;
    // a periodic projection bounds it at negligible cost.
    if ((t % SYM_EVERY) == 0) {
      double* tile = lds + 96;  // 16 × 17 (padded) doubles
#pragma unroll
      for (int r = 0; r < 4; ++r) tile[(q + 4 * r) * 17 + c] = Sp[r];
      wave_lds_fence();
#pragma unroll
      for (int r = 0; r < KS; ++r) {
        const int i = q + 4 * r;
        const double other = tile[c * 17 + (i < NX ? i : 0)];  // unconditional read
        const double avg = 0.5 * (Sp[r] + other);
        Sp[r] = (i < NX && cx) ? avg : Sp[r];
      }
      wave_lds_fence();
    }
  }
  return __any(nan);
}

// ---------------------------------------------------------------------------
// Forward pass of up to 4 trajectories by one wave, 16 lanes each — one DPP row
// per trajectory (forward_pass.jl:55-93, total_cost :182-196). Lane j < nx owns
// x̄_j, lanes nx.. own ū. Mat-vecs broadcast the distributed vector with DPP
// (no LDS); per-step inputs are prefetched PF steps ahead into a register ring.
// ---------------------------------------------------------------------------
template <int NX>
struct FwdStepIn {
  double xr, xtr, ur, dr;  // xₖ[j], x_trajₖ[j] (x lanes); uₖ, δuₖ (u lanes)
  double Kr[NX];           // row of Kₖ (u lanes)
};

template <int NX, int NU, int PF = 2>  // PF: prefetch distance (steps)
__device__ FwdOut lq_forward_group(const LQParams& P, int b, int T, const double* __restrict__ x,
                                   const double* __restrict__ u, const double* __restrict__ xtraj,
                                   const double* __restrict__ dg, const double* __restrict__ Kg,
                                   double prev_cost, double* __restrict__ xnew,
                                   double* __restrict__ unew, double* du2_out,
                                   const LSParams& ls) {
  static_assert(NX + NU == 16, "one 16-lane DPP row per trajectory: nx + nu == 16");
  static_assert(NX == 12, "dpp_dot12 is the K·δx product");
  const int j = threadIdx.x & 15;
  const bool is_x = j < NX;
  const bool is_u = !is_x;
  const int iu = is_u ? j - NX : 0;
  const int jx = is_x ? j : 0;

  const double* Ab = P.A + (size_t)b * NX * NX;
  const double* Bb = P.B + (size_t)b * NX * NU;
  const double* Qb = P.Q + (size_t)b * NX * NX;
  const double* Rb = P.R + (size_t)b * NU * NU;
  const double* Qfb = P.Qf + (size_t)b * NX * NX;

  // row j of F = [A B] (lanes j < NX) and of L = blockdiag(Q, R) (ℓ = vᵀ L v)
  double Fr[16], Lr[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double a = ldz(is_x && k < NX, Ab + jx * NX + (k < NX ? k : 0), Ab);
    const double bb = ldz(is_x && k >= NX, Bb + jx * NU + (k >= NX ? k - NX : 0), Bb);
    Fr[k] = a + bb;
    const double lq = ldz(is_x && k < NX, Qb + jx * NX + (k < NX ? k : 0), Qb);
    const double lr = ldz(is_u && k >= NX, Rb + iu * NU + (k >= NX ? k - NX : 0), Rb);
    Lr[k] = lq + lr;
  }

  const double* xb0 = x + (size_t)b * (T + 1) * NX;
  const double* ub0 = u + (size_t)b * T * NU;
  // x_traj = NULL means zeros: read x itself with weight 0 (no branch around the load,
  // which would make the compiler drain every prefetch with vmcnt(0))
  const double* xt0 = (xtraj ? xtraj : x) + (size_t)b * (T + 1) * NX;
  const double xtw = xtraj ? 1.0 : 0.0;
  const double* d0 = dg + (size_t)b * T * NU;
  const double* K0 = Kg + (size_t)b * T * NU * NX;
  // each lane stores one element per step: x̄ₖ[j] (x lanes) or ūₖ[iu] (u lanes)
  double* const out0 = is_x ? xnew + (size_t)b * (T + 1) * NX + jx : unew + (size_t)b * T * NU + iu;
  const int out_stride = is_x ? NX : NU;

  auto load = [&](int t, FwdStepIn<NX>& in) {
    const int tt = t < T ? t : T - 1;  // clamped: loads past the horizon are discarded
    in.xr = xb0[(size_t)tt * NX + jx];
    in.xtr = xt0[(size_t)tt * NX + jx];
    in.ur = ub0[(size_t)tt * NU + iu];
    in.dr = d0[(size_t)tt * NU + iu];
    const double2* kr = reinterpret_cast<const double2*>(K0 + ((size_t)tt * NU + iu) * NX);
#pragma unroll
    for (int k = 0; k < NX / 2; ++k) {
      const double2 v = kr[k];
      in.Kr[2 * k] = v.x;
      in.Kr[2 * k + 1] = v.y;
    }
  };

  double alpha = ls.alpha0;
  FwdOut out{0.0, 0, 0};
  double du2 = 0.0;
  for (int trial = 1; trial <= ls.max_trials; ++trial) {
    double xb = is_x ? xb0[jx] : 0.0;  // x̄₁ = x₁ (:65)
    double cost = 0.0;
    du2 = 0.0;
    FwdStepIn<NX> ring[PF];
#pragma unroll
    for (int s = 0; s < PF; ++s) load(s, ring[s]);
    auto step = [&](int t, FwdStepIn<NX>& in) {
      // δx = x̄ₖ − xₖ (:72); ūₖ = uₖ + α δuₖ + Kₖ δx (:73), α scales δu only
      const double dx = is_x ? xb - in.xr : 0.0;
      const double kdx = dpp_dot12(dx, in.Kr);
      const double ub = fma(alpha, in.dr, in.ur) + kdx;
      const double z = is_x ? xb : ub;
      const double v = is_x ? fma(-xtw, in.xtr, xb) : ub;
      const double e = is_x ? 0.0 : ub - in.ur;
      load(t + PF, in);  // refill this slot PF steps ahead
      // ℓ(x̄ₖ − x_trajₖ, ūₖ) (:187-190) and x̄ₖ₊₁ = f(x̄ₖ, ūₖ) = A x̄ₖ + B ūₖ (:74)
      const double lv = dpp_dot16(v, Lr);
      const double xn = dpp_dot16(z, Fr);
      cost = fma(v, lv, cost);
      out0[(size_t)t * out_stride] = z;
      du2 = fma(e, e, du2);
      xb = xn;
    };
    const int Tm = T - T % PF;
    for (int t0 = 0; t0 < Tm; t0 += PF) {
#pragma unroll
      for (int s = 0; s < PF; ++s) step(t0 + s, ring[s]);
    }
#pragma unroll
    for (int s = 0; s < PF - 1; ++s)
      if (Tm + s < T) step(Tm + s, ring[s]);
    // final cost ℓ_f(x̄_N) on the raw state (:192)
    if (is_x) xnew[(size_t)b * (T + 1) * NX + (size_t)T * NX + j] = xb;
    double Qfr[NX];
#pragma unroll
    for (int k = 0; k < NX; ++k) Qfr[k] = ldz(is_x, Qfb + jx * NX + k, Qfb);
    const double lf = dpp_dot12(is_x ? xb : 0.0, Qfr);
    cost = fma(is_x ? xb : 0.0, lf, cost);
    cost = rowsum16(cost);
    out.trials = trial;
    out.cost = cost;
    if (prev_cost - cost > 0.0) {  // (:77-80); NaN compares false → keep searching
      out.accepted = 1;
      break;
    }
    alpha *= ls.shrink;  // (:82)
  }
  if (du2_out) *du2_out = rowsum16(du2);
  return out;
}

// ---------------------------------------------------------------------------
// Kernels
// ---------------------------------------------------------------------------
template <int NX, int NU>
__global__ __launch_bounds__(256, 4) void lq_backward_kernel(LQParams P, int B, int T,
                                                          const double* __restrict__ x,
                                                          const double* __restrict__ u,
                                                          double* __restrict__ d,
                                                          double* __restrict__ K,
                                                          int32_t* __restrict__ status, double mu) {
  __shared__ __attribute__((aligned(16))) double lds[WAVES_PER_WG * BW_LDS];
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.x * WAVES_PER_WG + w;
  if (b >= B) return;
  const bool nan = lq_backward_wave<NX, NU>(P, b, T, x, u, d, K, mu, lds + w * BW_LDS);
  if (status && (threadIdx.x & 63) == 0) status[b] = nan ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

template <int NX, int NU>
__global__ __launch_bounds__(64) void lq_forward_kernel(
    LQParams P, int B, int T, const double* __restrict__ x, const double* __restrict__ u,
    const double* __restrict__ xtraj, const double* __restrict__ d, const double* __restrict__ K,
    const double* __restrict__ prev_cost, double* __restrict__ xnew, double* __restrict__ unew,
    double* __restrict__ new_cost, int32_t* __restrict__ trials, int32_t* __restrict__ status,
    LSParams ls) {
  const int g = threadIdx.x >> 4;
  const int j = threadIdx.x & 15;
  const int b = blockIdx.x * 4 + g;
  if (b >= B) return;  // whole 16-lane group: no cross-group LDS traffic
  const double pc = prev_cost ? prev_cost[b] : INFINITY;
  FwdOut r = lq_forward_group<NX, NU>(P, b, T, x, u, xtraj, d, K, pc, xnew, unew, nullptr, ls);
  if (!r.accepted) {
    // line search exhausted (the reference would loop forever): return the inputs.
    // Lanes of a group write disjoint elements; nothing reads them in this launch.
    for (int i = j; i < (T + 1) * NX; i += 16) xnew[(size_t)b * (T + 1) * NX + i] = x[(size_t)b * (T + 1) * NX + i];
    for (int i = j; i < T * NU; i += 16) unew[(size_t)b * T * NU + i] = u[(size_t)b * T * NU + i];
  }
  if (j == 0) {
    new_cost[b] = r.cost;
    if (trials) trials[b] = r.trials;
    if (status) status[b] = r.accepted ? ILQR_TRAJ_OK
                                       : (r.cost != r.cost ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED);
  }
}

// One fit iteration (forward_pass.jl:161-176), part 1: backward_pass for every
// trajectory whose status is OK (4 waves / workgroup, one trajectory per wave).
template <int NX, int NU>
__global__ __launch_bounds__(256, 4) void lq_iter_backward_kernel(LQParams P, int B, int T, IterArgs a,
                                                               double mu) {
  __shared__ __attribute__((aligned(16))) double lds[WAVES_PER_WG * BW_LDS];
  const int w = threadIdx.x >> 6;
  const int b = blockIdx.x * WAVES_PER_WG + w;
  if (b >= B || a.status[b] != ILQR_TRAJ_OK) return;
  const bool nan = lq_backward_wave<NX, NU>(P, b, T, a.x, a.u, a.d, a.K, mu, lds + w * BW_LDS);
  if (nan && (threadIdx.x & 63) == 0) {
    a.status[b] = ILQR_TRAJ_NAN;  // reference: AssertionError at backward_pass.jl:353
    if (a.res_parity) a.res_parity[b] = a.parity;
  }
}

// Part 2: forward_pass + line search + the convergence test (:163-175), four
// trajectories per wave. The backward and forward are separate launches so the
// backward keeps its 4 waves/SIMD register budget (≤128 VGPRs).
template <int NX, int NU>
__global__ __launch_bounds__(64) void lq_iter_forward_kernel(LQParams P, int B, int T, IterArgs a,
                                                             LSParams ls) {
  const int g = threadIdx.x >> 4;
  const int j = threadIdx.x & 15;
  const int b = blockIdx.x * 4 + g;
  if (b >= B || a.status[b] != ILQR_TRAJ_OK) return;
  double du2 = 0.0;
  const double pc = a.prev_cost ? a.prev_cost[b] : INFINITY;
  const FwdOut r = lq_forward_group<NX, NU>(P, b, T, a.x, a.u, a.xtraj, a.d, a.K, pc,
                                            a.xnew, a.unew, &du2, ls);
  if (j == 0) {
    if (a.trials) a.trials[b] = r.trials;
    if (a.du2) a.du2[b] = du2;
    if (a.iters) a.iters[b] = a.iter;
    if (!r.accepted) {
      a.status[b] = (r.cost != r.cost) ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED;
      if (a.res_parity) a.res_parity[b] = a.parity;
    } else {
      a.new_cost[b] = r.cost;  // @assert(prev_cost > new_cost); prev_cost = new_cost (:168)
      if (du2 <= ls.tol) {      // (:171) break BEFORE the update → result is the input iterate
        a.status[b] = ILQR_TRAJ_CONVERGED;
        if (a.res_parity) a.res_parity[b] = a.parity;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Pipelined fit iteration (DESIGN.md §fit driver): the backward pass is bound by the
// FP64 pipe and the forward pass by HBM, so one launch runs both at once on
// different trajectories. Workgroups (4 trajectories each) have one of two roles:
//   role B: backward(iteration i) → barrier → wave 0: forward(iteration i)
//   role A: wave 0: forward(iteration i−1) → barrier → backward(iteration i)
// so while B's waves run Riccati recursions, A's first waves stream their forward
// passes, and vice versa at the end of the launch. `cur` describes iteration i
// (B, and A's backward), `prev` iteration i−1 (A's forward, which reads the gains
// A's backward wrote in the previous launch). fit runs max_iter + 1 launches: the
// first without A's forward, the last with A's forward only.
// ---------------------------------------------------------------------------
constexpr int PIPE_LDS = (PIPE_R * RING_SLOT + RING_LAREA > WAVES_PER_WG * BW_LDS)
                             ? PIPE_R * RING_SLOT + RING_LAREA : WAVES_PER_WG * BW_LDS;
enum : int { PIPE_A_FW = PIPE_A_FW_FLAG, PIPE_A_BW = PIPE_A_BW_FLAG, PIPE_B = PIPE_B_FLAG };

// role of workgroup g: two of the four workgroups each CU hosts at B = 4096 are A,
// whether the dispatcher spreads consecutive workgroups of an XCD over its CUs
// (CU mates g, g+256, g+512, g+768) or packs them (g, g+8, g+16, g+24)
__host__ __device__ __forceinline__ bool pipe_role_a(int g) { return (((g >> 8) ^ (g >> 3)) & 1) != 0; }

// forward_pass (the ilqr_forward entry) with the LDS-ring forward: every trajectory
// runs; an exhausted line search returns the inputs (as lq_forward_kernel).
// Four waves per workgroup, each with its own ring (116 KB of LDS: one workgroup per
// CU, one wave per SIMD); one-wave workgroups let the dispatcher pack two waves onto a
// SIMD (the fused kernel).
constexpr int FW_WAVES = 4;
template <int NX, int NU, bool MF = false>
__global__ __launch_bounds__(64 * FW_WAVES) void lq_forward_ring_kernel(
    LQParams P, int B, int T, const double* __restrict__ x, const double* __restrict__ u,
    const double* __restrict__ xtraj, const double* __restrict__ d, const double* __restrict__ K,
    const double* __restrict__ prev_cost, double* __restrict__ xnew, double* __restrict__ unew,
    double* __restrict__ new_cost, int32_t* __restrict__ trials, int32_t* __restrict__ status,
    LSParams ls) {
  __shared__ __attribute__((aligned(16))) double ring_all[FW_WAVES * (PIPE_R * RING_SLOT + RING_LAREA)];
  const int w = threadIdx.x >> 6;
  double* ring = ring_all + w * (PIPE_R * RING_SLOT + RING_LAREA);
  const int b0 = (blockIdx.x * FW_WAVES + w) * 4;
  if (b0 >= B) return;
  // the row form: trajectory of lane l = l >> 4, index j = l & 15 within it; the MFMA
  // form: trajectory (l >> 2) & 3, index 4ρ + κ
  const int l = threadIdx.x & 63;
  const int j = MF ? ((l >> 4) << 2) | (l & 3) : l & 15;
  const int b = b0 + (MF ? (l >> 2) & 3 : l >> 4);
  const bool active = b < B;
  const double pc = (prev_cost && active) ? prev_cost[b] : INFINITY;
  FwdOut r;
  if constexpr (MF)
    r = lq_forward_wave_mfma<PIPE_R, PIPE_PF>(P, b0, B, T, 0xFu, x, u, xtraj, d, K, pc, xnew, unew, nullptr, ls,
                                              ring);
  else
    r = lq_forward_wave_ring<NX, NU, PIPE_R, PIPE_PF>(P, b0, B, T, active, x, u, xtraj, d, K, pc, xnew, unew,
                                                      nullptr, ls, ring);
  if (!active) return;
  if (!r.accepted) {
    for (int i = j; i < (T + 1) * NX; i += 16) xnew[(size_t)b * (T + 1) * NX + i] = x[(size_t)b * (T + 1) * NX + i];
    for (int i = j; i < T * NU; i += 16) unew[(size_t)b * T * NU + i] = u[(size_t)b * T * NU + i];
  }
  if (j == 0) {
    new_cost[b] = r.cost;
    if (trials) trials[b] = r.trials;
    if (status) status[b] = r.accepted ? ILQR_TRAJ_OK
                                       : (r.cost != r.cost ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED);
  }
}

// Part 2 with the LDS-ring forward (one wave, four trajectories per workgroup).
template <int NX, int NU, bool MF = false>
__global__ __launch_bounds__(64 * FW_WAVES) void lq_iter_forward_ring_kernel(LQParams P, int B, int T,
                                                                            IterArgs a, LSParams ls) {
  __shared__ __attribute__((aligned(16))) double ring_all[FW_WAVES * (PIPE_R * RING_SLOT + RING_LAREA)];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * FW_WAVES + w) * 4;
  if (b0 >= B) return;
  double* ring = ring_all + w * (PIPE_R * RING_SLOT + RING_LAREA);
  if constexpr (MF) {
    unsigned run = 0;
    for (int q = 0; q < 4; ++q)
      if (b0 + q < B && a.status[b0 + q] == ILQR_TRAJ_OK) run |= 1u << q;
    iter_forward_wave_mfma(P, b0, B, T, a, ls, ring, run);
  } else {
    iter_forward_wave<NX, NU>(P, b0, B, T, a, ls, ring);
  }
}

template <int NX, int NU>
__global__ __launch_bounds__(256, 4) void lq_iter_pipe_kernel(LQParams P, int B, int T,
                                                              IterArgs cur, IterArgs prev,
                                                              LSParams ls, int flags) {
  __shared__ __attribute__((aligned(16))) double lds[PIPE_LDS];
  const int w = threadIdx.x >> 6;
  const int b0 = blockIdx.x * WAVES_PER_WG;
  const bool role_a = pipe_role_a(blockIdx.x);
  auto forward4 = [&](const IterArgs& a) {  // wave 0: the workgroup's 4 trajectories
    if (w == 0) iter_forward_wave<NX, NU, false>(P, b0, B, T, a, ls, lds);  // ring: the whole WG's scratch
  };
  auto backward = [&](const IterArgs& a) {
    const int b = b0 + w;
    if (b < B && a.status[b] == ILQR_TRAJ_OK) {
      const bool nan = lq_backward_wave<NX, NU>(P, b, T, a.x, a.u, a.d, a.K, ls.mu, lds + w * BW_LDS);
      if (nan && (threadIdx.x & 63) == 0) {
        a.status[b] = ILQR_TRAJ_NAN;  // reference: AssertionError at backward_pass.jl:353
        if (a.res_parity) a.res_parity[b] = a.parity;
      }
    }
  };
  if (role_a) {
    if (flags & PIPE_A_FW) forward4(prev);
    __syncthreads();  // x̄, ū and the status of iteration i−1 are visible to the workgroup
    if (flags & PIPE_A_BW) backward(cur);
  } else if (flags & PIPE_B) {
    backward(cur);
    __syncthreads();  // the gains of iteration i are visible to wave 0
    forward4(cur);
  }
}

// dst[0, n) = src[0, n) by one wave: eight loads per lane in flight before their stores
// (a load-store pair per element waits out the memory latency once per 64 elements)
__device__ inline void wave_copy(double* __restrict__ dst, const double* __restrict__ src, int n, int l) {
  for (int i0 = 0; i0 < n; i0 += 64 * 8) {
    double v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = i0 + j * 64 + l;
      if (i < n) v[j] = src[i];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int i = i0 + j * 64 + l;
      if (i < n) dst[i] = v[j];
    }
  }
}

// One wave per trajectory (four per block). The call status (bit 0 a NaN trajectory,
// bit 1 an exhausted line search) is OR-ed into a DEVICE word, dflags[0], with
// relaxed device-scope atomics (only by trajectories that set a bit);
// gather_flags_kernel, the next launch, copies it to `flags` (host-mapped, may be null)
// with one plain store and re-arms it — no device atomics on host memory (those need
// PCIe AtomicOps). A last-block ticket in this kernel instead (a release fence and an
// acq_rel agent-scope atomic per block: an L2 write-back each) cost 42 µs per fit at
// B = 4096 against ≈2 µs for the second launch.
__global__ __launch_bounds__(256) void gather_kernel(int B, int T, int nx, int nu, const double* xin,
                                                     const double* uin, const double* x0, const double* u0,
                                                     const double* x1, const double* u1,
                                                     const int32_t* res_parity, int32_t* status,
                                                     int final_parity, const double* fit_cost,
                                                     const int32_t* fit_iters, double* x_out, double* u_out,
                                                     double* cost_out, int32_t* iters_out,
                                                     int32_t* status_out, int32_t* dflags) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int l = threadIdx.x & 63;
  if (b < B) {
    const int32_t st0 = status[b];
    const bool running = st0 == ILQR_TRAJ_OK;
    const int par = running ? final_parity : res_parity[b];
    if (par != PARITY_OUT) {  // PARITY_OUT: the last iteration wrote x_out / u_out itself
      const double* xs = (par == PARITY_INPUT ? xin : (par ? x1 : x0)) + (size_t)b * (T + 1) * nx;
      const double* us = (par == PARITY_INPUT ? uin : (par ? u1 : u0)) + (size_t)b * T * nu;
      wave_copy(x_out + (size_t)b * (T + 1) * nx, xs, (T + 1) * nx, l);
      wave_copy(u_out + (size_t)b * T * nu, us, T * nu, l);
    }
    if (l == 0) {  // the lane that read status[b] is the one that rewrites it
      const int32_t st = running ? ILQR_TRAJ_MAX_ITER : st0;
      status[b] = st;
      if (status_out) status_out[b] = st;
      if (cost_out) cost_out[b] = fit_cost[b];
      if (iters_out) iters_out[b] = fit_iters[b];
      const int f = (st == ILQR_TRAJ_NAN ? 1 : 0) | (st == ILQR_TRAJ_LS_EXHAUSTED ? 2 : 0);
      if (f) __hip_atomic_fetch_or(dflags, f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// the gather's call-status word to the host-mapped `flags` (after gather_kernel on the
// same stream: its atomics are complete and visible at the kernel boundary), re-armed
// `seq` tags the host word (bits 2..31): the host knows the fit's last kernel ran when
// the word carries its fit's number (ilqr_fit_ex waits on it)
__global__ void gather_flags_kernel(int32_t* dflags, int32_t* flags, uint32_t seq) {
  const int32_t v = __hip_atomic_load(dflags, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (flags) *(volatile int32_t*)flags = (int32_t)((seq << 2) | ((uint32_t)v & 3u));
  __hip_atomic_store(dflags, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// linearize_dynamics of the LQ family (ilqr_linearize): f(x, u) = A x + B u is linear,
// so ∂f/∂x = A and ∂f/∂u = B at every (x_t, u_t) — the instance's matrix broadcast
// over the T steps, one thread per output element (coalesced stores; the E-element
// source block of a trajectory is read T times from cache)
__global__ void lq_broadcast_steps_kernel(const double* __restrict__ src, double* __restrict__ dst, int T,
                                          int E, size_t n) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const size_t per_traj = (size_t)T * E;
  const size_t b = i / per_traj;
  dst[i] = src[b * E + (i - b * per_traj) % E];
}

template <class V>
__global__ void record_history_kernel(int B, int stride, int it, const int32_t* __restrict__ status,
                                      const int32_t* __restrict__ iters, const int32_t* __restrict__ trials,
                                      const V* __restrict__ cost, const V* __restrict__ du2, V alpha0, V shrink,
                                      double* h_cost, int32_t* h_trials, double* h_alpha, double* h_du2) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const size_t o = (size_t)(it - 1) * stride + b;
  const bool ran = iters[b] == it;
  const int32_t st = status[b];
  const bool acc = ran && (st == ILQR_TRAJ_OK || st == ILQR_TRAJ_CONVERGED);
  const int n = ran ? trials[b] : 0;
  if (h_trials) h_trials[o] = n;
  if (h_cost) h_cost[o] = acc ? (double)cost[b] : (double)NAN;
  if (h_alpha) {
    V a = alpha0;  // the forward's repeated α *= shrink (forward_pass.jl:82)
    for (int k = 1; k < n; ++k) a *= shrink;
    h_alpha[o] = acc ? (double)a : (double)NAN;
  }
  if (h_du2) h_du2[o] = ran ? (double)du2[b] : (double)NAN;
}

__global__ void fit_init_kernel(int B, double* prev_cost, int32_t* status, int32_t* res_parity,
                                int32_t* iters) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  prev_cost[b] = INFINITY;
  status[b] = ILQR_TRAJ_OK;
  res_parity[b] = PARITY_INPUT;
  iters[b] = 0;
}

// one thread per destination element; consecutive threads → consecutive elements
__global__ void pad3_kernel(const double* __restrict__ src, double* __restrict__ dst, size_t total,
                            int R, int C, int R2, int C2) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C2);
  const size_t rr = i / C2;
  const int r = (int)(rr % R2);
  const size_t n = rr / R2;
  dst[i] = (r < R && c < C) ? src[(n * R + r) * C + c] : 0.0;
}
__global__ void unpad3_kernel(const double* __restrict__ src, double* __restrict__ dst, size_t total,
                              int R, int C, int R2, int C2) {
  const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int c = (int)(i % C);
  const size_t rr = i / C;
  const int r = (int)(rr % R);
  const size_t n = rr / R;
  dst[i] = src[(n * R2 + r) * C2 + c];
}

__global__ void fill_i32_kernel(int32_t* p, int n, int32_t v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}
__global__ void fill_f64_kernel(double* p, int n, double v) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = v;
}

// -------- self-test of the lane maps the kernels depend on -------------------
__global__ void selftest_kernel(int32_t* fails) {
  const int l = threadIdx.x;
  const int c = l & 15, q = l >> 4;
  int bad = 0;
  // permlane all-reduces
  const double v = (double)(l * l + 1);
  const double s16 = xor16_sum(v), s32 = xor32_sum(v), s4 = colsum4(v);
  const double e16 = v + (double)((l ^ 16) * (l ^ 16) + 1);
  const double e32 = v + (double)((l ^ 32) * (l ^ 32) + 1);
  double e4 = 0;
  for (int k = 0; k < 4; ++k) e4 += (double)((c + 16 * k) * (c + 16 * k) + 1);
  bad += (s16 != e16) + (s32 != e32) + (s4 != e4);
  // MFMA f64 16x16x4: A-operand lane l = A[l&15][l>>4], B = B[l>>4][l&15],
  // C/D reg r of lane l = D[(l>>4) + 4r][l&15]. Use asymmetric integer data.
  const double Aij = (double)(c * 7 + q * 3 + 1);   // A[c][q]
  const double Bij = (double)(q * 5 + c * 2 + 2);   // B[q][c]
  d4 acc = {0, 0, 0, 0};
  acc = mfma(Aij, Bij, acc);
  for (int r = 0; r < 4; ++r) {
    const int i = q + 4 * r, jj = c;
    double e = 0;
    for (int k = 0; k < 4; ++k) e += (double)(i * 7 + k * 3 + 1) * (double)(k * 5 + jj * 2 + 2);
    bad += (acc[r] != e);
  }
  // row-16 shuffle sum
  const double rs = rowsum16((double)l);
  double er = 0;
  for (int k = 0; k < 16; ++k) er += (double)((l & ~15) + k);
  bad += (rs != er);
  if (bad) atomicAdd(fails, bad);
}

}  // namespace

// ---------------------------------------------------------------------------
// Launchers
// ---------------------------------------------------------------------------
bool lq_supported(int nx, int nu) { return nx == 12 && nu == 4; }

#define ILQR_DISPATCH(NXV, NUV, CALL)            \
  if (nx == NXV && nu == NUV) {                  \
    constexpr int NX_ = NXV, NU_ = NUV;          \
    CALL;                                        \
    return hipGetLastError();                    \
  }

hipError_t launch_lq_backward(int nx, int nu, const LQParams& p, int B, int T, const double* x,
                              const double* u, double* d, double* K, int32_t* status, double mu,
                              hipStream_t s, bool wave) {
  if (wave) return launch_lq_backward_v6(nx, nu, p, B, T, x, u, d, K, status, mu, s);
  if (nx == 12 && nu == 4) return launch_lq_backward4(p, B, T, x, u, d, K, status, mu, s);
  return hipErrorInvalidValue;
}

hipError_t launch_lq_backward_v6(int nx, int nu, const LQParams& p, int B, int T, const double* x,
                                 const double* u, double* d, double* K, int32_t* status, double mu,
                                 hipStream_t s) {
  const int grid = (B + WAVES_PER_WG - 1) / WAVES_PER_WG;
  ILQR_DISPATCH(12, 4, (lq_backward_kernel<NX_, NU_><<<grid, 256, 0, s>>>(p, B, T, x, u, d, K, status, mu)));
  return hipErrorInvalidValue;
}

hipError_t launch_lq_forward(int nx, int nu, const LQParams& p, int B, int T, const double* x,
                             const double* u, const double* xtraj, const double* d,
                             const double* K, const double* prev_cost, double* xnew,
                             double* unew, double* new_cost, int32_t* trials, int32_t* status,
                             const LSParams& ls, hipStream_t s, bool ring, bool mfma) {
  const int grid = (B + 3) / 4;
  if (ring) {
    const int gridr = (B + 4 * FW_WAVES - 1) / (4 * FW_WAVES);
    if (mfma)
      ILQR_DISPATCH(12, 4, (lq_forward_ring_kernel<NX_, NU_, true><<<gridr, 64 * FW_WAVES, 0, s>>>(p, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls)));
    ILQR_DISPATCH(12, 4, (lq_forward_ring_kernel<NX_, NU_><<<gridr, 64 * FW_WAVES, 0, s>>>(p, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls)));
  }
  ILQR_DISPATCH(12, 4, (lq_forward_kernel<NX_, NU_><<<grid, 64, 0, s>>>(p, B, T, x, u, xtraj, d, K, prev_cost, xnew, unew, new_cost, trials, status, ls)));
  return hipErrorInvalidValue;
}

namespace {
LQParams shift(const LQParams& p, int nx, int nu, int b0) {
  return LQParams{p.A + (size_t)b0 * nx * nx, p.B + (size_t)b0 * nx * nu, p.Q + (size_t)b0 * nx * nx,
                  p.R + (size_t)b0 * nu * nu, p.Qf + (size_t)b0 * nx * nx};
}
template <class T>
T* off(T* p, size_t n) { return p ? p + n : p; }
IterArgs shift(const IterArgs& a, int nx, int nu, int T, int b0) {
  IterArgs r = a;
  const size_t b = (size_t)b0;
  r.x = off(a.x, b * (T + 1) * nx);
  r.u = off(a.u, b * T * nu);
  r.xtraj = off(a.xtraj, b * (T + 1) * nx);
  r.xnew = off(a.xnew, b * (T + 1) * nx);
  r.unew = off(a.unew, b * T * nu);
  r.K = off(a.K, b * T * nu * nx);
  r.d = off(a.d, b * T * nu);
  r.prev_cost = off(a.prev_cost, b);
  r.new_cost = off(a.new_cost, b);
  r.du2 = off(a.du2, b);
  r.trials = off(a.trials, b);
  r.status = off(a.status, b);
  r.res_parity = off(a.res_parity, b);
  r.iters = off(a.iters, b);
  return r;
}
}  // namespace

hipError_t launch_lq_iter_backward(int nx, int nu, const LQParams& p, int b0, int b1, int T,
                                   const IterArgs& a, double mu, hipStream_t s, bool wave) {
  const int B = b1 - b0;
  if (B <= 0) return hipSuccess;
  const LQParams ps = shift(p, nx, nu, b0);
  const IterArgs as = shift(a, nx, nu, T, b0);
  if (wave) {
    const int grid = (B + WAVES_PER_WG - 1) / WAVES_PER_WG;
    ILQR_DISPATCH(12, 4, (lq_iter_backward_kernel<NX_, NU_><<<grid, 256, 0, s>>>(ps, B, T, as, mu)));
    return hipErrorInvalidValue;
  }
  if (nx == 12 && nu == 4) return launch_lq_iter_backward4(ps, B, T, as, mu, s);
  return hipErrorInvalidValue;
}

hipError_t launch_lq_iter_forward(int nx, int nu, const LQParams& p, int b0, int b1, int T,
                                  const IterArgs& a, const LSParams& ls, hipStream_t s, bool ring,
                                  bool mfma) {
  const int B = b1 - b0;
  if (B <= 0) return hipSuccess;
  const LQParams ps = shift(p, nx, nu, b0);
  const IterArgs as = shift(a, nx, nu, T, b0);
  if (ring) {
    if (mfma)
      ILQR_DISPATCH(12, 4, (lq_iter_forward_ring_kernel<NX_, NU_, true><<<(B + 4 * FW_WAVES - 1) / (4 * FW_WAVES), 64 * FW_WAVES, 0, s>>>(ps, B, T, as, ls)));
    ILQR_DISPATCH(12, 4, (lq_iter_forward_ring_kernel<NX_, NU_><<<(B + 4 * FW_WAVES - 1) / (4 * FW_WAVES), 64 * FW_WAVES, 0, s>>>(ps, B, T, as, ls)));
  }
  ILQR_DISPATCH(12, 4, (lq_iter_forward_kernel<NX_, NU_><<<(B + 3) / 4, 64, 0, s>>>(ps, B, T, as, ls)));
  return hipErrorInvalidValue;
}

hipError_t launch_lq_iter_pipe(int nx, int nu, const LQParams& p, int B, int T, const IterArgs& cur,
                               const IterArgs& prev, const LSParams& ls, int flags, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  const int grid = (B + WAVES_PER_WG - 1) / WAVES_PER_WG;
  ILQR_DISPATCH(12, 4, (lq_iter_pipe_kernel<NX_, NU_><<<grid, 256, 0, s>>>(p, B, T, cur, prev, ls, flags)));
  return hipErrorInvalidValue;
}

hipError_t launch_gather_result(int B, int T, int nx, int nu, const double* xin, const double* uin,
                                const double* x0, const double* u0, const double* x1,
                                const double* u1, const int32_t* res_parity, int32_t* status,
                                int final_parity, const double* fit_cost, const int32_t* fit_iters,
                                double* x_out, double* u_out, double* cost_out,
                                int32_t* iters_out, int32_t* status_out, int32_t* dflags,
                                int32_t* flags, hipStream_t s, uint32_t seq) {
  if (B <= 0) return hipSuccess;
  gather_kernel<<<(B + 3) / 4, 256, 0, s>>>(B, T, nx, nu, xin, uin, x0, u0, x1, u1, res_parity, status,
                                            final_parity, fit_cost, fit_iters, x_out, u_out, cost_out,
                                            iters_out, status_out, dflags);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  gather_flags_kernel<<<1, 1, 0, s>>>(dflags, flags, seq);
  return hipGetLastError();
}

hipError_t launch_lq_linearize(int nx, int nu, const LQParams& p, int B, int T, double* A, double* Bm,
                               hipStream_t s) {
  if (B <= 0 || T <= 0) return hipSuccess;
  const size_t nA = (size_t)B * T * nx * nx, nB = (size_t)B * T * nx * nu;
  lq_broadcast_steps_kernel<<<(unsigned)((nA + 255) / 256), 256, 0, s>>>(p.A, A, T, nx * nx, nA);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  lq_broadcast_steps_kernel<<<(unsigned)((nB + 255) / 256), 256, 0, s>>>(p.B, Bm, T, nx * nu, nB);
  return hipGetLastError();
}

hipError_t launch_record_history(int B, int it, const int32_t* status, const int32_t* iters,
                                 const int32_t* trials, const void* cost, const void* du2, bool f32,
                                 double alpha0, double shrink, double* h_cost, int32_t* h_trials,
                                 double* h_alpha, double* h_du2, hipStream_t s, int stride) {
  if (B <= 0) return hipSuccess;
  if (stride <= 0) stride = B;
  const unsigned g = (unsigned)((B + 255) / 256);
  if (f32)
    record_history_kernel<float><<<g, 256, 0, s>>>(B, stride, it, status, iters, trials, (const float*)cost,
                                                   (const float*)du2, (float)alpha0, (float)shrink, h_cost,
                                                   h_trials, h_alpha, h_du2);
  else
    record_history_kernel<double><<<g, 256, 0, s>>>(B, stride, it, status, iters, trials, (const double*)cost,
                                                    (const double*)du2, alpha0, shrink, h_cost, h_trials,
                                                    h_alpha, h_du2);
  return hipGetLastError();
}

hipError_t launch_fit_init(int B, double* prev_cost, int32_t* status, int32_t* res_parity,
                           int32_t* iters, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  fit_init_kernel<<<(B + 255) / 256, 256, 0, s>>>(B, prev_cost, status, res_parity, iters);
  return hipGetLastError();
}

hipError_t launch_pad3(const double* src, double* dst, size_t N, int R, int C, int R2, int C2,
                       hipStream_t s) {
  const size_t total = N * R2 * C2;
  if (total == 0) return hipSuccess;
  pad3_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(src, dst, total, R, C, R2, C2);
  return hipGetLastError();
}
hipError_t launch_unpad3(const double* src, double* dst, size_t N, int R, int C, int R2, int C2,
                         hipStream_t s) {
  const size_t total = N * R * C;
  if (total == 0) return hipSuccess;
  unpad3_kernel<<<(unsigned)((total + 255) / 256), 256, 0, s>>>(src, dst, total, R, C, R2, C2);
  return hipGetLastError();
}

hipError_t launch_fill_i32(int32_t* p, int n, int32_t v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  fill_i32_kernel<<<(n + 255) / 256, 256, 0, s>>>(p, n, v);
  return hipGetLastError();
}
hipError_t launch_fill_f64(double* p, int n, double v, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  fill_f64_kernel<<<(n + 255) / 256, 256, 0, s>>>(p, n, v);
  return hipGetLastError();
}

// number of trajectories still running (status OK) → *out (host-mapped memory: the fit
// driver polls it one iteration behind to stop enqueueing once every trajectory has
// stopped, as the reference's loop breaks, forward_pass.jl:171)
__global__ __launch_bounds__(256) void count_running_kernel(int B, const int32_t* __restrict__ status,
                                                            int32_t* out) {
  __shared__ int total;
  if (threadIdx.x == 0) total = 0;
  __syncthreads();
  int n = 0;
  for (int b = threadIdx.x; b < B; b += 256) n += status[b] == ILQR_TRAJ_OK;
  atomicAdd(&total, n);
  __syncthreads();
  if (threadIdx.x == 0) *out = total;
}

hipError_t launch_publish_flags(int32_t* dflags, int32_t* flags, uint32_t seq, hipStream_t s) {
  gather_flags_kernel<<<1, 1, 0, s>>>(dflags, flags, seq);
  return hipGetLastError();
}

hipError_t launch_count_running(int B, const int32_t* status, int32_t* out, hipStream_t s) {
  count_running_kernel<<<1, 256, 0, s>>>(B, status, out);
  return hipGetLastError();
}

int run_selftest(int device) {
  if (hipSetDevice(device) != hipSuccess) return -1;
  int32_t* f = nullptr;
  if (hipMalloc(&f, sizeof(int32_t)) != hipSuccess) return -1;
  int32_t h = 0;
  if (hipMemset(f, 0, sizeof(int32_t)) != hipSuccess) return -1;
  selftest_kernel<<<1, 64>>>(f);
  if (hipGetLastError() != hipSuccess) return -1;
  if (hipMemcpy(&h, f, sizeof(int32_t), hipMemcpyDeviceToHost) != hipSuccess) return -1;
  (void)hipFree(f);
  return h;
}

}  // namespace ilqr
