// Backward pass of the LQ family with FOUR trajectories per wave on the 4-block
// f64 MFMA, v_mfma_f64_4x4x4f64 (backward v7).
//
// Reference path: backward_pass (aabouman/iLQR.jl src/backward_pass.jl:324-357) —
// the same recursion as lq_backward_wave in ilqr_lq.hip, re-tiled:
//  * the 4-block MFMA computes four independent 4×4×4 products per instruction
//    (one per trajectory slot β) at 63-66 TF/s against 42-44 TF/s for the 16×16×4
//    tile (profiles/r01/ubench_f64_4x4.log), and its 4×4 blocks fit the 12-state,
//    4-input shape exactly: no zero padding of the 13×16 augmented tile;
//  * the 4×4 gain solve runs once per slot (16 lanes) instead of once per wave,
//    so the VALU share is amortised over four trajectories.
//
// Lane layout (measured by tools/mfma4_probe.hip): lane l = 16ρ + 4β + κ holds
// element [ρ][κ] of slot β's 4×4 block ("D layout"). The instruction computes
//     mf4(a, b, c) = c + aᵀ·b      for D-layout blocks a, b, c
// i.e. a D-layout register is the B operand as is and the A operand transposed.
// Vectors are kept "replicated": block register v[I] holds v[4I+ρ] in every κ.
//
// Per step (nx = 12 → 3 blocks, nu = 4 → 1 block; F = [A | B] = F[K][J], K < 3, J < 4):
//   Y[I][J]  = Σ_K mf4(S[K][I], F[K][J])                 S·F            36 MFMAs
//   Z[I][J]  = L[I][J] + Σ_K mf4(F[K][I], Y[K][J])       FᵀSF, I ≤ J    30 MFMAs
//   gv[I]    = Σ_K mf4(L[K][I], z[K]) + Σ_K mf4(F[K][I], s[K])
//            = [lx + Aᵀs | lu + Bᵀs]                                     22 MFMAs
//   H_reg = Z[3][3] + μI = L D Lᵀ (every lane of the slot, VALU), M = L⁻¹:
//   P[J]     = Mᵀ D⁻¹ M [G | g][J]  = (H + μI)⁻¹[G | g]   (K_aug = −P)   8 MFMAs
//   W        = (H + 2μI) K_aug = −([G | g] + μP)
//   S[I][J]  = mf4(P[I], W[J], Z[I][J])  (I ≤ J < 3),  s[I] = mf4(P[I], W[3], gv[I])
//            = [Qxx | lx + Aᵀs] − K_augᵀ(H + 2μI)K_aug   (step_back :268-270)
//   S[J][I]  = S[I][J]ᵀ by an MFMA transpose (mf4(a, I, 0) = aᵀ, exact), diagonal
//              blocks symmetrised every SYM_EVERY steps as in the 16×16 kernel.
// The solve is LDLᵀ as in the one-trajectory kernel, applied as the triangular
// factors' explicit inverses on the MFMA (M = L⁻¹ has six entries). The step loop runs
// four steps at a time (each step's column of its L z block is then static). At one
// wave per SIMD the step is issue-bound: every instruction costs the wave's issue
// (≈16 cycles an MFMA, ≈6 any VALU op, tools/ubench_mix.hip), so the step is written
// for instruction count.
#include <hip/hip_runtime.h>
#include <math.h>

#include "ilqr_internal.h"
#include "ilqr_device.h"
#include "ilqr_fwd_ring.h"
#include "../../include/ilqr.h"

namespace ilqr {
namespace {

// Measured choices of the step (the alternates they replaced, and the probe bits of
// tools/bw4_probe.hip, live in tools/ablation/restore_alternates.patch):
//  * μ folded into H's MFMA accumulator (R + Rᵀ + μI): no per-step pivot adds
//    (backward 103.8 -> 102.7 us; the alternate added it in the factorisation);
//  * the lower S blocks, the solve's Mᵀ and the diagonal symmetrisation as MFMA
//    transposes (mf4(a, I, 0) = aᵀ, exact) instead of ds_bpermute lane permutations;
//  * the solve's per-lane operands (M[ρ][κ], D⁻¹[ρ]) by 0/1-mask FMAs instead of select
//    chains: every VALU instruction beside the MFMAs costs the wave ≈6 cycles of issue,
//    b32 selects as much as f64 FMAs (tools/ubench_mix.hip);
//  * L z for four steps per MFMA set, its columns moved by lane permutations (one per
//    step, behind the S·F products) rather than one MFMA set per step or an LDS pass.

constexpr int BW4_SLOTS = 4;          // trajectories per wave
constexpr int BW4_WAVES = 4;          // waves per workgroup
constexpr int BW4_LDS = 64 + 256;     // doubles of LDS per wave: the four H tiles, L z columns

__device__ __forceinline__ double mf4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

// v from lane `src_byte / 4` (ds_bpermute, both dwords)
__device__ __forceinline__ double lane_perm(double v, int src_byte) {
  u2v p = __builtin_bit_cast(u2v, v);
  p.x = (unsigned)__builtin_amdgcn_ds_bpermute(src_byte, (int)p.x);
  p.y = (unsigned)__builtin_amdgcn_ds_bpermute(src_byte, (int)p.y);
  return __builtin_bit_cast(double, p);
}

// lanes of slot β: bits [3:2] of the lane index
__device__ __forceinline__ unsigned long long slot_lanes(int beta) {
  return (0xFull << (4 * beta)) * 0x0001000100010001ull;
}

// mf4 with a negated A operand (the f64 MFMA's neg modifier, blgp bit 0)
__device__ __forceinline__ double mf4n(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 1);
}

__device__ __forceinline__ double buf_ld(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, voff, soff, 0));
}
__device__ __forceinline__ void buf_st(double v, __amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, v), r, voff, soff, 0);
}

// Backward pass of trajectories b0 .. b0+3 (slots with active bit clear, or past B,
// compute on clamped data and store nothing). Returns the slots whose gains hold a
// NaN (bit β): the reference's @assert !any(isnan, ...) (:353-354). A NaN in any K_t
// or d_t reaches K_0 or d_0 (S and s carry it down the recursion; no step compares,
// selects or clamps), so the test reads the last step's gains only.
__device__ unsigned lq_backward4_wave(const LQParams& P, int b0, int B, unsigned active, int T,
                                      const double* __restrict__ x, const double* __restrict__ u,
                                      double* __restrict__ d_out, double* __restrict__ K_out,
                                      double mu, double* lds) {
  constexpr int NX = 12, NU = 4;
  b0 = __builtin_amdgcn_readfirstlane(b0);
  const int l = threadIdx.x & 63;
  const int rho = l >> 4;
  const int beta = (l >> 2) & 3;
  const int kap = l & 3;
  const int b = b0 + beta;
  const bool live = b < B && ((active >> beta) & 1u);
  const int bc = b < B ? b : B - 1;  // clamped: every load stays in bounds
  const int nslot = B - b0 < 4 ? B - b0 : 4;

  const double* Ab = P.A + (size_t)bc * NX * NX;
  const double* Bb = P.B + (size_t)bc * NX * NU;
  const double* Qb = P.Q + (size_t)bc * NX * NX;
  const double* Rb = P.R + (size_t)bc * NU * NU;
  const double* Qfb = P.Qf + (size_t)bc * NX * NX;

  // F = [A | B] blocks, L = Q + Qᵀ blocks (immediate_cost_quadratization :101-106)
  double F[3][4], L[3][3];
#pragma unroll
  for (int K = 0; K < 3; ++K) {
    const int r = 4 * K + rho;
#pragma unroll
    for (int J = 0; J < 3; ++J) F[K][J] = Ab[r * NX + 4 * J + kap];
    F[K][3] = Bb[r * NU + kap];
#pragma unroll
    for (int I = 0; I < 3; ++I) L[K][I] = Qb[r * NX + 4 * I + kap] + Qb[(4 * I + kap) * NX + r];
  }
  const double LR = Rb[rho * NU + kap] + Rb[kap * NU + rho];
  const double LRmu = rho == kap ? LR + mu : LR;  // R + Rᵀ + μI

  // the block transpose within each slot on the MFMA: mf4(a, I, 0) = aᵀ, exact (products
  // with 1 and 0); mf4(a, I/2, a/2) = (a + aᵀ)/2 with one rounding, = 0.5·(a + aᵀ) bit
  // for bit (a ≈50-cycle MFMA result instead of a ds_bpermute round trip on the solve's
  // and the symmetrisation's dependent chains)
  const double Id = rho == kap ? 1.0 : 0.0, Ih = rho == kap ? 0.5 : 0.0;
  // lane masks of the solve's per-lane entries: M[i][j] (i > j) at lane (ρ, κ) = (i, j),
  // the unit diagonal, D⁻¹[i] at row ρ = i
  double sel_m[4][4], sel_r[4];
  const double sel_d = Id;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    sel_r[i] = rho == i ? 1.0 : 0.0;
#pragma unroll
    for (int j = 0; j < 4; ++j) sel_m[i][j] = (rho == i && kap == j) ? 1.0 : 0.0;
  }

  // terminal value function (final_cost_quadratization :134-153): S = Qf + Qfᵀ, s = S x_N
  double S[3][3], s[3];
  {
    const double* xN = x + ((size_t)bc * (T + 1) + T) * NX;
    double xr[3];
#pragma unroll
    for (int K = 0; K < 3; ++K) {
      const int r = 4 * K + rho;
      xr[K] = xN[r];
#pragma unroll
      for (int I = 0; I < 3; ++I) S[K][I] = Qfb[r * NX + 4 * I + kap] + Qfb[(4 * I + kap) * NX + r];
    }
#pragma unroll
    for (int I = 0; I < 3; ++I) {
      double v = 0.0;
#pragma unroll
      for (int K = 0; K < 3; ++K) v = mf4(S[K][I], xr[K], v);
      s[I] = v;
    }
  }

  // the wave's x, u, K, d through buffer resources over its slots (records end at
  // slot nslot: loads past it read 0, stores are dropped); per-lane offsets are
  // loop constants, the step enters as the scalar offset
  const auto rX = buffer_rsrc(const_cast<double*>(x) + (size_t)b0 * (T + 1) * NX, (uint32_t)(nslot * (T + 1) * NX * 8));
  const auto rU = buffer_rsrc(const_cast<double*>(u) + (size_t)b0 * T * NU, (uint32_t)(nslot * T * NU * 8));
  const auto rK = buffer_rsrc(K_out + (size_t)b0 * T * NU * NX, (uint32_t)(nslot * T * NU * NX * 8));
  const auto rD = buffer_rsrc(d_out + (size_t)b0 * T * NU, (uint32_t)(nslot * T * NU * 8));
  const uint32_t DEAD = 0x80000000u;  // beyond every record count
  const uint32_t kv = live ? (uint32_t)((beta * T * NU * NX + rho * NX + kap) * 8) : DEAD;
  const uint32_t dv = (live && kap == 0) ? (uint32_t)((beta * T * NU + rho) * 8) : DEAD;

  // z_t = [x_t; u_t] (cost gradient L z, :101-106): one MFMA set gives L z for steps
  // t0 .. t0-3 (column κ = step t0-κ); each step permutes its column out.
  double Lzq[4] = {0.0, 0.0, 0.0, 0.0}, zq[4];
  auto load_zq = [&](int t0) {  // clamped at step 0
    const int tz = t0 - kap > 0 ? t0 - kap : 0;
    const uint32_t xo = (uint32_t)(((beta * (T + 1) + tz) * NX + rho) * 8);
    const uint32_t uo = (uint32_t)(((beta * T + tz) * NU + rho) * 8);
#pragma unroll
    for (int K = 0; K < 3; ++K) zq[K] = buf_ld(rX, xo + 32 * K, 0);
    zq[3] = buf_ld(rU, uo, 0);
  };
  // L z for the four steps from t0 (column κ = step t0 − κ), from zq; then the next
  // four steps' z. Computed one step ahead of its first use, so each step's column
  // permutes can issue at the top of the step, behind the S·F MFMAs.
  auto lz_block = [&](int t0) {
#pragma unroll
    for (int I = 0; I < 3; ++I) {
      double v = 0.0;
#pragma unroll
      for (int K = 0; K < 3; ++K) v = mf4(L[K][I], zq[K], v);
      Lzq[I] = v;
    }
    Lzq[3] = mf4(LR, zq[3], 0.0);
    load_zq(t0 - 4);
  };
  load_zq(T - 1);

  double* Hl = lds + beta * 16;
  double Klast[4];
  // every load of the prologue lands here, so the loop's waits only count the loop's
  // own loads
  __builtin_amdgcn_s_waitcnt(0);
  lz_block(T - 1);

  // lane-permutation sources of the L z columns, one per step of a block of four
  int lz_src[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) lz_src[j] = ((l & ~3) | j) * 4;
  // one step of the recursion; JJ = (T − 1 − t) mod 4 (the step's column of its L z block)
  // is static: the loop below runs the steps four at a time
  auto step = [&](const int t, auto jc) {
    constexpr int JJ = decltype(jc)::value;
    // this step's L z columns: the permutes issue here, their LDS latency hidden behind
    // the S·F products
    double lzp[4];
#pragma unroll
    for (int I = 0; I < 4; ++I) lzp[I] = lane_perm(Lzq[I], lz_src[JJ]);
    // Y = S·F, column block 3 (B) first: H needs it. Each sum runs over K = 0, 1, 2;
    // its K ≤ I terms read stored upper blocks S[K][I], its K > I terms the lower blocks
    // that the previous step's lane permutations produce: all 24 upper-block products
    // issue first (same summation order), so the permutes' latency hides behind them.
    double Y[3][4];
#pragma unroll
    for (int J = 3; J >= 0; --J)
#pragma unroll
      for (int I = 0; I < 3; ++I) {
        double v = 0.0;
#pragma unroll
        for (int K = 0; K <= I; ++K) v = mf4(S[K][I], F[K][J], v);
        Y[I][J] = v;
      }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int J = 3; J >= 0; --J)
#pragma unroll
      for (int I = 0; I < 2; ++I)
#pragma unroll
        for (int K = I + 1; K < 3; ++K) Y[I][J] = mf4(S[K][I], F[K][J], Y[I][J]);
    // H = R + Rᵀ + BᵀSB → LDS, read back whole by the slot's lanes
    double H = LRmu;
#pragma unroll
    for (int K = 0; K < 3; ++K) H = mf4(F[K][3], Y[K][3], H);
    Hl[rho * 4 + kap] = H;

    // gradient [lx + Aᵀs | lu + Bᵀs] (:181, :269)
    double gv[4];
#pragma unroll
    for (int I = 0; I < 4; ++I) {
      double v = lzp[I];
#pragma unroll
      for (int K = 0; K < 3; ++K) v = mf4(F[K][I], s[K], v);
      gv[I] = v;
    }
    // G = BᵀSA (lux = 0) and Qxx = lxx + AᵀSA (upper blocks)
    double G[3], Z[3][3];
#pragma unroll
    for (int J = 0; J < 3; ++J) {
      double v = 0.0;
#pragma unroll
      for (int K = 0; K < 3; ++K) v = mf4(F[K][3], Y[K][J], v);
      G[J] = v;
    }
#pragma unroll
    for (int I = 0; I < 3; ++I)
#pragma unroll
      for (int J = I; J < 3; ++J) {
        double v = L[I][J];
#pragma unroll
        for (int K = 0; K < 3; ++K) v = mf4(F[K][I], Y[K][J], v);
        Z[I][J] = v;
      }

    // (H + μI) = L D Lᵀ in every lane of the slot (feedback_parameters :207-218)
    // (read right after the write instead — its latency behind the gradient, G and
    // Qxx MFMAs — measured slower: 103.8 -> 105.6 us)
    wave_lds_fence();
    double h[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int k = 0; k <= i; ++k) h[i][k] = Hl[i * 4 + k];
    wave_lds_fence();
    LDLT<4, 1> f;
    f.factor<false>(h, mu);  // μ is in H already
    // M = L⁻¹ (unit lower)
    double Mf[4][4];
    Mf[1][0] = -f.l[1][0];
    Mf[2][1] = -f.l[2][1];
    Mf[2][0] = fma(f.l[2][1], f.l[1][0], -f.l[2][0]);
    Mf[3][2] = -f.l[3][2];
    Mf[3][1] = fma(f.l[3][2], f.l[2][1], -f.l[3][1]);
    Mf[3][0] = fma(-f.l[3][2], Mf[2][0], fma(-f.l[3][1], Mf[1][0], -f.l[3][0]));
    // this lane's entries: Mn = M[ρ][κ], D⁻¹[ρ]
    // Σ (0/1 lane mask) × entry: exact (x·1 = x, x·0 = ±0 and x ± 0 = x), so the same
    // bits as selects, in 10 f64 ops where the selects took 18 b32 ones
    double Mn = sel_d;
#pragma unroll
    for (int i = 1; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < i; ++j) Mn = fma(sel_m[i][j], Mf[i][j], Mn);
    double dsel = sel_r[0] * f.dinv[0];
#pragma unroll
    for (int i = 1; i < 4; ++i) dsel = fma(sel_r[i], f.dinv[i], dsel);

    // K_aug = −(H + μI)⁻¹ [G | g] = −(D⁻¹M)ᵀ (M [G | g]): the LDLᵀ solve's two
    // triangular sweeps as two MFMA stages. A operands: M·  wants M[κ][ρ] (the
    // transpose of Mn, by the lane permutation), (D⁻¹M)ᵀ· wants D⁻¹[ρ] M[ρ][κ].
    // (Forming (H + μI)⁻¹ = Mᵀ D⁻¹ M explicitly instead costs two digits on the
    // headline's near-rank-1 H: 2e-11 against the oracle where the sweeps give 1.7e-13,
    // profiles/r01/bw4_quad.txt; a residual-checked Newton-Schulz inverse measured
    // slower, tools/ablation/bw4_newton_schulz.patch.)
    double Kg[4];
    const double Mt = mf4(Mn, Id, 0.0), Mnd = Mn * dsel;
#pragma unroll
    for (int J = 0; J < 4; ++J) Kg[J] = mf4n(Mnd, mf4(Mt, J < 3 ? G[J] : gv[3], 0.0), 0.0);
#pragma unroll
    for (int J = 0; J < 3; ++J) buf_st(Kg[J], rK, kv + 32 * J, (uint32_t)(t * NU * NX * 8));
    buf_st(Kg[3], rD, dv, (uint32_t)(t * NU * 8));

    // step_back (:268-270): W = (H + 2μI) K_aug = μ K_aug − [G | g],
    // [S | s] = [Qxx | lx + Aᵀs] − K_augᵀ W
    double W[4];
#pragma unroll
    for (int J = 0; J < 3; ++J) W[J] = fma(mu, Kg[J], -G[J]);
    W[3] = fma(mu, Kg[3], -gv[3]);
#pragma unroll
    for (int I = 0; I < 3; ++I) {
#pragma unroll
      for (int J = I; J < 3; ++J) S[I][J] = mf4n(Kg[I], W[J], Z[I][J]);
      s[I] = mf4n(Kg[I], W[3], gv[I]);
    }
    if ((t % SYM_EVERY) == 0) {
#pragma unroll
      for (int I = 0; I < 3; ++I) S[I][I] = mf4(S[I][I], Ih, 0.5 * S[I][I]);
    }
#pragma unroll
    for (int I = 0; I < 3; ++I)
#pragma unroll
      for (int J = I + 1; J < 3; ++J) S[J][I] = mf4(S[I][J], Id, 0.0);
#pragma unroll
    for (int J = 0; J < 4; ++J) Klast[J] = Kg[J];
    // the next step starts a block of four: its L z now
    if constexpr (JJ == 3) {
      if (t > 0) lz_block(t - 1);
    }
  };
  using I0 = std::integral_constant<int, 0>;
  using I1 = std::integral_constant<int, 1>;
  using I2 = std::integral_constant<int, 2>;
  using I3 = std::integral_constant<int, 3>;
  int t = T - 1;
  for (; t >= 3; t -= 4) {
    step(t, I0{});
    step(t - 1, I1{});
    step(t - 2, I2{});
    step(t - 3, I3{});
  }
  if (t >= 0) step(t, I0{});
  if (t >= 1) step(t - 1, I1{});
  if (t >= 2) step(t - 2, I2{});
  bool nan = false;
#pragma unroll
  for (int J = 0; J < 4; ++J) nan |= __builtin_isnan(Klast[J]);
  const unsigned long long nb = __ballot(nan);
  unsigned r = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) r |= (nb & slot_lanes(q)) ? (1u << q) : 0u;
  return r;
}

__global__ __launch_bounds__(256) void lq_backward4_kernel(LQParams P, int B, int T,
                                                           const double* __restrict__ x,
                                                           const double* __restrict__ u,
                                                           double* __restrict__ d,
                                                           double* __restrict__ K,
                                                           int32_t* __restrict__ status, double mu) {
  __shared__ __attribute__((aligned(16))) double lds[BW4_WAVES * BW4_LDS];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * BW4_WAVES + w) * BW4_SLOTS;
  if (b0 >= B) return;
  const unsigned nan = lq_backward4_wave(P, b0, B, 0xFu, T, x, u, d, K, mu, lds + w * BW4_LDS);
  const int l = threadIdx.x & 63;
  if (status && l < BW4_SLOTS && b0 + l < B) status[b0 + l] = ((nan >> l) & 1u) ? ILQR_TRAJ_NAN : ILQR_TRAJ_OK;
}

// fit iteration, part 1 (see lq_iter_backward_kernel): slots whose status is not OK
// are skipped (computed on, never stored)
__global__ __launch_bounds__(256) void lq_iter_backward4_kernel(LQParams P, int B, int T, IterArgs a,
                                                                double mu) {
  __shared__ __attribute__((aligned(16))) double lds[BW4_WAVES * BW4_LDS];
  const int w = threadIdx.x >> 6;
  const int b0 = (blockIdx.x * BW4_WAVES + w) * BW4_SLOTS;
  if (b0 >= B) return;
  unsigned active = 0;
#pragma unroll
  for (int q = 0; q < BW4_SLOTS; ++q)
    if (b0 + q < B && a.status[b0 + q] == ILQR_TRAJ_OK) active |= 1u << q;
  if (active == 0) return;
  const unsigned nan = lq_backward4_wave(P, b0, B, active, T, a.x, a.u, a.d, a.K, mu, lds + w * BW4_LDS) & active;
  const int l = threadIdx.x & 63;
  if (l < BW4_SLOTS && ((nan >> l) & 1u)) {
    a.status[b0 + l] = ILQR_TRAJ_NAN;  // reference: AssertionError at backward_pass.jl:353
    if (a.res_parity) a.res_parity[b0 + l] = a.parity;
  }
}

// One fit iteration (forward_pass.jl:162-175) in ONE launch: each wave runs the
// backward pass of its four trajectories (lq_backward4_wave) and then their forward
// pass with the LDS-ring input stream (lq_forward_wave_ring, ilqr_fwd_ring.h) — the
// kernels of lq_iter_backward4_kernel and lq_iter_forward_ring_kernel back to back,
// same arithmetic, same bits. One wave per workgroup (the ring's 29 KB of LDS); no
// kernel boundary between the passes, and the gains the forward streams in were
// written by the same wave moments before. Four waves per workgroup, each with its
// own 29 KB ring (116 KB of LDS: one workgroup per CU, its four waves on the CU's four
// SIMDs); one-wave workgroups measured 225 µs instead of 157 µs on some launches — the
// dispatcher packed two of them onto one SIMD.
constexpr int FUSED_WAVES = 4;
constexpr int FUSED_LDS = PIPE_R * RING_SLOT + RING_LAREA;  // doubles per wave
template <bool MF>
__global__ __launch_bounds__(64 * FUSED_WAVES) void lq_iter_fused4_kernel(LQParams P, int B, int T,
                                                                         IterArgs a, LSParams ls) {
  __shared__ __attribute__((aligned(16))) double lds_all[FUSED_WAVES * FUSED_LDS];
  static_assert(FUSED_LDS >= BW4_LDS, "backward scratch fits the ring");
  const int w = threadIdx.x >> 6;
  double* lds = lds_all + w * FUSED_LDS;
  const int wid = blockIdx.x * FUSED_WAVES + w;
  const int b0 = wid * BW4_SLOTS;
  // the cooperative line search (row-form forward, 2 ≤ max_trials ≤ 64): every wave of
  // the launch takes part, present or not
  const bool coop = !MF && a.coop && ls.max_trials >= 2 && ls.max_trials <= COOP_MAX_TRIALS;
  const int l = threadIdx.x & 63;
  // the lane that writes slot q's per-trajectory words (the forward's writer: lane 16q
  // in the row form, lane 4q in the MFMA form), so the writes of one slot keep program order
  const bool owner = MF ? (l < 16 && (l & 3) == 0) : (l & 15) == 0;
  const int q = MF ? (l >> 2) & 3 : l >> 4;
  unsigned active = 0;
  unsigned own = 0;  // the wave's published trajectories (iter_forward_wave_coop)
  IterArgs ai = a;
  if (a.coop && wid == 0 && l == 0) {
    // the next launch's list length (this launch counts in ctl[gen & 1])
    __hip_atomic_store(a.coop_ctl + ((a.coop_gen + 1) & 1), 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (b0 < B) {
    if (a.init) {
      // fit's first iteration (fit_init_kernel's job, :159): every present trajectory
      // runs from prev_cost = Inf
      const int nt = B - b0 < BW4_SLOTS ? B - b0 : BW4_SLOTS;
      active = (1u << nt) - 1u;
      if (owner && q < nt) {
        const int b = b0 + q;
        a.new_cost[b] = INFINITY;  // = prev_cost (in place)
        a.status[b] = ILQR_TRAJ_OK;
        a.res_parity[b] = PARITY_INPUT;
        a.iters[b] = 0;
      }
      ai.prev_cost = nullptr;  // +Inf without reading
    } else {
#pragma unroll
      for (int q = 0; q < BW4_SLOTS; ++q)
        if (b0 + q < B && a.status[b0 + q] == ILQR_TRAJ_OK) active |= 1u << q;
    }
  }
#if ILQR_FUSED_DEPHASE_PROBE
  // TIMING-ONLY probe (tools/archive/r05/dephase_probe.sh, not the product): half of the waves
  // (PROBE 1: odd waves of every workgroup; 2: odd workgroups) run the forward FIRST on
  // the gains already in K/d, then the backward — the phase mix of a de-phased schedule
  // (forward(i−1) then backward(i) beside backward(i) then forward(i)) at one wave/SIMD.
  // PROBE 3 is that schedule's first launch (odd waves: backward only), PROBE 4 its
  // drain launch (odd waves: forward only, even waves nothing).
  if (ILQR_FUSED_DEPHASE_PROBE == 3 && active != 0 && (w & 1)) {
    (void)lq_backward4_wave(P, b0, B, active, T, a.x, a.u, a.d, a.K, ls.mu, lds);
    return;
  }
  if (ILQR_FUSED_DEPHASE_PROBE == 4) {
    if (active != 0 && (w & 1))
      iter_forward_wave_active<12, 4>(P, b0, B, T, ai, ls, lds, ((active >> (l >> 4)) & 1u) != 0);
    return;
  }
  if (active != 0 && ((ILQR_FUSED_DEPHASE_PROBE != 2 ? w : (int)blockIdx.x) & 1)) {
    iter_forward_wave_active<12, 4>(P, b0, B, T, ai, ls, lds, ((active >> (l >> 4)) & 1u) != 0);
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    (void)lq_backward4_wave(P, b0, B, active, T, a.x, a.u, a.d, a.K, ls.mu, lds);
    return;
  }
#endif
  if (active != 0) {
    const unsigned nan = lq_backward4_wave(P, b0, B, active, T, a.x, a.u, a.d, a.K, ls.mu, lds) & active;
    if (owner && ((nan >> q) & 1u)) {
      a.status[b0 + q] = ILQR_TRAJ_NAN;  // reference: AssertionError at backward_pass.jl:353
      if (a.res_parity) a.res_parity[b0 + q] = a.parity;
    }
    // the gains this wave stored are what its forward streams in: every store complete,
    // and the LDS scratch free for the ring
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    const unsigned run = active & ~nan;
    if constexpr (MF)
      iter_forward_wave_mfma(P, b0, B, T, ai, ls, lds, run);
    else if (coop)
      own = iter_forward_wave_coop<12, 4>(P, b0, B, T, ai, ls, lds, ((run >> (l >> 4)) & 1u) != 0);
    else
      iter_forward_wave_active<12, 4>(P, b0, B, T, ai, ls, lds, ((run >> (l >> 4)) & 1u) != 0);
  }
  if (coop) lq_coop_search<12, 4>(P, B, T, ai, ls, lds, wid, b0, own);
}

}  // namespace

hipError_t launch_lq_iter_fused4(const LQParams& p, int B, int T, const IterArgs& a, const LSParams& ls,
                                 hipStream_t s, bool mfma) {
  if (B <= 0) return hipSuccess;
  const int per_wg = FUSED_WAVES * BW4_SLOTS;
  if (mfma)
    lq_iter_fused4_kernel<true><<<(B + per_wg - 1) / per_wg, 64 * FUSED_WAVES, 0, s>>>(p, B, T, a, ls);
  else
    lq_iter_fused4_kernel<false><<<(B + per_wg - 1) / per_wg, 64 * FUSED_WAVES, 0, s>>>(p, B, T, a, ls);
  return hipGetLastError();
}

int bw4_grid(int B) {
  const int per_wg = BW4_WAVES * BW4_SLOTS;
  return (B + per_wg - 1) / per_wg;
}

hipError_t launch_lq_backward4(const LQParams& p, int B, int T, const double* x, const double* u,
                               double* d, double* K, int32_t* status, double mu, hipStream_t s) {
  if (B <= 0) return hipSuccess;
  lq_backward4_kernel<<<bw4_grid(B), 256, 0, s>>>(p, B, T, x, u, d, K, status, mu);
  return hipGetLastError();
}

hipError_t launch_lq_iter_backward4(const LQParams& p, int B, int T, const IterArgs& a, double mu,
                                    hipStream_t s) {
  if (B <= 0) return hipSuccess;
  lq_iter_backward4_kernel<<<bw4_grid(B), 256, 0, s>>>(p, B, T, a, mu);
  return hipGetLastError();
}

}  // namespace ilqr

#ifdef ILQR_COOP_TRACE
// the trace build's records (ilqr_fwd_ring.h coop_trace): copies up to max_recs of them
// (4 words each) and resets the count; → the number copied, -1 on a HIP error
extern "C" int ilqr_debug_trace(unsigned long long* out, int max_recs) {
  unsigned n = 0;
  if (hipMemcpyFromSymbol(&n, HIP_SYMBOL(ilqr::g_trace_n), sizeof(n)) != hipSuccess) return -1;
  if (n > ilqr::COOP_TRACE_MAX) n = ilqr::COOP_TRACE_MAX;
  const unsigned m = n < (unsigned)max_recs ? n : (unsigned)max_recs;
  if (m && hipMemcpyFromSymbol(out, HIP_SYMBOL(ilqr::g_trace), sizeof(unsigned long long) * 4 * m) != hipSuccess)
    return -1;
  const unsigned z = 0;
  if (hipMemcpyToSymbol(HIP_SYMBOL(ilqr::g_trace_n), &z, sizeof(z)) != hipSuccess) return -1;
  return (int)m;
}
#endif
