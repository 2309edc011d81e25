// Forward pass + line search of the LQ family, four trajectories per wave with the
// per-step inputs streamed HBM → LDS (the "ring" forward), and the DPP
// mat-vec helpers it uses. Private header: included by ilqr_lq.hip (the forward and
// pipelined kernels) and ilqr_bw4.hip (the fused backward + forward iteration kernel).
#pragma once
#include <hip/hip_runtime.h>
#include <type_traits>

#include "../../include/ilqr.h"
#include "ilqr_internal.h"
#include "ilqr_device.h"

namespace ilqr {
namespace {

// Σ_k<16 bcast_k(src)·c[k]: src is broadcast from lane k of each 16-lane row
// (DPP64 row_newbcast, gfx90a+), 4 independent accumulators. `s_nop 4` covers the
// VALU→DPP and EXEC→DPP hazards for whatever the compiler scheduled in front.
__device__ __forceinline__ double dpp_dot16(double src, const double (&c)[16]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  asm("s_nop 4\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3)
      : [s] "v"(src), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]), [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]), [c11] "v"(c[11]), [c12] "v"(c[12]), [c13] "v"(c[13]), [c14] "v"(c[14]), [c15] "v"(c[15]));
  return (a0 + a1) + (a2 + a3);
}

// Σ_k<12 bcast_k(src)·c[k]: src is broadcast from lane k of each 16-lane row
// (DPP64 row_newbcast, gfx90a+), 4 independent accumulators. `s_nop 4` covers the
// VALU→DPP and EXEC→DPP hazards for whatever the compiler scheduled in front.
__device__ __forceinline__ double dpp_dot12(double src, const double (&c)[12]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  asm("s_nop 4\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3)
      : [s] "v"(src), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]), [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]), [c11] "v"(c[11]));
  return (a0 + a1) + (a2 + a3);
}

// dpp_dot16 in two parts with the same four accumulators and the same order per
// accumulator (a0: k = 0, 4, 8, 12; a1: 1, 5, 9, 13; …), so (a0 + a1) + (a2 + a3) after
// both parts is dpp_dot16's bits: the first 12 terms from `src` (lanes 0..11 of the
// row), the last 4 from `src2` (lanes 12..15), issued once src2 exists.
struct Acc4 {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  __device__ __forceinline__ double sum() const { return (a0 + a1) + (a2 + a3); }
};
__device__ __forceinline__ void dpp_acc16_head(Acc4& r, double src, const double (&c)[16]) {
  asm("s_nop 4\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c0] row_newbcast:0 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c1] row_newbcast:1 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c2] row_newbcast:2 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c3] row_newbcast:3 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c4] row_newbcast:4 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c5] row_newbcast:5 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c6] row_newbcast:6 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c7] row_newbcast:7 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c8] row_newbcast:8 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c9] row_newbcast:9 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c10] row_newbcast:10 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c11] row_newbcast:11 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(r.a0), [a1] "+v"(r.a1), [a2] "+v"(r.a2), [a3] "+v"(r.a3)
      : [s] "v"(src), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]), [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]), [c11] "v"(c[11]));
}
__device__ __forceinline__ void dpp_acc16_tail(Acc4& r, double src2, const double (&c)[16]) {
  asm("s_nop 4\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c12] row_newbcast:12 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c13] row_newbcast:13 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c14] row_newbcast:14 row_mask:0xf bank_mask:0xf\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c15] row_newbcast:15 row_mask:0xf bank_mask:0xf\n\t"
      : [a0] "+v"(r.a0), [a1] "+v"(r.a1), [a2] "+v"(r.a2), [a3] "+v"(r.a3)
      : [s] "v"(src2), [c12] "v"(c[12]), [c13] "v"(c[13]), [c14] "v"(c[14]), [c15] "v"(c[15]));
}

// dpp_dot16 for a block-diagonal row held in 12 registers: lanes 0..11 of each row
// (banks 0-2) take Σ_k<12 bcast_k(src)·c[k], lanes 12..15 (bank 3) Σ_m<4
// bcast_{12+m}(src)·c[m] — the same accumulators and order as dpp_dot16 on the
// zero-padded row [c[0..11] | 0] resp. [0 | c[0..3]].
__device__ __forceinline__ double dpp_dot16_bd(double src, const double (&c)[12]) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  asm("s_nop 4\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c0] row_newbcast:0 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c1] row_newbcast:1 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c2] row_newbcast:2 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c3] row_newbcast:3 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c4] row_newbcast:4 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c5] row_newbcast:5 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c6] row_newbcast:6 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c7] row_newbcast:7 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c8] row_newbcast:8 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c9] row_newbcast:9 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c10] row_newbcast:10 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c11] row_newbcast:11 row_mask:0xf bank_mask:0x7\n\t"
      "v_fmac_f64_dpp %[a0], %[s], %[c0] row_newbcast:12 row_mask:0xf bank_mask:0x8\n\t"
      "v_fmac_f64_dpp %[a1], %[s], %[c1] row_newbcast:13 row_mask:0xf bank_mask:0x8\n\t"
      "v_fmac_f64_dpp %[a2], %[s], %[c2] row_newbcast:14 row_mask:0xf bank_mask:0x8\n\t"
      "v_fmac_f64_dpp %[a3], %[s], %[c3] row_newbcast:15 row_mask:0xf bank_mask:0x8\n\t"
      : [a0] "+v"(a0), [a1] "+v"(a1), [a2] "+v"(a2), [a3] "+v"(a3)
      : [s] "v"(src), [c0] "v"(c[0]), [c1] "v"(c[1]), [c2] "v"(c[2]), [c3] "v"(c[3]), [c4] "v"(c[4]), [c5] "v"(c[5]), [c6] "v"(c[6]), [c7] "v"(c[7]), [c8] "v"(c[8]), [c9] "v"(c[9]), [c10] "v"(c[10]), [c11] "v"(c[11]));
  return (a0 + a1) + (a2 + a3);
}

// Cache policy of the ring forward's memory traffic (measured, round 2): the slot loads
// carry a " nt" hint on the first load alone (64 of the step's 96 K-row chunks, read
// once, dead after the step: forward 52.6 → 48.9 µs at B = 4096, bench 6,530 → 6,650
// batched it/s, profiles/r02/bench_ab_k_nt.log); on all three loads it cost 10 µs (the
// x_traj = NULL re-reads of x then miss), nt/sc0/sc1 result stores were slower and a
// slot layout with both K loads pure and hinted measured 52.6 µs. Row broadcasts
// through LDS instead of DPP gave the same bits and measured slower. (These alternates
// and the forward's timing-only ablations live in tools/ablation/restore_alternates.patch.)
#define ILQR_FW_LDS_OP1 "global_load_lds_dwordx4 %0, off nt"
#define ILQR_FW_LDS_OP "global_load_lds_dwordx4 %0, off"

struct FwdOut {
  double cost;
  int trials;
  int accepted;  // 1 accepted, 0 exhausted / NaN
  bool eo;       // candidate pass: α·δu vanished at every step (see CandPass)
};

// One CANDIDATE pass of the cooperative line search (lq_coop_search below): the wave's
// four groups roll out the SAME trajectory, each at its own α (trial j's α, formed by
// the reference's repeated `α *= shrink`, :82), once, with the sequential search's
// arithmetic and order — so a candidate's cost is bit for bit that trial's cost. Only
// the group `store_group` stores its rollout (−1: none). Each group also reports `eo`:
// fma(α, δuₖ, uₖ) == uₖ at every step. Then every later trial j' > j rolls out
// identically (exact: α' ≤ α and rounding is monotone, so fma(α', δu, u) rounds to u as
// well, every ūₖ = uₖ + Kₖδxₖ is the same and so is the whole rollout), i.e. once such
// a trial is rejected the search of forward_pass.jl:70-87 capped at max_trials ends
// exhausted with that rollout and cost.
struct CandPass {
  double alpha;     // this lane's group's α
  int store_group;  // group that stores its rollout into x_new/u_new of the trajectory
  // scratch rollouts (LSCoop::sx / su, byte sizes): when set, EVERY group stores its
  // rollout there, group g at trial index sidx + g, instead of into x_new / u_new
  double* sx = nullptr;
  double* su = nullptr;
  int sidx = 0;
  uint32_t sx_bytes = 0, su_bytes = 0;
};


// Forward pass of a wave's four trajectories b0 .. b0+3 (contiguous) with the per-step
// inputs streamed HBM → LDS by the wave itself (global_load_lds_dwordx4, no VGPRs
// held in flight) PF steps ahead into a ring of R slots. Same lane roles and the
// same arithmetic in the same order as lq_forward_group — bit-identical results —
// but ≈100 VGPRs instead of ≈250 and a deeper prefetch: it runs inside kernels that
// also run the backward pass (128 VGPRs at 4 waves/SIMD). Called by the WHOLE wave
// (every lane produces a slice of every group's inputs); `active` masks the groups
// that compute, and the line-search loop is uniform (a group that accepted stops
// storing). One slot (3 KB): K rows [0,192), x [192,240), u [240,256), x_traj
// [256,304), δu [304,320) doubles; group g at K + 48g, x/x_traj + 12g, u/δu + 4g.
constexpr int RING_SLOT = 384;  // doubles per ring slot
// Q, R of the wave's 4 trajectories (+ read overhang), then four 64-double vectors of
// scratch (unused since the LDS row broadcasts went; kept so the kernels' LDS size and
// occupancy stay those measured)
constexpr int RING_LAREA = 4 * 160 + 16 + 4 * 64;

// LR_REGS: the wave's Q/R cost rows live in registers for the whole pass (kernels with
// one wave per SIMD and VGPRs to spare); otherwise they are re-read from LDS every step
// (the pipelined kernel's 128-VGPR budget). An LDS read in the step is a wait the
// in-order wave cannot issue past.
//
// CAND: one candidate pass (CandPass above) of trajectory b0 in all four groups — no
// search loop; the result is this group's cost, du2 and eo.
template <int NX, int NU, int R, int PF, bool LR_REGS = true, bool CAND = false>
__device__ FwdOut lq_forward_wave_ring(const LQParams& P, int b0, int B, int T, bool active,
                                       const double* __restrict__ x, const double* __restrict__ u,
                                       const double* __restrict__ xtraj, const double* __restrict__ dg,
                                       const double* __restrict__ Kg, double prev_cost,
                                       double* __restrict__ xnew, double* __restrict__ unew,
                                       double* du2_out, const LSParams& ls, double* ring,
                                       const CandPass& cand = CandPass{0.0, -1}) {
  static_assert(NX == 12 && NU == 4, "slot layout and lane map are written for nx = 12, nu = 4");
  static_assert(R > PF && PF >= 1, "the slot being refilled must not be the one being read");
  constexpr uint32_t OOR = 0x80000000u;
  // wave-uniform in an SGPR: the result stores' buffer resources derive from it (a VGPR
  // resource makes every store a readfirstlane waterfall loop)
  b0 = __builtin_amdgcn_readfirstlane(b0);
  const int l = threadIdx.x & 63;
  const int g = l >> 4;
  const int j = l & 15;
  const bool is_x = j < NX;
  const bool is_u = !is_x;
  const int iu = is_u ? j - NX : 0;
  const int jx = is_x ? j : 0;
  // trajectories present in this wave (a candidate pass: one, in every group)
  const int nt = CAND ? 1 : (B - b0 < 4 ? B - b0 : 4);
  const int b = b0 + (g < nt ? g : 0);     // absent groups alias trajectory b0 (never stored)

  const double* Ab = P.A + (size_t)b * NX * NX;
  const double* Bb = P.B + (size_t)b * NX * NU;
  const double* Qfb = P.Qf + (size_t)b * NX * NX;
  double Fr[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double a = ldz(is_x && k < NX, Ab + jx * NX + (k < NX ? k : 0), Ab);
    const double bb = ldz(is_x && k >= NX, Bb + jx * NU + (k >= NX ? k - NX : 0), Bb);
    Fr[k] = a + bb;
  }
  // the cost Hessian rows live in LDS after the ring (re-read every step: registers
  // are the scarce resource): trajectory g's Q at 160g, R at 160g + 144
  double* const Ls = ring + R * RING_SLOT;
  for (int i = l; i < 4 * 160; i += 64) {
    const int gg = i / 160, e = i % 160;
    const size_t bt = (size_t)b0 + (gg < nt ? gg : 0);
    Ls[i] = e < NX * NX ? P.Q[bt * NX * NX + e] : P.R[bt * NU * NU + (e < NX * NX ? 0 : e - NX * NX)];
  }
  const int la = is_x ? g * 160 + jx * NX : g * 160 + NX * NX + iu * NU;  // this lane's L row
  double Lk[NX];  // the cost row in registers (LR_REGS)
  if constexpr (LR_REGS) {
    const double2* lr = reinterpret_cast<const double2*>(Ls + la);
#pragma unroll
    for (int k = 0; k < NX / 2; ++k) {
      const double2 q = lr[k];
      Lk[2 * k] = q.x;
      Lk[2 * k + 1] = q.y;
    }
  }
  wave_lds_fence();

  // producer: lane l moves 16 B per instruction; three instructions fill one slot
  //   #1: K chunk l (of 96)   #2: K chunk 64+l | x chunk l−32 | u chunk l−56
  //   #3: x_traj chunk l | δu chunk l−24 | (lanes 32..63 repeat lanes 0..31)
  // A candidate pass rolls out ONE trajectory in all four groups: one instruction fills
  // the slot's first 40 chunks with its step (K 0..23, x 24..29, u 30..31, x_traj 32..37,
  // δu 38..39; lanes 40..63 repeat lanes 0..23 past them) and every group reads those.
  auto tr = [&](int gg) { return (size_t)(b0 + (gg < nt ? gg : 0)); };
  const double* xt0 = xtraj ? xtraj : x;  // x_traj = NULL: read x with weight 0
  const double xtw = xtraj ? 1.0 : 0.0;
  const char *p1, *p2, *p3;
  uint32_t s1, s2, s3;  // bytes per step
  if constexpr (CAND) {
    const int c = l < 40 ? l : l - 40;
    if (c < 24) {
      p1 = reinterpret_cast<const char*>(Kg + tr(0) * T * NU * NX + 2 * c);
      s1 = NU * NX * 8;
    } else if (c < 30) {
      p1 = reinterpret_cast<const char*>(x + tr(0) * (T + 1) * NX + 2 * (c - 24));
      s1 = NX * 8;
    } else if (c < 32) {
      p1 = reinterpret_cast<const char*>(u + tr(0) * T * NU + 2 * (c - 30));
      s1 = NU * 8;
    } else if (c < 38) {
      p1 = reinterpret_cast<const char*>(xt0 + tr(0) * (T + 1) * NX + 2 * (c - 32));
      s1 = NX * 8;
    } else {
      p1 = reinterpret_cast<const char*>(dg + tr(0) * T * NU + 2 * (c - 38));
      s1 = NU * 8;
    }
    p2 = p3 = p1;
    s2 = s3 = s1;
  } else {
    const int c = l;
    p1 = reinterpret_cast<const char*>(Kg + tr(c / 24) * T * NU * NX + 2 * (c % 24));
    s1 = NU * NX * 8;
    if (l < 32) {
      const int c2 = 64 + l;
      p2 = reinterpret_cast<const char*>(Kg + tr(c2 / 24) * T * NU * NX + 2 * (c2 % 24));
      s2 = NU * NX * 8;
    } else if (l < 56) {
      const int m = l - 32;
      p2 = reinterpret_cast<const char*>(x + tr(m / 6) * (T + 1) * NX + 2 * (m % 6));
      s2 = NX * 8;
    } else {
      const int m = l - 56;
      p2 = reinterpret_cast<const char*>(u + tr(m / 2) * T * NU + 2 * (m % 2));
      s2 = NU * 8;
    }
    const int l3 = l & 31;
    if (l3 < 24) {
      p3 = reinterpret_cast<const char*>(xt0 + tr(l3 / 6) * (T + 1) * NX + 2 * (l3 % 6));
      s3 = NX * 8;
    } else {
      const int m = l3 - 24;
      p3 = reinterpret_cast<const char*>(dg + tr(m / 2) * T * NU + 2 * (m % 2));
      s3 = NU * 8;
    }
  }
  const uint32_t ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)ring;
  auto produce = [&](int t) {
    uint32_t tt = (uint32_t)(t < T ? t : T - 1);  // clamped: loaded, never read
    asm volatile("" : "+s"(tt));  // no hoisting of the prologue's addresses out of the trial loop
    const uint32_t m0 = ring_lds + (uint32_t)((t % R) * RING_SLOT * 8);
    asm volatile(ILQR_FW_LDS_OP1 ::"v"(p1 + (size_t)tt * s1), "{m0}"(m0) : "memory");
    if constexpr (!CAND) {
      asm volatile(ILQR_FW_LDS_OP ::"v"(p2 + (size_t)tt * s2), "{m0}"(m0 + 1024) : "memory");
      asm volatile(ILQR_FW_LDS_OP ::"v"(p3 + (size_t)tt * s3), "{m0}"(m0 + 2048) : "memory");
    }
  };
  // vmcnt immediates (gfx9: vmcnt[3:0] | expcnt 7 << 4 | lgkmcnt 15 << 8 | vmcnt[5:4] << 14):
  // per step the wave issues NL slot loads then 2 result stores, so slot t is
  // complete once ≤ (NL + 2)·PF − NL ops are outstanding (≤ NL·PF − NL while the
  // prologue loads are the newest)
  constexpr int NL = CAND ? 1 : 3;
  constexpr int N_SS = (NL + 2) * PF - NL, N_PRO = NL * PF - NL;
  auto wait_slot = [](auto n) {
    constexpr int v = decltype(n)::value;
    static_assert(v >= 0 && v < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((v & 15) | (7 << 4) | (15 << 8) | ((v >> 4) << 14));
    asm volatile("" ::: "memory");
  };

  // K row of (g, iu); x (x lanes) / u (u lanes); x_traj / δu — a candidate pass's slot
  // holds its one trajectory's step at the front (producer above)
  const int ka = CAND ? iu * NX : g * 48 + iu * NX;
  const int va = CAND ? (is_x ? 48 + jx : 60 + iu) : (is_x ? 192 + g * 12 + jx : 240 + g * 4 + iu);
  const int vb = CAND ? (is_x ? 64 + jx : 76 + iu) : (is_x ? 256 + g * 12 + jx : 304 + g * 4 + iu);
  // the resources' words made provably wave-uniform (the candidate passes run inside
  // the cooperative search's loops, where the compiler loses track of it: a divergent
  // resource is a readfirstlane waterfall loop around every store)
  const bool scr = CAND && cand.sx != nullptr;  // wave-uniform
  const auto rXN = scr ? buffer_rsrc(uniform_ptr(cand.sx), (uint32_t)__builtin_amdgcn_readfirstlane(cand.sx_bytes))
                       : buffer_rsrc(uniform_ptr(xnew + (size_t)b0 * (T + 1) * NX),
                                     (uint32_t)__builtin_amdgcn_readfirstlane(nt * (T + 1) * NX * 8));
  const auto rUN = scr ? buffer_rsrc(uniform_ptr(cand.su), (uint32_t)__builtin_amdgcn_readfirstlane(cand.su_bytes))
                       : buffer_rsrc(uniform_ptr(unew + (size_t)b0 * T * NU),
                                     (uint32_t)__builtin_amdgcn_readfirstlane(nt * T * NU * 8));
  // this group's rollout within the stored span: its trajectory (g), the candidate pass's
  // one trajectory (0), or its trial's scratch slot
  const int gs = scr ? cand.sidx + g : (CAND ? 0 : g);
  const uint32_t oxs = is_x ? (uint32_t)(gs * (T + 1) * NX + jx) * 8 : OOR;
  const uint32_t ous = is_u ? (uint32_t)(gs * T * NU + iu) * 8 : OOR;

  double alpha = CAND ? cand.alpha : ls.alpha0;
  FwdOut out{INFINITY, 0, 0, false};
  bool open = active;  // still line-searching
  double du2_acc = 0.0;
  const int trials_max = CAND ? 1 : ls.max_trials;
  for (int trial = 1; trial <= trials_max && __any(open); ++trial) {
#pragma unroll
    for (int t = 0; t < PF; ++t) produce(t);
    double cost = 0.0, du2 = 0.0;
    bool eo = true;  // CAND: fma(α, δuₖ, uₖ) == uₖ so far (u lanes)
    const bool st = open && (!CAND || scr || g == cand.store_group);
    const uint32_t ox = st ? oxs : OOR, ou = st ? ous : OOR;  // closed groups store nothing
    // slot t's operands are read into registers at the end of step t − 1 (software
    // pipelining of the LDS reads: their latency is off the step's dependent chain)
    struct Slot {
      double a, bq, Kr[NX];
    };
    auto read_slot = [&](int t, Slot& o) {
      const double* sl = ring + (t % R) * RING_SLOT;
      o.a = sl[va];
      o.bq = sl[vb];
      const double2* kr = reinterpret_cast<const double2*>(sl + ka);
#pragma unroll
      for (int k = 0; k < NX / 2; ++k) {
        const double2 v = kr[k];
        o.Kr[2 * k] = v.x;
        o.Kr[2 * k + 1] = v.y;
      }
    };
    Slot cur;
    wait_slot(std::integral_constant<int, N_PRO>{});
    read_slot(0, cur);
    double xb = is_x ? cur.a : 0.0;  // x̄₁ = x₁ (:65)
    auto step = [&](int t, auto next_wait) {
      // x̄ₖ₊₁ = A x̄ₖ + B ūₖ: the A part (broadcasts from the x lanes) does not need ūₖ
      Acc4 xa;
      dpp_acc16_head(xa, xb, Fr);
      // δx = x̄ₖ − xₖ (:72); ūₖ = uₖ + α δuₖ + Kₖ δx (:73)
      const double dx = is_x ? xb - cur.a : 0.0;
      const double kdx = dpp_dot12(dx, cur.Kr);
      const double ua = fma(alpha, cur.bq, cur.a);
      const double ub = ua + kdx;
      if constexpr (CAND) eo = eo && (is_x || ua == cur.a);
      const double z = is_x ? xb : ub;
      const double v = is_x ? fma(-xtw, cur.bq, xb) : ub;
      const double e = is_x ? 0.0 : ub - cur.a;
      dpp_acc16_tail(xa, ub, Fr);  // the B part: broadcasts from the u lanes
      produce(t + PF);  // slot (t+PF)%R was last read at step t+PF−R < t
      double Lr[NX];  // Q row (x lanes); R row in slots 0..NU-1 (u lanes), rest unused
      if constexpr (LR_REGS) {
#pragma unroll
        for (int k = 0; k < NX; ++k) Lr[k] = Lk[k];
      } else {
        const double2* lr = reinterpret_cast<const double2*>(Ls + la);
#pragma unroll
        for (int k = 0; k < NX / 2; ++k) {
          const double2 q = lr[k];
          Lr[2 * k] = q.x;
          Lr[2 * k + 1] = q.y;
        }
      }
      const double lv = dpp_dot16_bd(v, Lr);
      cost = fma(v, lv, cost);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, z), rXN, ox, (uint32_t)t * NX * 8, 0);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, z), rUN, ou, (uint32_t)t * NU * 8, 0);
      du2 = fma(e, e, du2);
      xb = xa.sum();
      // slot t + 1 (past the horizon: a clamped step's slot, read and never used)
      wait_slot(next_wait);
      read_slot(t + 1, cur);
    };
    const int tp = T < PF ? T : PF;
    for (int t = 0; t < tp - 1; ++t) step(t, std::integral_constant<int, N_PRO>{});
    for (int t = tp - 1; t < T; ++t) step(t, std::integral_constant<int, N_SS>{});
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xb), rXN, ox, (uint32_t)T * NX * 8, 0);
    // Qf row (x lanes; u lanes read row 0 and zero it): one base address, 6 × 16 B
    const double2* qrow = reinterpret_cast<const double2*>(Qfb + jx * NX);
    asm volatile("" : "+v"(qrow));  // keep the row address from being hoisted as 12 pointers
    double Qfr[NX];
#pragma unroll
    for (int k = 0; k < NX / 2; ++k) {
      const double2 q = qrow[k];
      Qfr[2 * k] = is_x ? q.x : 0.0;
      Qfr[2 * k + 1] = is_x ? q.y : 0.0;
    }
    const double lf = dpp_dot12(is_x ? xb : 0.0, Qfr);
    cost = fma(is_x ? xb : 0.0, lf, cost);
    cost = rowsum16(cost);
    du2 = rowsum16(du2);
    if constexpr (CAND) {
      const uint64_t bad = __ballot(!eo);
      out.eo = ((bad >> (16 * g)) & 0xFFFFull) == 0;
      out.trials = 1;
      out.cost = cost;
      du2_acc = du2;
      __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));
      asm volatile("" ::: "memory");
      break;
    }
    if (open) {
      out.trials = trial;
      out.cost = cost;
      du2_acc = du2;
      if (prev_cost - cost > 0.0) {  // (:77-80); NaN compares false → keep searching
        out.accepted = 1;
        open = false;
      }
    }
    alpha *= ls.shrink;  // (:82); unused by closed groups
    // the loads of the clamped steps past the horizon (and the read of slot T) are
    // still in flight: drain them before the next trial's prologue reuses the slots
    __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));
    asm volatile("" ::: "memory");
  }
  if (du2_out) *du2_out = du2_acc;
  return out;
}

// ---------------------------------------------------------------------------
// The WIDE candidate pass (round 6, the cooperative search's default: ILQR_COOP_WIDTH).
// Sixteen trials of ONE trajectory per wave instead of four: trial τ = lane & 15 runs on
// the four lanes ρ = lane >> 4, lane ρ owning rows 3ρ..3ρ+2 of x̄ and row ρ of ū. Each
// row is computed with the row form's arithmetic in the row form's order — the same
// four accumulators per dot product (term k into accumulator k mod 4, k ascending, the
// x̄ part before the ū part), the same (a0 + a1) + (a2 + a3), the same per-row cost and
// Σ(ū − u)² accumulators and, at the end, rowsum16's butterfly over the sixteen rows —
// so a trial's rollout, cost, Σ(ū − u)² and `eo` are bit for bit the row form's
// (lq_forward_wave_ring<CAND>) and the sequential search's. What changes is how the
// operands meet: the row form broadcasts x̄ₖ and ūₘ from their lanes with DPP
// (row_newbcast, the only f64 DPP mode: one trial per 16-lane row); here the rows of a
// trial exchange x̄, δx = x̄ − x, v = x̄ − x_traj and ū through the LDS (ds_write_b64 by
// the owner, ds_read_b128 by the trial's four lanes; in-order LDS within the wave, no
// barrier), and each lane keeps its three [A | B] and Q rows in registers. Per step and
// lane ≈150 VALU ops for sixteen trials against ≈140 for four in the row form.
// Exchange area (the ring's LAREA, unused by a candidate pass): per trial C16_ES
// doubles, x̄ [0,12), δx [12,24), v [24,36), ū [36,40); stride 42 doubles puts the
// sixteen trials of a ds_read_b128 lane group on sixteen different 4-bank quarters.
constexpr int C16_ES = 42;
static_assert(16 * C16_ES <= RING_LAREA, "the exchange area fits the ring's LAREA");
struct Cand16 {
  double cost, du2;
  bool eo;  // fma(α, δuₖ, uₖ) == uₖ at every step (CandPass)
};

// `alpha`: this lane's trial's α. `st`: this lane's trial stores its rollout through rXN /
// rUN at rollout index gs (x̄ (T+1)·12, ū T·4 doubles per rollout). Whole wave.
// STORE = false: no lane stores its rollout (a pass neither at trial 2 nor on a scratch
// row), and the pass issues no store instructions at all — a pass that issues them, even
// out of range, runs measurably slower (the memory pipeline takes every lane's address)
template <int R, int PF, bool STORE>
__device__ Cand16 lq_cand16_pass(const LQParams& P, int b, int T, const double* __restrict__ x,
                                 const double* __restrict__ u, const double* __restrict__ xtraj,
                                 const double* __restrict__ dg, const double* __restrict__ Kg, double alpha, bool st,
                                 __amdgpu_buffer_rsrc_t rXN, __amdgpu_buffer_rsrc_t rUN, int gs, double* ring) {
  constexpr int NX = 12, NU = 4;
  static_assert(R > PF && PF >= 1, "the slot being refilled must not be the one being read");
  constexpr uint32_t OOR = 0x80000000u;
  b = __builtin_amdgcn_readfirstlane(b);
  const int l = threadIdx.x & 63;
  const int r = l >> 4;   // rows 3r .. 3r+2 of x̄, row r of ū
  const int tt = l & 15;  // the trial

  // this lane's rows: [A | B] as the row form's Fr (A + 0, 0 + B) and R in registers;
  // Q in slot 0's tail, doubles [QO, QO + 144), read per step: the candidate producer's
  // one load per step writes a slot's first 128 doubles (lanes 40..63 repeat the K
  // chunks of lanes 0..23 into [80, 128)) and nothing past them
  constexpr int QO = 128;
  static_assert(QO >= 128 && QO + NX * NX <= RING_SLOT, "Q fits slot 0's tail, past the producer's 64 chunks");
  double F[3][16], Rr[NU];
#ifndef ILQR_CAND16_QREG  // 1: Q rows in registers (iteration 5: 540-553 → 518-530 µs), 0: from the slot
#define ILQR_CAND16_QREG 1
#endif
  double Qr[ILQR_CAND16_QREG ? 3 : 1][NX];  // Q rows in registers (ILQR_CAND16_QREG), else LDS
  {
    const double* Ab = P.A + (size_t)b * NX * NX;
    const double* Bb = P.B + (size_t)b * NX * NU;
    const double* Qb = P.Q + (size_t)b * NX * NX;
    const double2* rr = reinterpret_cast<const double2*>(P.R + (size_t)b * NU * NU + r * NU);
    if constexpr (!ILQR_CAND16_QREG)
      for (int i = l; i < NX * NX; i += 64) ring[QO + i] = Qb[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double2* ar = reinterpret_cast<const double2*>(Ab + (3 * r + i) * NX);
      const double2* br = reinterpret_cast<const double2*>(Bb + (3 * r + i) * NU);
      const double2* qr = reinterpret_cast<const double2*>(Qb + (3 * r + i) * NX);
#pragma unroll
      for (int k = 0; k < NX / 2; ++k) {
        const double2 a2 = ar[k];
        F[i][2 * k] = a2.x + 0.0;
        F[i][2 * k + 1] = a2.y + 0.0;
        if constexpr (ILQR_CAND16_QREG) {
          const double2 q2 = qr[k];
          Qr[i][2 * k] = q2.x;
          Qr[i][2 * k + 1] = q2.y;
        }
      }
#pragma unroll
      for (int m = 0; m < NU / 2; ++m) {
        const double2 b2 = br[m];
        F[i][NX + 2 * m] = 0.0 + b2.x;
        F[i][NX + 2 * m + 1] = 0.0 + b2.y;
      }
    }
#pragma unroll
    for (int m = 0; m < NU / 2; ++m) {
      const double2 r2 = rr[m];
      Rr[2 * m] = r2.x;
      Rr[2 * m + 1] = r2.y;
    }
  }
  // the ring's loads below are inline asm, invisible to the compiler's wait counting:
  // every constant is in its register before the first of them
  __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");

  // producer: the candidate pass's one instruction per step (lq_forward_wave_ring<CAND>):
  // K 0..23, x 24..29, u 30..31, x_traj 32..37, δu 38..39 (chunks of 16 B)
  const double* xt0 = xtraj ? xtraj : x;  // x_traj = NULL: read x with weight 0
  const double xtw = xtraj ? 1.0 : 0.0;
  const char* p1;
  uint32_t s1;
  {
    const int c = l < 40 ? l : l - 40;
    const size_t bb = (size_t)b;
    if (c < 24) {
      p1 = reinterpret_cast<const char*>(Kg + bb * T * NU * NX + 2 * c);
      s1 = NU * NX * 8;
    } else if (c < 30) {
      p1 = reinterpret_cast<const char*>(x + bb * (T + 1) * NX + 2 * (c - 24));
      s1 = NX * 8;
    } else if (c < 32) {
      p1 = reinterpret_cast<const char*>(u + bb * T * NU + 2 * (c - 30));
      s1 = NU * 8;
    } else if (c < 38) {
      p1 = reinterpret_cast<const char*>(xt0 + bb * (T + 1) * NX + 2 * (c - 32));
      s1 = NX * 8;
    } else {
      p1 = reinterpret_cast<const char*>(dg + bb * T * NU + 2 * (c - 38));
      s1 = NU * 8;
    }
  }
  const uint32_t ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)ring;
  auto produce = [&](int t) {
    uint32_t tq = (uint32_t)(t < T ? t : T - 1);  // clamped: loaded, never read
    asm volatile("" : "+s"(tq));
    const uint32_t m0 = ring_lds + (uint32_t)((t % R) * RING_SLOT * 8);
    asm volatile(ILQR_FW_LDS_OP1 ::"v"(p1 + (size_t)tq * s1), "{m0}"(m0) : "memory");
  };
  // per step: one slot load, then four result stores (three x̄ rows, one ū row) if STORE
  constexpr int NL = 1, NS = STORE ? 4 : 0;
  constexpr int N_SS = (NL + NS) * PF - NL, N_PRO = NL * PF - NL;
  auto wait_slot = [](auto n) {
    constexpr int v = decltype(n)::value;
    static_assert(v >= 0 && v < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((v & 15) | (7 << 4) | (15 << 8) | ((v >> 4) << 14));
    asm volatile("" ::: "memory");
  };
  // slot offsets (doubles): K row m at 12m, x 48, u 60, x_traj 64, δu 76
  constexpr int SX = 48, SU = 60, SXT = 64, SD = 76;

  double* const my = ring + R * RING_SLOT + tt * C16_ES;  // this trial's exchange row
  const uint32_t oxs = st ? (uint32_t)(gs * (T + 1) * NX + 3 * r) * 8 : OOR;
  const uint32_t ous = st ? (uint32_t)(gs * T * NU + r) * 8 : OOR;
  auto rd12 = [](const double* p, double (&v)[NX]) {
    const double2* q = reinterpret_cast<const double2*>(p);
#pragma unroll
    for (int k = 0; k < NX / 2; ++k) {
      const double2 w = q[k];
      v[2 * k] = w.x;
      v[2 * k + 1] = w.y;
    }
  };
  // Σ_k<12 v[k]·c[k], accumulator k mod 4, (a0 + a1) + (a2 + a3): dpp_dot12's order
  auto dot12 = [](const double (&v)[NX], const double* c) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
    for (int k = 0; k < NX; k += 4) {
      a0 = fma(v[k], c[k], a0);
      a1 = fma(v[k + 1], c[k + 1], a1);
      a2 = fma(v[k + 2], c[k + 2], a2);
      a3 = fma(v[k + 3], c[k + 3], a3);
    }
    return (a0 + a1) + (a2 + a3);
  };

#pragma unroll
  for (int t = 0; t < PF; ++t) produce(t);
  wait_slot(std::integral_constant<int, N_PRO>{});
  double xo[3], vo[3];  // this lane's rows of x̄ₖ and vₖ = x̄ₖ − x_trajₖ
  {
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double xk = ring[SX + 3 * r + i];
      xo[i] = xk;  // x̄₁ = x₁ (:65)
      vo[i] = fma(-xtw, ring[SXT + 3 * r + i], xo[i]);
      my[3 * r + i] = xo[i];
      my[NX + 3 * r + i] = xo[i] - xk;
      my[2 * NX + 3 * r + i] = vo[i];
    }
  }
  wave_lds_fence();
  double cost[3] = {0.0, 0.0, 0.0}, costu = 0.0, du2 = 0.0;
  bool eo = true;
  auto step = [&](int t, auto next_wait) {
    const double* sl = ring + (t % R) * RING_SLOT;
    // ūₖ row r = uₖ + α δuₖ + Kₖ δx (:72-73)
    double Kr[NX], DX[NX];
    rd12(sl + NX * r, Kr);
    rd12(my + NX, DX);
    const double urk = sl[SU + r], durk = sl[SD + r];
    const double kdx = dot12(DX, Kr);
    const double ua = fma(alpha, durk, urk);
    const double ub = ua + kdx;
    eo = eo && (ua == urk);
    const double e = ub - urk;
    du2 = fma(e, e, du2);
    my[3 * NX + r] = ub;
    // x̄ₖ₊₁ = A x̄ₖ + B ūₖ (:74): the A part first, it does not need ūₖ
    double XB[NX];
    rd12(my, XB);
    double acc[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0.0;
#pragma unroll
    for (int k = 0; k < NX; ++k)
#pragma unroll
      for (int i = 0; i < 3; ++i) acc[i][k & 3] = fma(XB[k], F[i][k], acc[i][k & 3]);
    // ℓ(x̄ₖ − x_trajₖ, ·) rows (:187-190): vᵀ(Q row)
    double V[NX];
    rd12(my + 2 * NX, V);
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      if constexpr (ILQR_CAND16_QREG) {
        cost[i] = fma(vo[i], dot12(V, Qr[i]), cost[i]);
      } else {
        double qr[NX];
        rd12(ring + QO + (3 * r + i) * NX, qr);
        cost[i] = fma(vo[i], dot12(V, qr), cost[i]);
      }
    }
    produce(t + PF);  // slot (t+PF)%R was last read at step t+PF−R < t
    wave_lds_fence();  // ū of every row written before it is read
    double U4[NU];
    {
      const double2* q = reinterpret_cast<const double2*>(my + 3 * NX);
      const double2 w0 = q[0], w1 = q[1];
      U4[0] = w0.x;
      U4[1] = w0.y;
      U4[2] = w1.x;
      U4[3] = w1.y;
    }
#pragma unroll
    for (int m = 0; m < NU; ++m)
#pragma unroll
      for (int i = 0; i < 3; ++i) acc[i][m] = fma(U4[m], F[i][NX + m], acc[i][m]);
    // the ū row's cost: ūᵀ(R row) with one accumulator per term (dpp_dot16_bd's bank 3)
    const double lvu = (fma(U4[0], Rr[0], 0.0) + fma(U4[1], Rr[1], 0.0)) +
                       (fma(U4[2], Rr[2], 0.0) + fma(U4[3], Rr[3], 0.0));
    costu = fma(ub, lvu, costu);
    if constexpr (STORE) {
#pragma unroll
      for (int i = 0; i < 3; ++i)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xo[i]), rXN, oxs,
                                              (uint32_t)(t * NX + i) * 8, 0);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, ub), rUN, ous, (uint32_t)t * NU * 8, 0);
    }
    double xn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) xn[i] = (acc[i][0] + acc[i][1]) + (acc[i][2] + acc[i][3]);
    // slot t + 1 (past the horizon: a clamped step's slot, read and never used)
    wait_slot(next_wait);
    const double* sn = ring + ((t + 1) % R) * RING_SLOT;
    double dn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      dn[i] = xn[i] - sn[SX + 3 * r + i];
      vo[i] = fma(-xtw, sn[SXT + 3 * r + i], xn[i]);
      xo[i] = xn[i];
    }
    wave_lds_fence();  // this step's reads of the exchange row issued before its overwrite
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      my[3 * r + i] = xo[i];
      my[NX + 3 * r + i] = dn[i];
      my[2 * NX + 3 * r + i] = vo[i];
    }
    wave_lds_fence();
  };
  const int tp = T < PF ? T : PF;
  for (int t = 0; t < tp - 1; ++t) step(t, std::integral_constant<int, N_PRO>{});
  for (int t = tp - 1; t < T; ++t) step(t, std::integral_constant<int, N_SS>{});
  if constexpr (STORE) {
#pragma unroll
    for (int i = 0; i < 3; ++i)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xo[i]), rXN, oxs, (uint32_t)(T * NX + i) * 8,
                                            0);
  }
  // final_cost(x̄_N) = x̄ᵀQf x̄ on the raw state (:192): the rows' Qf dots; the ū rows
  // take the row form's 0·(x̄ · 0) (a NaN state stays NaN there as well)
  {
    double XB[NX];
    rd12(my, XB);
    const double* Qfb = P.Qf + (size_t)b * NX * NX;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double qf[NX];
      rd12(Qfb + (3 * r + i) * NX, qf);
      cost[i] = fma(xo[i], dot12(XB, qf), cost[i]);
    }
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    const double z = 0.0;
#pragma unroll
    for (int k = 0; k < NX; k += 4) {
      a0 = fma(XB[k], z, a0);
      a1 = fma(XB[k + 1], z, a1);
      a2 = fma(XB[k + 2], z, a2);
      a3 = fma(XB[k + 3], z, a3);
    }
    costu = fma(z, (a0 + a1) + (a2 + a3), costu);
  }
  // rowsum16 over the trial's sixteen rows (x̄ rows 0..11, ū rows 12..15): lane 0's
  // butterfly (xor 8, 4, 2, 1) is (((c0+c8)+(c4+c12)) + ((c2+c10)+(c6+c14))) +
  // (((c1+c9)+(c5+c13)) + ((c3+c11)+(c7+c15))), and every lane of the row ends equal
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    my[3 * r + i] = cost[i];
    my[16 + 3 * r + i] = 0.0;  // the x̄ rows' Σ(ū − u)²: fma(0, 0, ·) from 0
  }
  my[12 + r] = costu;
  my[16 + 12 + r] = du2;
  wave_lds_fence();
  auto tree16 = [](const double* c) {
    return (((c[0] + c[8]) + (c[4] + c[12])) + ((c[2] + c[10]) + (c[6] + c[14]))) +
           (((c[1] + c[9]) + (c[5] + c[13])) + ((c[3] + c[11]) + (c[7] + c[15])));
  };
  double cs[16], ds[16];
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    const double2 w = *reinterpret_cast<const double2*>(my + k);
    const double2 v = *reinterpret_cast<const double2*>(my + 16 + k);
    cs[k] = w.x;
    cs[k + 1] = w.y;
    ds[k] = v.x;
    ds[k + 1] = v.y;
  }
  Cand16 out;
  out.cost = tree16(cs);
  out.du2 = tree16(ds);
  const uint64_t bad = __ballot(!eo);
  out.eo = ((bad | (bad >> 16) | (bad >> 32) | (bad >> 48)) & (1ull << tt)) == 0;
  wave_lds_fence();  // the tree's reads before the next pass writes the exchange rows
  // the loads of the clamped steps past the horizon are still in flight: drain them (and
  // the result stores) before the next pass's prologue reuses the slots
  __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));
  asm volatile("" ::: "memory");
  return out;
}

// The same sixteen-trial pass with ONE exchange per step (ILQR_CAND16_FORM 2, the
// default): every lane forms all four ū rows itself (its own K·δx dots, the row form's
// order) and δx = x̄ − x, v = x̄ − x_traj for all twelve rows from the slot, so only x̄
// crosses lanes (three ds_write_b64 by the owner, six ds_read_b128 by the trial's lanes)
// — one LDS round trip on a step's dependent chain instead of three, for 36 more K·δx
// FMAs and 18 more ds_read_b128 of the (broadcast) slot. Same bits as lq_cand16_pass.
constexpr int C16B_ES = 14;  // doubles per trial's x̄ row: 16 trials on 16 different 4-bank quarters
static_assert(16 * C16B_ES <= RING_LAREA, "the exchange area fits the ring's LAREA");
template <int R, int PF>
__device__ Cand16 lq_cand16b_pass(const LQParams& P, int b, int T, const double* __restrict__ x,
                                  const double* __restrict__ u, const double* __restrict__ xtraj,
                                  const double* __restrict__ dg, const double* __restrict__ Kg, double alpha, bool st,
                                  __amdgpu_buffer_rsrc_t rXN, __amdgpu_buffer_rsrc_t rUN, int gs, double* ring) {
  constexpr int NX = 12, NU = 4;
  static_assert(R > PF && PF >= 1, "the slot being refilled must not be the one being read");
  constexpr uint32_t OOR = 0x80000000u;
  b = __builtin_amdgcn_readfirstlane(b);
  const int l = threadIdx.x & 63;
  const int r = l >> 4;   // rows 3r .. 3r+2 of x̄, row r of ū's cost and Σ(ū − u)²
  const int tt = l & 15;  // the trial
  constexpr int QO = 128;  // Q in slot 0's tail (see lq_cand16_pass)
  static_assert(QO + NX * NX <= RING_SLOT, "Q fits slot 0's tail, past the producer's 64 chunks");
  double F[3][16], Rr[NU];
  {
    const double* Ab = P.A + (size_t)b * NX * NX;
    const double* Bb = P.B + (size_t)b * NX * NU;
    const double* Qb = P.Q + (size_t)b * NX * NX;
    const double2* rr = reinterpret_cast<const double2*>(P.R + (size_t)b * NU * NU + r * NU);
    for (int i = l; i < NX * NX; i += 64) ring[QO + i] = Qb[i];
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const double2* ar = reinterpret_cast<const double2*>(Ab + (3 * r + i) * NX);
      const double2* br = reinterpret_cast<const double2*>(Bb + (3 * r + i) * NU);
#pragma unroll
      for (int k = 0; k < NX / 2; ++k) {
        const double2 a2 = ar[k];
        F[i][2 * k] = a2.x + 0.0;
        F[i][2 * k + 1] = a2.y + 0.0;
      }
#pragma unroll
      for (int m = 0; m < NU / 2; ++m) {
        const double2 b2 = br[m];
        F[i][NX + 2 * m] = 0.0 + b2.x;
        F[i][NX + 2 * m + 1] = 0.0 + b2.y;
      }
    }
#pragma unroll
    for (int m = 0; m < NU / 2; ++m) {
      const double2 r2 = rr[m];
      Rr[2 * m] = r2.x;
      Rr[2 * m + 1] = r2.y;
    }
  }
  __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");

  const double* xt0 = xtraj ? xtraj : x;
  const double xtw = xtraj ? 1.0 : 0.0;
  const char* p1;
  uint32_t s1;
  {
    const int c = l < 40 ? l : l - 40;
    const size_t bb = (size_t)b;
    if (c < 24) {
      p1 = reinterpret_cast<const char*>(Kg + bb * T * NU * NX + 2 * c);
      s1 = NU * NX * 8;
    } else if (c < 30) {
      p1 = reinterpret_cast<const char*>(x + bb * (T + 1) * NX + 2 * (c - 24));
      s1 = NX * 8;
    } else if (c < 32) {
      p1 = reinterpret_cast<const char*>(u + bb * T * NU + 2 * (c - 30));
      s1 = NU * 8;
    } else if (c < 38) {
      p1 = reinterpret_cast<const char*>(xt0 + bb * (T + 1) * NX + 2 * (c - 32));
      s1 = NX * 8;
    } else {
      p1 = reinterpret_cast<const char*>(dg + bb * T * NU + 2 * (c - 38));
      s1 = NU * 8;
    }
  }
  const uint32_t ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)ring;
  auto produce = [&](int t) {
    uint32_t tq = (uint32_t)(t < T ? t : T - 1);
    asm volatile("" : "+s"(tq));
    const uint32_t m0 = ring_lds + (uint32_t)((t % R) * RING_SLOT * 8);
    asm volatile(ILQR_FW_LDS_OP1 ::"v"(p1 + (size_t)tq * s1), "{m0}"(m0) : "memory");
  };
  constexpr int NL = 1, NS = 4;
  constexpr int N_SS = (NL + NS) * PF - NL, N_PRO = NL * PF - NL;
  auto wait_slot = [](auto n) {
    constexpr int v = decltype(n)::value;
    static_assert(v >= 0 && v < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((v & 15) | (7 << 4) | (15 << 8) | ((v >> 4) << 14));
    asm volatile("" ::: "memory");
  };
  constexpr int SX = 48, SU = 60, SXT = 64, SD = 76;
  double* const my = ring + R * RING_SLOT + tt * C16B_ES;
  const uint32_t oxs = st ? (uint32_t)(gs * (T + 1) * NX + 3 * r) * 8 : OOR;
  const uint32_t ous = st ? (uint32_t)(gs * T * NU + r) * 8 : OOR;
  auto rd12 = [](const double* p, double (&v)[NX]) {
    const double2* q = reinterpret_cast<const double2*>(p);
#pragma unroll
    for (int k = 0; k < NX / 2; ++k) {
      const double2 w = q[k];
      v[2 * k] = w.x;
      v[2 * k + 1] = w.y;
    }
  };
  auto rd4 = [](const double* p, double (&v)[NU]) {
    const double2* q = reinterpret_cast<const double2*>(p);
    const double2 w0 = q[0], w1 = q[1];
    v[0] = w0.x;
    v[1] = w0.y;
    v[2] = w1.x;
    v[3] = w1.y;
  };
  auto dot12 = [](const double (&v)[NX], const double* c) {
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
#pragma unroll
    for (int k = 0; k < NX; k += 4) {
      a0 = fma(v[k], c[k], a0);
      a1 = fma(v[k + 1], c[k + 1], a1);
      a2 = fma(v[k + 2], c[k + 2], a2);
      a3 = fma(v[k + 3], c[k + 3], a3);
    }
    return (a0 + a1) + (a2 + a3);
  };
  auto pick4 = [r](const double (&v)[NU]) {
    const double a = r & 1 ? v[1] : v[0], c = r & 1 ? v[3] : v[2];
    return r & 2 ? c : a;
  };

#pragma unroll
  for (int t = 0; t < PF; ++t) produce(t);
  wait_slot(std::integral_constant<int, N_PRO>{});
  double xo[3];  // this lane's rows of x̄ₖ
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    xo[i] = ring[SX + 3 * r + i];  // x̄₁ = x₁ (:65)
    my[3 * r + i] = xo[i];
  }
  wave_lds_fence();
  double cost[3] = {0.0, 0.0, 0.0}, costu = 0.0, du2 = 0.0;
  bool eo = true;
  auto step = [&](int t, auto next_wait) {
    const double* sl = ring + (t % R) * RING_SLOT;
    double XB[NX], DX[NX];
    rd12(my, XB);
    {
      double X[NX];
      rd12(sl + SX, X);
#pragma unroll
      for (int k = 0; k < NX; ++k) DX[k] = XB[k] - X[k];  // δx (:72)
    }
    // ūₖ = uₖ + α δuₖ + Kₖ δx (:73), all four rows
    double U4[NU], D4[NU], UB[NU];
    rd4(sl + SU, U4);
    rd4(sl + SD, D4);
#pragma unroll
    for (int m = 0; m < NU; ++m) {
      const double kdx = dot12(DX, sl + NX * m);
      const double ua = fma(alpha, D4[m], U4[m]);
      UB[m] = ua + kdx;
      eo = eo && (ua == U4[m]);
    }
    const double ubr = pick4(UB), urr = pick4(U4);
    const double e = ubr - urr;
    du2 = fma(e, e, du2);
    // x̄ₖ₊₁ = A x̄ₖ + B ūₖ (:74), this lane's rows
    double acc[3][4];
#pragma unroll
    for (int i = 0; i < 3; ++i) acc[i][0] = acc[i][1] = acc[i][2] = acc[i][3] = 0.0;
#pragma unroll
    for (int k = 0; k < NX; ++k)
#pragma unroll
      for (int i = 0; i < 3; ++i) acc[i][k & 3] = fma(XB[k], F[i][k], acc[i][k & 3]);
#pragma unroll
    for (int m = 0; m < NU; ++m)
#pragma unroll
      for (int i = 0; i < 3; ++i) acc[i][m] = fma(UB[m], F[i][NX + m], acc[i][m]);
    double xn[3];
#pragma unroll
    for (int i = 0; i < 3; ++i) xn[i] = (acc[i][0] + acc[i][1]) + (acc[i][2] + acc[i][3]);
    produce(t + PF);  // slot (t+PF)%R was last read at step t+PF−R < t
    wave_lds_fence();  // every lane's reads of the exchange row before its overwrite
#pragma unroll
    for (int i = 0; i < 3; ++i) my[3 * r + i] = xn[i];
    // ℓ(x̄ₖ − x_trajₖ, ūₖ) rows (:187-190): v = x̄ − x_traj, vᵀ(Q row); ūᵀ(R row)
    {
      double V[NX];
      rd12(sl + SXT, V);
#pragma unroll
      for (int k = 0; k < NX; ++k) V[k] = fma(-xtw, V[k], XB[k]);
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const double vi = fma(-xtw, sl[SXT + 3 * r + i], xo[i]);
        cost[i] = fma(vi, dot12(V, ring + QO + (3 * r + i) * NX), cost[i]);
      }
    }
    const double lvu = (fma(UB[0], Rr[0], 0.0) + fma(UB[1], Rr[1], 0.0)) +
                       (fma(UB[2], Rr[2], 0.0) + fma(UB[3], Rr[3], 0.0));
    costu = fma(ubr, lvu, costu);
#pragma unroll
    for (int i = 0; i < 3; ++i)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xo[i]), rXN, oxs,
                                            (uint32_t)(t * NX + i) * 8, 0);
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, ubr), rUN, ous, (uint32_t)t * NU * 8, 0);
#pragma unroll
    for (int i = 0; i < 3; ++i) xo[i] = xn[i];
    wait_slot(next_wait);  // slot t + 1 (past the horizon: a clamped step's, read and never used)
    wave_lds_fence();      // the x̄ rows written before the next step reads them
  };
  const int tp = T < PF ? T : PF;
  for (int t = 0; t < tp - 1; ++t) step(t, std::integral_constant<int, N_PRO>{});
  for (int t = tp - 1; t < T; ++t) step(t, std::integral_constant<int, N_SS>{});
#pragma unroll
  for (int i = 0; i < 3; ++i)
    __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xo[i]), rXN, oxs, (uint32_t)(T * NX + i) * 8, 0);
  {
    double XB[NX];
    rd12(my, XB);
    const double* Qfb = P.Qf + (size_t)b * NX * NX;
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      double qf[NX];
      rd12(Qfb + (3 * r + i) * NX, qf);
      cost[i] = fma(xo[i], dot12(XB, qf), cost[i]);
    }
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    const double z = 0.0;
#pragma unroll
    for (int k = 0; k < NX; k += 4) {
      a0 = fma(XB[k], z, a0);
      a1 = fma(XB[k + 1], z, a1);
      a2 = fma(XB[k + 2], z, a2);
      a3 = fma(XB[k + 3], z, a3);
    }
    costu = fma(z, (a0 + a1) + (a2 + a3), costu);
  }
  // rowsum16 over the trial's sixteen rows (lq_cand16_pass): the partials through the
  // trial's exchange row (32 doubles: the trial's row and the next one's, both idle now)
  double* const red = ring + R * RING_SLOT + tt * 32;
  static_assert(16 * 32 <= RING_LAREA, "the reduction rows fit the ring's LAREA");
  wave_lds_fence();
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    red[3 * r + i] = cost[i];
    red[16 + 3 * r + i] = 0.0;
  }
  red[12 + r] = costu;
  red[16 + 12 + r] = du2;
  wave_lds_fence();
  auto tree16 = [](const double* c) {
    return (((c[0] + c[8]) + (c[4] + c[12])) + ((c[2] + c[10]) + (c[6] + c[14]))) +
           (((c[1] + c[9]) + (c[5] + c[13])) + ((c[3] + c[11]) + (c[7] + c[15])));
  };
  double cs[16], ds[16];
#pragma unroll
  for (int k = 0; k < 16; k += 2) {
    const double2 w = *reinterpret_cast<const double2*>(red + k);
    const double2 v = *reinterpret_cast<const double2*>(red + 16 + k);
    cs[k] = w.x;
    cs[k + 1] = w.y;
    ds[k] = v.x;
    ds[k + 1] = v.y;
  }
  Cand16 out;
  out.cost = tree16(cs);
  out.du2 = tree16(ds);
  // every lane formed all four ū rows: its own eo is the trial's
  out.eo = eo;
  wave_lds_fence();
  __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));
  asm volatile("" ::: "memory");
  return out;
}

// ---------------------------------------------------------------------------
// The same forward pass on the 4-block f64 MFMA (round 2, ILQR_SCHED_FORWARD_MFMA):
// the backward's layout — lane 16ρ + 4β + κ holds element [ρ][κ] of trajectory slot β's
// 4×4 block, fm4(a, b, c) = c + aᵀb, vectors "replicated" (v[4I+ρ] in every κ). Per
// step: ū = u + αδu + Kδx (3 MFMAs, one per δx block, in parallel), x̄' = A x̄ + B ū
// (12: the A part does not wait for ū), ℓ = vᵀQv + ūᵀRū (9 for Qv, 3 + 1 + 1 for the
// dot products, which the MFMA leaves replicated over the slot's 16 lanes): 29 MFMAs
// for four trajectories against 44 DPP FMAs of the row form per four. The slot ring,
// its producer and its waits are the row form's; the operands are read from the slot
// in the block layout (Kᵀ blocks: K[κ][4J+ρ]). The constant blocks Aᵀ, Bᵀ, Qᵀ, Rᵀ
// (Qfᵀ at the end of a trial) are loaded once. Arithmetic order differs from the row
// form (MFMA sums of four): results agree to rounding (tests/test_gpu_parity.py).
// ---------------------------------------------------------------------------
__device__ __forceinline__ double fm4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

template <int R, int PF>
__device__ FwdOut lq_forward_wave_mfma(const LQParams& P, int b0, int B, int T, unsigned run,
                                       const double* __restrict__ x, const double* __restrict__ u,
                                       const double* __restrict__ xtraj, const double* __restrict__ dg,
                                       const double* __restrict__ Kg, double prev_cost,
                                       double* __restrict__ xnew, double* __restrict__ unew,
                                       double* du2_out, const LSParams& ls, double* ring) {
  constexpr int NX = 12, NU = 4;
  static_assert(R > PF && PF >= 1, "the slot being refilled must not be the one being read");
  constexpr uint32_t OOR = 0x80000000u;
  const int l = threadIdx.x & 63;
  const int rho = l >> 4, beta = (l >> 2) & 3, kap = l & 3;
  b0 = __builtin_amdgcn_readfirstlane(b0);  // wave-uniform: SGPR buffer resources, no waterfall
  const int nt = B - b0 < 4 ? B - b0 : 4;
  const int bb = b0 + (beta < nt ? beta : 0);  // absent slots alias trajectory b0 (never stored)
  const bool active = beta < nt && ((run >> beta) & 1u);

  // constant blocks (the A operand of fm4 is the block transposed)
  const double* Ab = P.A + (size_t)bb * NX * NX;
  const double* Bb = P.B + (size_t)bb * NX * NU;
  const double* Qb = P.Q + (size_t)bb * NX * NX;
  double AT[3][3], BT[3], QT[3][3];
#pragma unroll
  for (int I = 0; I < 3; ++I) {
#pragma unroll
    for (int J = 0; J < 3; ++J) {
      AT[I][J] = Ab[(4 * I + kap) * NX + 4 * J + rho];
      QT[I][J] = Qb[(4 * I + kap) * NX + 4 * J + rho];
    }
    BT[I] = Bb[(4 * I + kap) * NU + rho];
  }
  const double RT = P.R[(size_t)bb * NU * NU + kap * NU + rho];

  // producer (the row form's: three global_load_lds_dwordx4 per step fill one slot)
  auto tr = [&](int gg) { return (size_t)(b0 + (gg < nt ? gg : 0)); };
  const double* xt0 = xtraj ? xtraj : x;
  const double xtw = xtraj ? 1.0 : 0.0;
  const char *p1, *p2, *p3;
  uint32_t s1, s2, s3;
  {
    const int c = l;
    p1 = reinterpret_cast<const char*>(Kg + tr(c / 24) * T * NU * NX + 2 * (c % 24));
    s1 = NU * NX * 8;
    if (l < 32) {
      const int c2 = 64 + l;
      p2 = reinterpret_cast<const char*>(Kg + tr(c2 / 24) * T * NU * NX + 2 * (c2 % 24));
      s2 = NU * NX * 8;
    } else if (l < 56) {
      const int m = l - 32;
      p2 = reinterpret_cast<const char*>(x + tr(m / 6) * (T + 1) * NX + 2 * (m % 6));
      s2 = NX * 8;
    } else {
      const int m = l - 56;
      p2 = reinterpret_cast<const char*>(u + tr(m / 2) * T * NU + 2 * (m % 2));
      s2 = NU * 8;
    }
    const int l3 = l & 31;
    if (l3 < 24) {
      p3 = reinterpret_cast<const char*>(xt0 + tr(l3 / 6) * (T + 1) * NX + 2 * (l3 % 6));
      s3 = NX * 8;
    } else {
      const int m = l3 - 24;
      p3 = reinterpret_cast<const char*>(dg + tr(m / 2) * T * NU + 2 * (m % 2));
      s3 = NU * 8;
    }
  }
  const uint32_t ring_lds = (uint32_t)(uintptr_t)(__attribute__((address_space(3))) double*)ring;
  auto produce = [&](int t) {
    uint32_t tt = (uint32_t)(t < T ? t : T - 1);
    asm volatile("" : "+s"(tt));
    const uint32_t m0 = ring_lds + (uint32_t)((t % R) * RING_SLOT * 8);
    asm volatile(ILQR_FW_LDS_OP ::"v"(p1 + (size_t)tt * s1), "{m0}"(m0) : "memory");
    asm volatile(ILQR_FW_LDS_OP ::"v"(p2 + (size_t)tt * s2), "{m0}"(m0 + 1024) : "memory");
    asm volatile(ILQR_FW_LDS_OP ::"v"(p3 + (size_t)tt * s3), "{m0}"(m0 + 2048) : "memory");
  };
  constexpr int N_SS = 5 * PF - 3, N_PRO = 3 * PF - 3;
  auto wait_slot = [](auto n) {
    constexpr int v = decltype(n)::value;
    static_assert(v >= 0 && v < 64, "vmcnt is 6 bits");
    __builtin_amdgcn_s_waitcnt((v & 15) | (7 << 4) | (15 << 8) | ((v >> 4) << 14));
    asm volatile("" ::: "memory");
  };
  // per step the wave issues 3 slot loads, then 4 result stores (3 x̄ blocks, ū): the
  // row form's wait counts assume 2 stores per step, so this form waits with its own
  constexpr int M_SS = 7 * PF - 3;
  (void)N_SS;

  // this lane's operands in a slot (block layout)
  const int oK = 48 * beta + 12 * kap + rho;        // + 4J: K[κ][4J+ρ] of slot β
  const int oX = 192 + 12 * beta + rho;             // + 4J: x[4J+ρ]
  const int oXT = 256 + 12 * beta + rho;            // + 4J: x_traj[4J+ρ]
  const int oU = 240 + 4 * beta + rho, oD = 304 + 4 * beta + rho;
  const auto rXN = buffer_rsrc(xnew + (size_t)b0 * (T + 1) * NX, (uint32_t)nt * (T + 1) * NX * 8);
  const auto rUN = buffer_rsrc(unew + (size_t)b0 * T * NU, (uint32_t)nt * T * NU * 8);
  const bool st_lane = kap == 0;
  const uint32_t oxs = (uint32_t)(beta * (T + 1) * NX + rho) * 8;  // + 32I + 96t
  const uint32_t ous = (uint32_t)(beta * T * NU + rho) * 8;        // + 32t

  double alpha = ls.alpha0;
  FwdOut out{INFINITY, 0, 0};
  bool open = active;
  double du2_acc = 0.0;
  for (int trial = 1; trial <= ls.max_trials && __any(open); ++trial) {
#pragma unroll
    for (int t = 0; t < PF; ++t) produce(t);
    double cost = 0.0, du2 = 0.0;
    double cq[3] = {0.0, 0.0, 0.0}, cr = 0.0;  // per-block cost accumulators (no chain between them)
    const bool so = open && st_lane;
    const uint32_t ox = so ? oxs : OOR, ou = so ? ous : OOR;
    wait_slot(std::integral_constant<int, N_PRO>{});
    double xb[3];
    {
      const double* sl = ring;
#pragma unroll
      for (int J = 0; J < 3; ++J) xb[J] = sl[oX + 4 * J];  // x̄₁ = x₁ (:65)
    }
    auto step = [&](int t, auto wait_n) {
      wait_n();
      const double* sl = ring + (t % R) * RING_SLOT;
      double xk[3], xt[3], KT[3];
#pragma unroll
      for (int J = 0; J < 3; ++J) {
        xk[J] = sl[oX + 4 * J];
        xt[J] = sl[oXT + 4 * J];
        KT[J] = sl[oK + 4 * J];
      }
      const double uk = sl[oU], dk = sl[oD];
      // x̄ₖ₊₁'s A part first: it does not need ūₖ
      double y[3];
#pragma unroll
      for (int I = 0; I < 3; ++I) y[I] = fm4(AT[I][2], xb[2], fm4(AT[I][1], xb[1], fm4(AT[I][0], xb[0], 0.0)));
      // δx = x̄ₖ − xₖ (:72); ūₖ = uₖ + α δuₖ + Kₖ δx (:73)
      const double k0 = fm4(KT[0], xb[0] - xk[0], 0.0);
      const double k1 = fm4(KT[1], xb[1] - xk[1], 0.0);
      const double k2 = fm4(KT[2], xb[2] - xk[2], fma(alpha, dk, uk));
      const double ub = k2 + (k0 + k1);
      produce(t + PF);
      // ℓ(x̄ₖ − x_trajₖ, ūₖ) = vᵀQv + ūᵀRū (:187-190), accumulated in every lane of the slot
      double v[3];
#pragma unroll
      for (int J = 0; J < 3; ++J) v[J] = fma(-xtw, xt[J], xb[J]);
      double qv[3];
#pragma unroll
      for (int I = 0; I < 3; ++I) qv[I] = fm4(QT[I][2], v[2], fm4(QT[I][1], v[1], fm4(QT[I][0], v[0], 0.0)));
      const double ru = fm4(RT, ub, 0.0);
#pragma unroll
      for (int I = 0; I < 3; ++I) cq[I] = fm4(v[I], qv[I], cq[I]);
      cr = fm4(ub, ru, cr);
#pragma unroll
      for (int I = 0; I < 3; ++I)
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xb[I]), rXN, ox,
                                              (uint32_t)(t * NX * 8 + 32 * I), 0);
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, ub), rUN, ou, (uint32_t)t * NU * 8, 0);
      const double e = ub - uk;
      du2 = fma(e, e, du2);
      // x̄ₖ₊₁ = A x̄ₖ + B ūₖ (:74)
#pragma unroll
      for (int I = 0; I < 3; ++I) xb[I] = fm4(BT[I], ub, y[I]);
    };
    const int tp = T < PF ? T : PF;
    auto w_pro = [&] { wait_slot(std::integral_constant<int, N_PRO>{}); };
    auto w_ss = [&] { wait_slot(std::integral_constant<int, M_SS>{}); };
    for (int t = 0; t < tp; ++t) step(t, w_pro);
    for (int t = tp; t < T; ++t) step(t, w_ss);
    cost = ((cq[0] + cq[1]) + cq[2]) + cr;
#pragma unroll
    for (int I = 0; I < 3; ++I)
      __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2v, xb[I]), rXN, ox,
                                            (uint32_t)(T * NX * 8 + 32 * I), 0);
    // final_cost(x̄_N) = x̄ᵀQf x̄ on the raw state (:192)
    {
      const double* Qfb = P.Qf + (size_t)bb * NX * NX;
#pragma unroll
      for (int I = 0; I < 3; ++I) {
        double qv = 0.0;
#pragma unroll
        for (int J = 0; J < 3; ++J) qv = fm4(Qfb[(4 * I + kap) * NX + 4 * J + rho], xb[J], qv);
        cost = fm4(xb[I], qv, cost);
      }
    }
    // Σ(ū − u)² over the slot's four u rows (lanes 16ρ + 4β + κ, ρ = 0..3)
    du2 += __shfl_xor(du2, 16);
    du2 += __shfl_xor(du2, 32);
    if (open) {
      out.trials = trial;
      out.cost = cost;
      du2_acc = du2;
      if (prev_cost - cost > 0.0) {  // (:77-80); NaN compares false → keep searching
        out.accepted = 1;
        open = false;
      }
    }
    alpha *= ls.shrink;  // (:82)
    __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (0 << 8));
    asm volatile("" ::: "memory");
  }
  if (du2_out) *du2_out = du2_acc;
  return out;
}

// forward ring inside the pipe kernel: the workgroup's backward scratch holds R slots
constexpr int PIPE_R = 8, PIPE_PF = 7;

// forward pass + convergence test (:163-175) of the wave's trajectories b0 .. b0+3;
// called by the whole wave, groups whose status is not OK (or past B) sit out
// (`active`: this lane's group runs; the caller read it from status)
template <int NX, int NU, bool LR_REGS = true>
__device__ __forceinline__ void iter_forward_wave_active(const LQParams& P, int b0, int B, int T,
                                                         const IterArgs& a, const LSParams& ls,
                                                         double* ring, bool active) {
  const int j = threadIdx.x & 15;
  const int b = b0 + ((threadIdx.x & 63) >> 4);
  double du2 = 0.0;
  const double pc = (a.prev_cost && active) ? a.prev_cost[b] : INFINITY;
  const FwdOut r = lq_forward_wave_ring<NX, NU, PIPE_R, PIPE_PF, LR_REGS>(P, b0, B, T, active, a.x, a.u,
                                                                 a.xtraj, a.d, a.K, pc, a.xnew,
                                                                 a.unew, &du2, ls, ring);
  if (j == 0 && active) {
    if (a.trials) a.trials[b] = r.trials;
    if (a.du2) a.du2[b] = du2;
    if (a.iters) a.iters[b] = a.iter;
    if (!r.accepted) {
      a.status[b] = (r.cost != r.cost) ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED;
      if (a.res_parity) a.res_parity[b] = a.parity;
    } else {
      a.new_cost[b] = r.cost;
      if (du2 <= ls.tol) {
        a.status[b] = ILQR_TRAJ_CONVERGED;
        if (a.res_parity) a.res_parity[b] = a.parity;
      }
    }
  }
}

// forward pass + convergence test of the wave's trajectories b0 .. b0+3 on the MFMA form;
// `run` masks the slots that run (bit β)
__device__ __forceinline__ void iter_forward_wave_mfma(const LQParams& P, int b0, int B, int T,
                                                       const IterArgs& a, const LSParams& ls,
                                                       double* ring, unsigned run) {
  const int l = threadIdx.x & 63;
  const int beta = (l >> 2) & 3;
  const int b = b0 + beta;
  const bool active = b < B && ((run >> beta) & 1u);
  double du2 = 0.0;
  const double pc = (a.prev_cost && active) ? a.prev_cost[b] : INFINITY;
  const FwdOut r = lq_forward_wave_mfma<PIPE_R, PIPE_PF>(P, b0, B, T, run, a.x, a.u, a.xtraj, a.d, a.K, pc,
                                                         a.xnew, a.unew, &du2, ls, ring);
  if (l < 16 && (l & 3) == 0 && active) {  // lane 4β: ρ = κ = 0 of slot β
    if (a.trials) a.trials[b] = r.trials;
    if (a.du2) a.du2[b] = du2;
    if (a.iters) a.iters[b] = a.iter;
    if (!r.accepted) {
      a.status[b] = (r.cost != r.cost) ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED;
      if (a.res_parity) a.res_parity[b] = a.parity;
    } else {
      a.new_cost[b] = r.cost;
      if (du2 <= ls.tol) {
        a.status[b] = ILQR_TRAJ_CONVERGED;
        if (a.res_parity) a.res_parity[b] = a.parity;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Cooperative line search (the fused LQ iteration, DESIGN.md §4 "line-search tail").
// The wave-lockstep search above runs trial after trial for as long as ANY of a wave's
// four trajectories is open: at the fp64 cost floor a few trajectories in a thousand
// reject every α and the whole launch waits ≈64 full passes for them (round 2:
// 1,482 batched it/s for a 5-iteration fit against 6,541 for 3). Here the search of
// forward_pass.jl:70-87 keeps its exact answer but not its sequence:
//  * every trajectory runs trial 1 in its own wave (the common case: accepted);
//  * one still open is PUBLISHED (record + list entry) and all waves of the launch that
//    are done with their own trajectories hand out its remaining trials four at a time
//    (lq_forward_wave_ring<CAND>: the four groups of a wave roll out one trajectory at
//    four α's, bit for bit the sequential trials' rollouts and costs);
//  * each evaluated trial lowers `best` (accepted) or `stop` (rejected with α·δu
//    vanished at every step: all later trials are that trial again, CandPass) and sets
//    its mask bit; the wave whose bits complete trials 1..min(best, stop, max_trials)
//    finalises: trial `best` if any (trial 2 was stored as it ran, another one is rolled
//    out once more, storing), else the exhausted search's last trial (its rollout stored
//    for ilqr_iterate; fit keeps the previous iterate and skips it) — the sequential
//    search's x̄, ū, cost, Σ(ū − u)², trial count and status;
//  * the last wave to leave re-arms the list for the next launch.
// Liveness: nobody waits for a result — each grabbed trial is evaluated by the wave that
// grabbed it, and the wave completing the needed set finalises. Idle waves wait for more
// work only while the launch is co-resident (coop.wait) and not past a time limit.
// ---------------------------------------------------------------------------
// Memory ordering. The search's shared words (records, list, counters, candidate costs)
// are only touched by agent-scope atomics, which the XCDs see coherently; the waves
// POLL them with relaxed loads and never with acquire semantics — an acquire at agent
// scope invalidates the XCD's L2 (buffer_inv sc1), and a thousand waiting waves doing
// that every microsecond ran the headline iteration at 349 µs instead of 154 µs.
// Values a decision depends on are read by read-modify-writes (the atomic's own
// coherent value); rollout stores that another XCD may overwrite later in the launch
// (trial 1's by the publisher, trial 2's stored as it ran) are written back by a
// release fence before the word that hands the trajectory on — a handful per launch.
// Trace build (ILQR_COOP_TRACE, the Makefile's `tracevariant`; never the product): every
// grab of the cooperative search records (kind, generation, trajectory, j0, lim,
// finalised, start / pass end / finaliser end on the 100 MHz real-time counter) and every
// wave the end of its own trial-1 work; tools/coop_trace.py reads them back through
// ilqr_debug_trace (ilqr_bw4.hip).
#ifdef ILQR_COOP_TRACE
constexpr unsigned COOP_TRACE_MAX = 262144;
__device__ unsigned long long g_trace[4 * COOP_TRACE_MAX];
__device__ unsigned g_trace_n;
__device__ __forceinline__ void coop_trace(unsigned kind, unsigned gen, unsigned id, unsigned j0, unsigned lim,
                                           unsigned fin, uint64_t t0, uint64_t t1, uint64_t t2) {
  const unsigned k = __hip_atomic_fetch_add(&g_trace_n, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (k >= COOP_TRACE_MAX) return;
  g_trace[4 * k] = (unsigned long long)kind | ((unsigned long long)fin << 4) | ((unsigned long long)(j0 & 255) << 8) |
                   ((unsigned long long)(lim & 255) << 16) | ((unsigned long long)(id & 0xFFFFFF) << 24) |
                   ((unsigned long long)(gen & 0xFFFF) << 48);
  g_trace[4 * k + 1] = t0;
  g_trace[4 * k + 2] = t1;
  g_trace[4 * k + 3] = t2;
}
#endif

#ifndef ILQR_COOP_DEEP_FIRST
#define ILQR_COOP_DEEP_FIRST 1
#endif
#ifndef ILQR_COOP_FRONTIER_DEEP
#define ILQR_COOP_FRONTIER_DEEP 1
#endif
constexpr int COOP_DEEP_FRONT = 5;  // trials 1..5 known rejected: past a first quad or sixteen
#ifndef ILQR_COOP_WAIT_TICKS
#define ILQR_COOP_WAIT_TICKS 20000
#endif
__device__ __forceinline__ int32_t ag_ld(const int32_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int32_t ag_rmw_ld(int32_t* p) {  // the coherent current value
  return __hip_atomic_fetch_or(p, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ag_rmw_ldd(double* p) {
  const uint64_t v = __hip_atomic_fetch_or(reinterpret_cast<uint64_t*>(p), (uint64_t)0, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_bit_cast(double, v);
}
__device__ __forceinline__ void ag_st(int32_t* p, int32_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void ag_std(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void release_agent() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent"); }
__device__ __forceinline__ void complete_vmem() {  // every issued load / store / atomic done
  __builtin_amdgcn_s_waitcnt((0) | (7 << 4) | (15 << 8));
  asm volatile("" ::: "memory");
}
// smallest of best, stop, max_trials: hint (relaxed loads) or exact (read-modify-writes)
__device__ __forceinline__ int coop_lim_hint(const LSCoopRec* R, int max_trials) {
  const int be = ag_ld(&R->best), st = ag_ld(&R->stop);
  const int m = be < st ? be : st;
  return m < max_trials ? m : max_trials;
}
__device__ __forceinline__ int coop_lim(LSCoopRec* R, int max_trials) {
  const int be = ag_rmw_ld(&R->best), st = ag_rmw_ld(&R->stop);
  const int m = be < st ? be : st;
  return m < max_trials ? m : max_trials;
}
// α of trial j: the reference's repeated α *= shrink (:82), j − 1 times
__device__ __forceinline__ double trial_alpha(const LSParams& ls, int j) {
  double a = ls.alpha0;
  for (int k = 1; k < j; ++k) a *= ls.shrink;
  return a;
}

// Publish trajectory b (trial 1 rejected) in launch `gen`: called by one lane.
__device__ __forceinline__ void coop_publish(const LSCoop& c, uint32_t gen, int b, int max_trials) {
  LSCoopRec* R = c.rec + b;
  ag_st(&R->next, 2);
  ag_st(&R->best, max_trials + 1);
  ag_st(&R->stop, max_trials + 1);
  ag_st(&R->fin, 0);
  __hip_atomic_store(&R->mask, (uint64_t)1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);  // trial 1 done
  const int slot = __hip_atomic_fetch_add(c.ctl + (gen & 1), 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  ag_st(&R->slot, slot);
  release_agent();  // the record (its slot too), and trial 1's rollout stores, before the entry
  __hip_atomic_store(c.list + slot, ((uint64_t)gen << 32) | (uint32_t)b, __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}

// A published trajectory with trials left to hand out, the least speculative first (the
// smallest distance of `next` past the trials its search has evaluated, then the largest
// `next` at the frontier — the smallest past it —, then the first entry at or after this
// wave's rotated start); -1
// if none. Relaxed
// reads: a hint, the grab itself is exact. `unwritten`: a reserved list slot is not
// written yet (its publisher is mid-way: the slot still holds another launch's entry).
__device__ __attribute__((unused)) int coop_find(const LSCoop& c, uint32_t gen, int n, int max_trials,
                                                 int start, bool& unwritten) {
  // The shared words are read at the coherence point (≈1 µs a round trip): each lane
  // takes CH entries of a batch of 64·CH, their list words in one round trip and their
  // records in a second, instead of two round trips per 64 entries.
  constexpr int CH = 8;
  const int l = threadIdx.x & 63;
  uint64_t best = ~0ull;  // (next << 32) | position from `start`: smallest next, then earliest
  for (int base = 0; base < n; base += 64 * CH) {
    uint64_t e[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int pos = base + 64 * k + l;
      int i = start + pos;
      i = i >= n ? i - n : i;
      e[k] = pos < n ? __hip_atomic_load(c.list + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                     : ((uint64_t)gen << 32) | 0xFFFFFFFFull;  // past the list: no entry
    }
    int nx[CH], lim[CH], dist[CH], fr[CH];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const uint32_t bb = (uint32_t)e[k];
      const bool ok = (uint32_t)(e[k] >> 32) == gen && bb != 0xFFFFFFFFu;
      const LSCoopRec* R = c.rec + (ok ? bb : 0);
      // the record's words as three 64-bit relaxed loads (hints; the grab is exact): every
      // idle wave scans the list, and with few searches they all hit the same few records
      const uint64_t nb = ok ? __hip_atomic_load(reinterpret_cast<const uint64_t*>(&R->next), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0;
      const uint64_t sf = ok ? __hip_atomic_load(reinterpret_cast<const uint64_t*>(&R->stop), __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0;
      const uint64_t m = ok ? __hip_atomic_load(&R->mask, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
      nx[k] = ok ? (int32_t)(uint32_t)nb : 0x7fffffff;
      {
        const int be = (int32_t)(uint32_t)(nb >> 32), st = (int32_t)(uint32_t)sf;
        const int mn = be < st ? be : st;
        lim[k] = ok ? (mn < max_trials ? mn : max_trials) : 0;
      }
      // how far its next quad lies past the trials known so far (1..front evaluated):
      // the least speculative quad first — a search's first quad, or the next quad of a
      // deep search whose handed-out trials have all come back rejected
      const int front = ~m ? __builtin_ctzll(~m) : 64;
      dist[k] = nx[k] - front;
      fr[k] = front;
      if ((uint32_t)(e[k] >> 32) != gen) unwritten = true;  // reserved, not yet written
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const uint32_t dk = dist[k] < 1 ? 1u : (dist[k] > 127 ? 127u : (uint32_t)dist[k]);
      // class: 0 a grab at its search's frontier; 1 a speculative grab of a search whose
      // first grab came back rejected (front past COOP_DEEP_FRONT: deep at the floor, its
      // later trials are likely needed); 2 a speculative grab of a search still at its
      // first grab (round 6, ILQR_COOP_DEEP_FIRST; 0: classes 1 and 2 merge)
      const uint32_t cls = dk <= 1 ? 0u : ((ILQR_COOP_DEEP_FIRST && fr[k] >= COOP_DEEP_FRONT) ? 1u : 2u);
      // within a class the smallest `next` first — except at the frontier (class 0), where
      // the largest goes first (ILQR_COOP_FRONTIER_DEEP): a deep search's next grab before
      // a fresh search's first (the co-headline fit 1.192-1.196 → 1.174-1.181 ms,
      // iteration 6 834-847 → 819-842 µs; profiles/r06/coop_frontier_deep_ab_r06.log)
      const uint32_t nk = (ILQR_COOP_FRONTIER_DEEP && cls == 0u) ? 0x7FFFFFu - ((uint32_t)nx[k] & 0x7FFFFFu)
                                                                 : ((uint32_t)nx[k] & 0x7FFFFFu);
      const uint64_t key = ((uint64_t)cls << 62) | ((uint64_t)dk << 55) | ((uint64_t)nk << 32) |
                           (uint32_t)(base + 64 * k + l);
      if (nx[k] <= lim[k] && key < best) best = key;
    }
    // wave minimum
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
      const uint64_t q = __shfl_xor(best, o);
      best = q < best ? q : best;
    }
    if ((best >> 62) == 0) break;  // a grab right at its search's frontier: nothing ranks before it
  }
  unwritten = __any(unwritten);
  if (best == ~0ull) return -1;
  const uint32_t pos = __builtin_amdgcn_readfirstlane((uint32_t)best);
  int i = start + (int)pos;
  i = i >= n ? i - n : i;
  const uint64_t e = __hip_atomic_load(c.list + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __builtin_amdgcn_readfirstlane((int)(uint32_t)e);
}

// Trajectory b's outcome, once trials 1..lim are evaluated (whole wave).
// dst[0, n) = src[0, n) by the whole wave, the source read coherently at agent scope (it
// was written by another wave, possibly on another XCD, and released before the mask
// bits that let this wave finalise; a plain load could hit a line this XCD's L2 kept from
// an earlier launch), eight loads per lane in flight
__device__ __forceinline__ void coop_copy(double* __restrict__ dst, const double* src, int n) {
  const int l = threadIdx.x & 63;
  for (int i0 = 0; i0 < n; i0 += 64 * 8) {
    uint64_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + 64 * k + l;
      v[k] = i < n ? __hip_atomic_load(reinterpret_cast<const uint64_t*>(src + i), __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_AGENT)
                   : 0ull;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int i = i0 + 64 * k + l;
      if (i < n) dst[i] = __builtin_bit_cast(double, v[k]);
    }
  }
}

// `sl`: the search's list position; below c.nslots every evaluated trial's rollout is in
// the scratch and the final one is copied from there instead of rolled out again.
template <int NX, int NU>
__device__ void coop_finalize(const LQParams& P, int b, int B, int T, const IterArgs& a, const LSCoop& c,
                              const LSParams& ls, double* ring, int lim, int sl) {
  LSCoopRec* R = c.rec + b;
  int best = 0;
  double cost = 0.0, du2 = 0.0;
  if ((threadIdx.x & 63) == 0) {
    best = ag_rmw_ld(&R->best);
    cost = ag_rmw_ldd(c.cost + (size_t)b * COOP_MAX_TRIALS + lim - 1);
    du2 = ag_rmw_ldd(c.du2 + (size_t)b * COOP_MAX_TRIALS + lim - 1);
  }
  const bool accepted = __builtin_amdgcn_readfirstlane(best) <= ls.max_trials;  // then best == lim
  // trial 2's group stored as it ran; any other final rollout is rolled out again,
  // storing (an exhausted one only for ilqr_iterate: fit keeps the previous iterate) —
  // or, for a search with a scratch slot, copied from the trial's scratch rollout
  const bool scr = sl < c.nslots;
  if (scr && (accepted || !a.res_parity)) {
    const int s0 = sl * COOP_MAX_TRIALS + lim - 1;
    coop_copy(a.xnew + (size_t)b * (T + 1) * NX, c.sx + (size_t)s0 * (T + 1) * NX, (T + 1) * NX);
    coop_copy(a.unew + (size_t)b * T * NU, c.su + (size_t)s0 * T * NU, T * NU);
  } else if (!scr && lim != 2 && (accepted || !a.res_parity)) {
    const int g = (threadIdx.x & 63) >> 4;
    double scratch = 0.0;
    (void)lq_forward_wave_ring<NX, NU, PIPE_R, PIPE_PF, true, true>(
        P, b, B, T, g == 0, a.x, a.u, a.xtraj, a.d, a.K, 0.0, a.xnew, a.unew, &scratch, ls, ring,
        CandPass{trial_alpha(ls, lim), 0});
  }
  if ((threadIdx.x & 63) == 0) {
    if (a.trials) a.trials[b] = accepted ? lim : ls.max_trials;
    if (a.du2) a.du2[b] = du2;
    if (a.iters) a.iters[b] = a.iter;
    if (!accepted) {
      a.status[b] = (cost != cost) ? ILQR_TRAJ_NAN : ILQR_TRAJ_LS_EXHAUSTED;
      if (a.res_parity) a.res_parity[b] = a.parity;
    } else {
      a.new_cost[b] = cost;  // prev_cost = new_cost (:168)
      if (du2 <= ls.tol) {   // (:171)
        a.status[b] = ILQR_TRAJ_CONVERGED;
        if (a.res_parity) a.res_parity[b] = a.parity;
      }
    }
  }
}

// Trials handed out per grab (round 6): sixteen (lq_cand16_pass: ≈2× the trials per µs of
// a wave, ≈1.8× the latency of a pass) when the launch published more than
// COOP_WIDE_MIN searches — the at-floor iteration 5's ~900, where the search phase is
// throughput-bound — else four (lq_forward_wave_ring's candidate pass, rounds 3-5: a few
// deep searches and a thousand idle waves, latency-bound; iteration 4's 9 searches of 63
// trials each: 97 µs in quads against 116 µs in sixteens, tools/coop_trace.py,
// profiles/r06/). ILQR_COOP_WIDTH = 4 or 16 fixes it (A/B builds). Every width evaluates
// each trial bit for bit as the sequential search does, so mixing them in one search
// changes nothing but the schedule.
#ifndef ILQR_COOP_WIDTH
#define ILQR_COOP_WIDTH 0
#endif
#ifndef ILQR_CAND16_FORM  // 1: lq_cand16_pass (three exchanges a step), 2: lq_cand16b_pass (one)
#define ILQR_CAND16_FORM 1
#endif
static_assert(ILQR_COOP_WIDTH == 0 || ILQR_COOP_WIDTH == 4 || ILQR_COOP_WIDTH == 16, "a grab is 4 or 16 trials");
constexpr int COOP_WIDE_MIN = 64;
__device__ __forceinline__ bool coop_wide(int published) {
  return ILQR_COOP_WIDTH == 16 || (ILQR_COOP_WIDTH == 0 && published > COOP_WIDE_MIN);
}

// Grab trials j0 .. j0+W−1 of trajectory b (W = 16 if `wide`, else 4), evaluate them, and
// finalise b if these were the last needed (whole wave).
template <int NX, int NU>
__device__ int coop_evaluate(const LQParams& P, int b, int B, int T, const IterArgs& a, const LSCoop& c,
                              const LSParams& ls, double* ring, bool wide) {
  const int W = wide ? 16 : 4;
  LSCoopRec* R = c.rec + b;
  const int l = threadIdx.x & 63;
  int j0 = 0, lim0 = 0, sl = 0;
  if (l == 0) {
    j0 = __hip_atomic_fetch_add(&R->next, W, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    lim0 = coop_lim(R, ls.max_trials);
    sl = ag_rmw_ld(&R->slot);  // picks the scratch rows: a decision, so read coherently
  }
  j0 = __builtin_amdgcn_readfirstlane(j0);
  lim0 = __builtin_amdgcn_readfirstlane(lim0);
  sl = __builtin_amdgcn_readfirstlane(sl);
  const bool scr = sl < c.nslots;  // every trial's rollout to the scratch
  if (j0 > lim0) return 0;  // raced past the needed set: nothing to do
#ifdef ILQR_COOP_TRACE
  const uint64_t tq0 = __builtin_amdgcn_s_memrealtime();
#endif
  // the cost to beat: written before this launch (in place by fit's finaliser of b only,
  // once no trial of b is needed any more)
  const double pc = a.prev_cost ? a.prev_cost[b] : INFINITY;
  double du2 = 0.0, cost;
  bool eo;
  int j;
  bool mine;
  if (wide) {
    const int tt = l & 15;  // this lane's trial
    j = j0 + tt;
    mine = j <= lim0;
    // trial 2's rollout into x_new / u_new as it runs (no scratch), else every trial's
    // into its scratch row
    const auto rXN =
        scr ? buffer_rsrc(uniform_ptr(c.sx),
                          (uint32_t)__builtin_amdgcn_readfirstlane(c.nslots * COOP_MAX_TRIALS * (T + 1) * NX * 8))
            : buffer_rsrc(uniform_ptr(a.xnew + (size_t)b * (T + 1) * NX),
                          (uint32_t)__builtin_amdgcn_readfirstlane((T + 1) * NX * 8));
    const auto rUN =
        scr ? buffer_rsrc(uniform_ptr(c.su),
                          (uint32_t)__builtin_amdgcn_readfirstlane(c.nslots * COOP_MAX_TRIALS * T * NU * 8))
            : buffer_rsrc(uniform_ptr(a.unew + (size_t)b * T * NU), (uint32_t)__builtin_amdgcn_readfirstlane(T * NU * 8));
    const bool st = mine && (scr || (j0 == 2 && tt == 0));
    const int gs = scr ? sl * COOP_MAX_TRIALS + j - 1 : 0;
#if ILQR_CAND16_FORM == 1
    // (a store-free instantiation for passes that store nothing measured slower in the
    // at-floor iteration: pass p50 90.5 → 99.0 µs, profiles/r06/coop_store_split_r06.log)
    const Cand16 r16 = lq_cand16_pass<PIPE_R, PIPE_PF, true>(P, b, T, a.x, a.u, a.xtraj, a.d, a.K,
                                                             trial_alpha(ls, j), st, rXN, rUN, gs, ring);
#else
    const Cand16 r16 = lq_cand16b_pass<PIPE_R, PIPE_PF>(P, b, T, a.x, a.u, a.xtraj, a.d, a.K, trial_alpha(ls, j),
                                                        st, rXN, rUN, gs, ring);
#endif
    cost = r16.cost;
    du2 = r16.du2;
    eo = r16.eo;
  } else {
    const int g = l >> 4;  // this group's trial
    j = j0 + g;
    mine = j <= lim0;
    CandPass cp{trial_alpha(ls, j), j0 == 2 ? 0 : -1};
    if (scr) {
      cp.sx = c.sx;
      cp.su = c.su;
      cp.sidx = sl * COOP_MAX_TRIALS + j0 - 1;
      cp.sx_bytes = (uint32_t)(c.nslots * COOP_MAX_TRIALS * (T + 1) * NX * 8);
      cp.su_bytes = (uint32_t)(c.nslots * COOP_MAX_TRIALS * T * NU * 8);
    }
    const FwdOut r = lq_forward_wave_ring<NX, NU, PIPE_R, PIPE_PF, true, true>(
        P, b, B, T, mine, a.x, a.u, a.xtraj, a.d, a.K, pc, a.xnew, a.unew, &du2, ls, ring, cp);
    cost = r.cost;
    eo = r.eo;
  }
  // one lane per trial records it (lanes 0..15 with W = 16; lane 16g with W = 4)
  const bool rec = wide ? l < 16 : (l & 15) == 0;
  if (rec && mine) {
    ag_std(c.cost + (size_t)b * COOP_MAX_TRIALS + j - 1, cost);
    ag_std(c.du2 + (size_t)b * COOP_MAX_TRIALS + j - 1, du2);
    if (pc - cost > 0.0)  // (:77-80); NaN compares false
      __hip_atomic_fetch_min(&R->best, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else if (eo)
      __hip_atomic_fetch_min(&R->stop, j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // costs and best/stop complete before the mask bits; trial 2's rollout (stored as it
  // ran) and scratch rollouts also written back from this XCD's L2
  if (j0 == 2 || scr)
    release_agent();
  else
    complete_vmem();
  int fin = 0, lim = 0;
  if (l == 0) {
    uint64_t bits = 0;
    for (int k = 0; k < W; ++k)
      if (j0 + k <= lim0) bits |= 1ull << (j0 + k - 1);
    const uint64_t m =
        __hip_atomic_fetch_or(&R->mask, bits, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) | bits;
    // the mask RMW performed before best/stop are read: two waves that each lower
    // best/stop and then set their bits cannot both read the other's mask without its
    // bits AND an old best (store-buffer pattern) — one of them sees the complete set
    complete_vmem();
    lim = coop_lim(R, ls.max_trials);
    const uint64_t need = lim >= 64 ? ~0ull : ((1ull << lim) - 1ull);
    if ((m & need) == need) {
      int z = 0;
      fin = __hip_atomic_compare_exchange_strong(&R->fin, &z, 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT) ? 1 : 0;
    }
  }
  fin = __builtin_amdgcn_readfirstlane(fin);
  lim = __builtin_amdgcn_readfirstlane(lim);
#ifdef ILQR_COOP_TRACE
  const uint64_t tq1 = __builtin_amdgcn_s_memrealtime();
#endif
  if (fin) coop_finalize<NX, NU>(P, b, B, T, a, c, ls, ring, lim, sl);
#ifdef ILQR_COOP_TRACE
  if (l == 0) coop_trace(2, a.coop_gen, b, j0, fin ? lim : lim0, fin, tq0, tq1, __builtin_amdgcn_s_memrealtime());
#endif
  return fin ? 2 : 1;  // 1: trials evaluated, the search not finalised here; 2: finalised
}

// The work loop every wave of the launch enters once it is done with its own
// trajectories: while a published trajectory has trials to hand out, grab and evaluate;
// then leave. Nobody waits for work that is not there yet: a wave always finds its own
// published trajectories (it wrote their entries), so a helper that left early costs
// only speed — and waves waiting for later publications measured expensive (a thousand
// waves polling the list length slowed the waves still working: cold iteration 144 →
// 219 µs; with a per-wave done counter and exit ticket, same-address atomics from every
// wave, 190 µs). Each launch counts its list in ctl[gen & 1] and zeroes the other half
// for the next launch; stale entries carry another generation.
template <int NX, int NU>
__device__ void lq_coop_search(const LQParams& P, int B, int T, const IterArgs& a, const LSParams& ls,
                               double* ring, int wid, int b0, unsigned own) {
  const uint32_t gen = a.coop_gen;
  // the no-publication launch (every iteration from cold, most of a fit's) leaves after
  // ONE load: the list length straight from the kernel arguments
  if (__builtin_amdgcn_readfirstlane(ag_ld(a.coop_ctl + (gen & 1))) == 0) return;
#ifdef ILQR_COOP_TRACE
  if ((threadIdx.x & 63) == 0) coop_trace(1, gen, wid, 0, 0, 0, __builtin_amdgcn_s_memrealtime(), 0, 0);
#endif
  const LSCoop c = *a.coop;  // scalar loads, only once there is work
  // first the quads of the wave's own published trajectories (`own`, bit q: b0 + q): a
  // search's first quad then starts as its trial 1 ends, not when some wave frees up
  // (≈50 µs later in the at-floor iteration, §4); a quad another wave took already
  // makes this grab the next one, or nothing
  auto wide_now = [&] { return coop_wide(__builtin_amdgcn_readfirstlane(ag_ld(c.ctl + (gen & 1)))); };
#pragma unroll 1
  for (int q = 0; q < 4; ++q)
    if ((own >> q) & 1u) coop_evaluate<NX, NU>(P, b0 + q, B, T, a, c, ls, ring, wide_now());
  // then stay on them: each further quad of an own search that is still open (the wave
  // knows its last quad's outcome first), up to the first one with nothing left to grab
#pragma unroll 1
  for (int q = 0; q < 4; ++q)
    if ((own >> q) & 1u)
      for (int k = 0; k < COOP_MAX_TRIALS / 4; ++k)
        if (coop_evaluate<NX, NU>(P, b0 + q, B, T, a, c, ls, ring, wide_now()) != 1) break;
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  // 200 µs at the 100 MHz real-time counter; the Makefile's `variants` target builds a
  // library with 0 (a wave leaves at the first unwritten slot it sees) for the test of
  // this exit (tests/test_gpu_line_search.py::test_coop_timeout_exit_variant)
  constexpr uint64_t WAIT_TICKS = ILQR_COOP_WAIT_TICKS;
  while (true) {
    const int n = __builtin_amdgcn_readfirstlane(ag_ld(c.ctl + (gen & 1)));
    if (n == 0) break;
    bool unwritten = false;
    const int b = coop_find(c, gen, n, ls.max_trials, (int)(((uint64_t)wid * 2654435761u) % (uint32_t)n),
                            unwritten);
    if (b >= 0) {
      coop_evaluate<NX, NU>(P, b, B, T, a, c, ls, ring, coop_wide(n));
      continue;
    }
    // a reserved entry is written moments after its slot: worth a short wait
    if (!unwritten || __builtin_amdgcn_s_memrealtime() - t0 > WAIT_TICKS) {
#ifdef ILQR_COOP_TRACE
      if ((threadIdx.x & 63) == 0) coop_trace(3, gen, wid, 0, 0, 0, __builtin_amdgcn_s_memrealtime(), 0, 0);
#endif
      break;
    }
    __builtin_amdgcn_s_sleep(8);
  }
}

// The fused iteration's forward with the cooperative search: trial 1 in the wave's own
// groups (the ring forward's sequential code at max_trials = 1); an accepted trajectory
// is done as in iter_forward_wave_active, an open one is published.
template <int NX, int NU>
__device__ __forceinline__ unsigned iter_forward_wave_coop(const LQParams& P, int b0, int B, int T,
                                                           const IterArgs& a, const LSParams& ls,
                                                           double* ring, bool active) {
  const int j = threadIdx.x & 15;
  const int b = b0 + ((threadIdx.x & 63) >> 4);
  LSParams ls1 = ls;
  ls1.max_trials = 1;
  double du2 = 0.0;
  const double pc = (a.prev_cost && active) ? a.prev_cost[b] : INFINITY;
  const FwdOut r = lq_forward_wave_ring<NX, NU, PIPE_R, PIPE_PF>(P, b0, B, T, active, a.x, a.u, a.xtraj, a.d,
                                                                 a.K, pc, a.xnew, a.unew, &du2, ls1, ring);
  if (j == 0 && active) {
    if (!r.accepted) {
      coop_publish(*a.coop, a.coop_gen, b, ls.max_trials);  // status stays OK until finalised
    } else {
      if (a.trials) a.trials[b] = 1;
      if (a.du2) a.du2[b] = du2;
      if (a.iters) a.iters[b] = a.iter;
      a.new_cost[b] = r.cost;
      if (du2 <= ls.tol) {
        a.status[b] = ILQR_TRAJ_CONVERGED;
        if (a.res_parity) a.res_parity[b] = a.parity;
      }
    }
  }
  // the published groups, bit q (wave-uniform)
  const uint64_t pub = __ballot(j == 0 && active && !r.accepted);
  unsigned own = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) own |= ((pub >> (16 * q)) & 1ull) ? (1u << q) : 0u;
  return own;
}

template <int NX, int NU, bool LR_REGS = true>
__device__ __forceinline__ void iter_forward_wave(const LQParams& P, int b0, int B, int T,
                                                  const IterArgs& a, const LSParams& ls,
                                                  double* ring) {
  const int b = b0 + ((threadIdx.x & 63) >> 4);
  const bool active = b < B && a.status[b < B ? b : b0] == ILQR_TRAJ_OK;
  iter_forward_wave_active<NX, NU, LR_REGS>(P, b0, B, T, a, ls, ring, active);
}

}  // namespace
}  // namespace ilqr
