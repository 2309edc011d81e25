// Forward rollout + line search (src/forward_pass.jl:55-93) of the families with a
// 4-dimensional state and a closed-form RK4 per lane: the 2-link arm (ilqr_twolink.hip)
// and 2-joint chains on their closed-form dynamics (ilqr_chain.hip). Private header.
//
// L line-search candidates per trajectory are evaluated side by side: lane `sub` of a
// trajectory's group of L adjacent lanes rolls out trial r·L + sub + 1 in round r, at
// α = α₀·shrinkʳᴸ⁺ˢᵘᵇ formed by the same repeated multiplication as the reference's
// `α *= shrink` (:82), and the group accepts the FIRST candidate in trial order whose
// cost decreased (:77-80) — the sequential search's answer, bit for bit. Lane sub = 0
// stores its rollout as it goes; an accepted candidate of another lane rolls out once
// more, storing (same α, same rollout). Trials 1..L cost one pass (L = 1 is the
// sequential search). An exhausted search leaves x_new / u_new holding the LAST trial's
// rollout, as the sequential search does (its lane rolls out once more, storing, when
// it is not lane 0) — unless `store_exhausted` is false (fit, which keeps the previous
// iterate of an exhausted trajectory and never reads them).
//
// A Model supplies the arithmetic of one family (value type V, NU inputs):
//   rk4_fast(x, u, out, bad)  one RK4 step without a branch; sets `bad` when an argument
//                             left the ranges its branch-free forms cover (HAS_CARRY:
//                             rk4_fast(x, u, out, bad, carry) after carry_init(x̄₁), a
//                             value the model hands from step to step)
//   rk4_robust(x, u, out)     the same step for every argument (the rollout is redone on
//                             it when a fast pass flagged `bad`)
//   stage_cost(xb, xt, xtw, ub), final_cost(xb)   ℓ(x̄ₖ − x_trajₖ, ūₖ) and ℓ_f(x̄_N)
#pragma once
#include <hip/hip_runtime.h>

#include <cstdlib>

#include "ilqr_device.h"
#include "ilqr_internal.h"

namespace ilqr {
namespace {

constexpr int FG_PF = 2;  // input prefetch depth (steps; 4 measured no faster, tools/tl_fw_probe)

template <bool ROBUST>
struct FgPath {
  static constexpr bool value = ROBUST;
};

template <class V>
struct FgOut {
  V cost;
  V du2;
  int trials;
  int accepted;
  bool owner;  // this lane holds the trajectory's result
};

// a model's per-rollout carry (HAS_CARRY: carry_init(x̄₁), then rk4_fast(…, carry) per
// step), or nothing
template <class M, bool = M::HAS_CARRY> struct FgCarry { struct T {}; };
template <class M> struct FgCarry<M, true> { using T = typename M::Carry; };
template <class M, class X>
__device__ __forceinline__ typename FgCarry<M>::T fg_carry_init(const M& m, const X& x) {
  if constexpr (M::HAS_CARRY) return m.carry_init(x);
  else return {};
}
template <class M, class X, class U, class O, class C>
__device__ __forceinline__ void fg_rk4_fast(const M& m, const X& x, const U& u, O& o, bool& bad, C& cy) {
  if constexpr (M::HAS_CARRY) m.rk4_fast(x, u, o, bad, cy);
  else m.rk4_fast(x, u, o, bad);
}

template <class V> struct Fg4;
template <> struct Fg4<double> { using T = double4; };
template <> struct Fg4<float> { using T = float4; };

// 16-byte stores of the state through a buffer resource (an out-of-range offset drops
// them); 4 values of V
__device__ __forceinline__ void fg_store_x(__amdgpu_buffer_rsrc_t r, uint32_t o, const double (&v)[4]) {
  typedef unsigned u4v_ __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v_, make_double2(v[0], v[1])), r, o, 0, 0);
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v_, make_double2(v[2], v[3])), r, o + 16, 0, 0);
}
__device__ __forceinline__ void fg_store_x(__amdgpu_buffer_rsrc_t r, uint32_t o, const float (&v)[4]) {
  typedef unsigned u4v_ __attribute__((ext_vector_type(4)));
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4v_, make_float4(v[0], v[1], v[2], v[3])), r, o, 0, 0);
}
__device__ __forceinline__ void fg_store_1(__amdgpu_buffer_rsrc_t r, uint32_t o, double v) {
  store_or_drop(v, r, true, o);
}
__device__ __forceinline__ void fg_store_1(__amdgpu_buffer_rsrc_t r, uint32_t o, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, o, 0, 0);
}

// the forward's buffer resources span one wave's trajectories: 64 · (T+1) · 4 · sizeof(V)
// bytes below 2³¹ (the out-of-range offset that drops a store)
template <class V>
inline bool fg_fits(int T) { return (size_t)64 * (T + 1) * 4 * sizeof(V) < 0x80000000ull; }

template <class Model, int L>
__device__ FgOut<typename Model::V> fwd_group(const Model& m, int b, int B, int T,
                                               const typename Model::V* __restrict__ x,
                                               const typename Model::V* __restrict__ u,
                                               const typename Model::V* __restrict__ xtraj,
                                               const typename Model::V* __restrict__ dg,
                                               const typename Model::V* __restrict__ Kg,
                                               typename Model::V prev_cost,
                                               typename Model::V* __restrict__ xnew,
                                               typename Model::V* __restrict__ unew, const LSParams& ls,
                                               bool store_exhausted = true) {
  using V = typename Model::V;
  using V4 = typename Fg4<V>::T;
  constexpr int NU = Model::NU, NX = 4;
  const V* xb0 = x + (size_t)b * (T + 1) * NX;
  const V* ub0 = u + (size_t)b * T * NU;
  const V* xt0 = (xtraj ? xtraj : x) + (size_t)b * (T + 1) * NX;
  const V xtw = xtraj ? V(1) : V(0);  // x_traj = NULL means zeros (forward_pass.jl:151)
  const V* d0 = dg + (size_t)b * T * NU;
  const V* K0 = Kg + (size_t)b * T * NU * NX;
  const int lane = threadIdx.x & 63, sub = lane & (L - 1), gbase = lane & ~(L - 1);

  struct StepIn {
    V x[4], xt[4], u[NU], d[NU], K[4 * NU];
  };
  auto load = [&](int t, StepIn& in) {
    const int tt = t < T ? t : T - 1;
    const V4 xv = *reinterpret_cast<const V4*>(xb0 + (size_t)tt * NX);
    const V4 tv = *reinterpret_cast<const V4*>(xt0 + (size_t)tt * NX);
    in.x[0] = xv.x; in.x[1] = xv.y; in.x[2] = xv.z; in.x[3] = xv.w;
    in.xt[0] = tv.x; in.xt[1] = tv.y; in.xt[2] = tv.z; in.xt[3] = tv.w;
#pragma unroll
    for (int a = 0; a < NU; ++a) {
      in.u[a] = ub0[(size_t)tt * NU + a];
      in.d[a] = d0[(size_t)tt * NU + a];
      const V4 kr = reinterpret_cast<const V4*>(K0 + (size_t)tt * NU * NX)[a];
      in.K[4 * a] = kr.x; in.K[4 * a + 1] = kr.y; in.K[4 * a + 2] = kr.z; in.K[4 * a + 3] = kr.w;
    }
  };

  // the wave's outputs through buffer resources on its first trajectory: a lane that
  // does not store gets an out-of-range offset (dropped by the bounds check), so the
  // stores need no branch and a pass's steps stay one basic block for the scheduler
  const int bw = __builtin_amdgcn_readfirstlane(b);
  const int nslot = B - bw < 64 / L ? B - bw : 64 / L;
  const auto rX = buffer_rsrc(xnew + (size_t)bw * (T + 1) * NX, (uint32_t)((size_t)nslot * (T + 1) * NX * sizeof(V)));
  const auto rU = buffer_rsrc(unew + (size_t)bw * T * NU, (uint32_t)((size_t)nslot * T * NU * sizeof(V)));
  const uint32_t offX = (uint32_t)((size_t)(b - bw) * (T + 1) * NX * sizeof(V));
  const uint32_t offU = (uint32_t)((size_t)(b - bw) * T * NU * sizeof(V));

  FgOut<V> out{V(0), V(0), 0, 0, false};
  V alpha_r = V(ls.alpha0);  // α of this round's first candidate
  V alpha = alpha_r;
  for (int j = 0; j < sub; ++j) alpha *= V(ls.shrink);
  int r = 0;
  bool store = sub == 0, rerun = false;
  struct Pass {
    V cost, du2;
    bool bad;
  };
  // one rollout at α (:64-76)
  auto pass = [&](auto robust) -> Pass {
    constexpr bool ROBUST = decltype(robust)::value;
    const uint32_t sx = store ? offX : 0x80000000u, su = store ? offU : 0x80000000u;
    V xb[4];
    {
      const V4 xv = *reinterpret_cast<const V4*>(xb0);  // x̄₁ = x₁ (:65)
      xb[0] = xv.x; xb[1] = xv.y; xb[2] = xv.z; xb[3] = xv.w;
    }
    Pass p{V(0), V(0), false};
    [[maybe_unused]] typename FgCarry<Model>::T cy{};
    if constexpr (!ROBUST) cy = fg_carry_init(m, xb);
    auto step = [&](int t, const StepIn& in) {
      // δx = x̄ₖ − xₖ (:72); ūₖ = uₖ + α δuₖ + Kₖ δx (:73)
      V dx[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) dx[i] = xb[i] - in.x[i];
      V ubar[NU];
#pragma unroll
      for (int a = 0; a < NU; ++a) {
        V kdx = V(0);
#pragma unroll
        for (int i = 0; i < 4; ++i) kdx = fma(in.K[a * 4 + i], dx[i], kdx);
        ubar[a] = fma(alpha, in.d[a], in.u[a]) + kdx;
      }
      p.cost += m.stage_cost(xb, in.xt, xtw, ubar);  // ℓ(x̄ₖ − x_trajₖ, ūₖ) (:187-190)
      fg_store_x(rX, sx + (uint32_t)(t * NX * sizeof(V)), xb);
#pragma unroll
      for (int a = 0; a < NU; ++a) fg_store_1(rU, su + (uint32_t)((t * NU + a) * sizeof(V)), ubar[a]);
#pragma unroll
      for (int a = NU - 1; a >= 0; --a) {  // Σ(ū − u)² (:165, the convergence test)
        const V e = ubar[a] - in.u[a];
        p.du2 = fma(e, e, p.du2);
      }
      // x̄ₖ₊₁ = f(x̄ₖ, ūₖ) (:74)
      V xn[4];
      if constexpr (ROBUST) m.rk4_robust(xb, ubar, xn);
      else fg_rk4_fast(m, xb, ubar, xn, p.bad, cy);
#pragma unroll
      for (int i = 0; i < 4; ++i) xb[i] = xn[i];
    };
    // inputs of the next FG_PF steps in flight (HBM latency ≈ one RK4 step)
    StepIn ring[FG_PF];
#pragma unroll
    for (int k = 0; k < FG_PF; ++k) load(k, ring[k]);
    int t = 0;
    for (; t + FG_PF <= T; t += FG_PF) {
#pragma unroll
      for (int k = 0; k < FG_PF; ++k) {
        step(t + k, ring[k]);
        load(t + k + FG_PF, ring[k]);
      }
    }
#pragma unroll
    for (int k = 0; k < FG_PF - 1; ++k)
      if (t + k < T) step(t + k, ring[k]);
    fg_store_x(rX, sx + (uint32_t)(T * NX * sizeof(V)), xb);
    p.cost += m.final_cost(xb);  // ℓ_f(x̄_N) on the raw state (:192)
    return p;
  };
  while (true) {
    Pass p = pass(FgPath<Model::HAS_FAST ? false : true>{});
    if constexpr (Model::HAS_FAST)
      if (p.bad) p = pass(FgPath<true>{});  // an argument out of rk4_fast's ranges: redo
    const V cost = p.cost, du2 = p.du2;
    if (rerun) break;  // the accepted candidate's rollout, now stored
    const int k = r * L + sub;  // 0-based trial index of this lane's candidate
    const bool acc = k < ls.max_trials && prev_cost - cost > V(0);  // NaN compares false
    constexpr uint64_t gmask = L >= 64 ? ~0ull : (1ull << L) - 1;
    const unsigned am = (unsigned)((__ballot(acc) >> gbase) & gmask);
    if (am) {
      const int first = __builtin_ctz(am);
      if (sub != first) break;
      out.trials = k + 1;
      out.accepted = 1;
      out.cost = cost;
      out.du2 = du2;
      out.owner = true;
      if (store) break;
      store = rerun = true;  // roll out once more, storing
      continue;
    }
    if ((r + 1) * L >= ls.max_trials) {  // exhausted (the reference would loop forever)
      if (k == ls.max_trials - 1) {
        out.trials = k + 1;
        out.cost = cost;
        out.du2 = du2;
        out.owner = true;
        if (store_exhausted && !store) {  // the last trial's rollout, stored
          store = rerun = true;
          continue;
        }
      }
      break;
    }
    ++r;
#pragma unroll
    for (int j = 0; j < L; ++j) alpha_r *= V(ls.shrink);
    alpha = alpha_r;
    for (int j = 0; j < sub; ++j) alpha *= V(ls.shrink);
  }
  return out;
}

// line-search candidates per trajectory: 4 up to B = 65536, one lane per trajectory past
// it (the candidates' extra waves are free at these batches); and
// in a fit past its first iteration (`wide`: prev_cost is finite, the search may be long)
// 32 up to B = 2048 — the lanes one wave per SIMD holds: a search capped at 64 trials then
// takes 2 rounds, not 16. Elsewhere 4: a search that accepts in its first round costs 7-30 %
// more on 32 lanes a trajectory (the whole chip's lanes busy), and a standalone forward
// cannot tell its prev_cost from +Inf without reading it back.
// ILQR_FG_LANES = 1/4/32 forces a width (measurement).
inline int fg_lanes(int B, bool wide = false) {
  const bool cold = !wide;
  static const int forced = [] {
    const char* e = std::getenv("ILQR_FG_LANES");
    const int v = e ? std::atoi(e) : 0;
    return v == 1 || v == 4 || v == 32 ? v : 0;
  }();
  if (forced) return forced;
  if (!cold && B <= 2048) return 32;
  return B <= 65536 ? 4 : 1;
}

}  // namespace
}  // namespace ilqr
